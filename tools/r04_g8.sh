set -e
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_rt.py tests/test_gpu_random.py > gpurun_out/g8_t.log 2>&1
timeout -k 10 300 python3 tools/bench_extra.py --workload rs8sweep > gpurun_out/g8_on.jsonl 2>/dev/null
NFEC_LIBRARY=$GRAFT_REPO_ROOT/norm_amd/_lib/libnfec_diag.so NFEC_RT_G8=0 timeout -k 10 300 python3 tools/bench_extra.py --workload rs8sweep > gpurun_out/g8_off.jsonl 2>/dev/null
for km in "100 100" "127 128" "64 48"; do set -- $km; timeout -k 10 120 python3 tools/bench_extra.py --workload rs8 --k $1 --m $2 --erasures 16 --blocks 16384 >> gpurun_out/g8_more_on.jsonl 2>/dev/null; NFEC_LIBRARY=$GRAFT_REPO_ROOT/norm_amd/_lib/libnfec_diag.so NFEC_RT_G8=0 timeout -k 10 120 python3 tools/bench_extra.py --workload rs8 --k $1 --m $2 --erasures 16 --blocks 16384 >> gpurun_out/g8_more_off.jsonl 2>/dev/null; done
