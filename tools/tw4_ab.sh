#!/bin/bash
# Tower kernel (shared columns, round 3) on the GPU: RS16 parity tests, RS16 (400,100) and C4
# timings, then the diagnostic probes on 1,024 C4 blocks when the diagnostic library is built.
#   bash tools/tw4_ab.sh   -> gpurun_out/tw4_*.{log,json}
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_rs16_kernels.py tests/test_gpu_tmvp.py tests/test_c4_c5.py tests/test_gpu_parity.py -m gpu -x -q \
    --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/tw4_pytest.log 2>&1 || { tail -30 gpurun_out/tw4_pytest.log; exit 1; }
tail -2 gpurun_out/tw4_pytest.log
timeout -k 10 200 python3 tools/bench_extra.py --workload rs16 --steps 3 > gpurun_out/tw4_rs16.json 2>&1 || exit 1
timeout -k 10 300 python3 tools/bench_extra.py --workload c4 --steps 2 > gpurun_out/tw4_c4.json 2>&1 || exit 1
tail -1 gpurun_out/tw4_rs16.json | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('rs16', d['encode_ms'], d['decode_ms'])"
tail -1 gpurun_out/tw4_c4.json | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('c4', d['encode_ms'])"
[ -f norm_amd/_lib/libnfec_diag.so ] || exit 0
for v in ${TW_PROBES:-0 1 2 3}; do
  NFEC_LIBRARY=$PWD/norm_amd/_lib/libnfec_diag.so NFEC_TW_VARIANT=$v timeout -k 10 200 \
      python3 tools/bench_extra.py --workload c4 --blocks 1024 --steps 2 > gpurun_out/tw4_probe_$v.json 2>&1 || exit 1
  echo "variant $v: $(tail -1 gpurun_out/tw4_probe_$v.json | python3 -c "import json,sys; print(json.loads(sys.stdin.read())['encode_ms'])")"
done
