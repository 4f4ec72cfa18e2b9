#!/bin/bash
# Tower-field RS16 kernel on the GPU (round 3): parity tests with it on, then RS16 (400,100)
# and C4 timings with it off / on, then the diagnostic probes on 1,024 C4 blocks.
#   bash tools/tw_r03.sh   -> gpurun_out/tw_*.{log,json}
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
NFEC_RS16_TW=1 timeout -k 10 400 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_tmvp.py -m gpu -x -q \
    --timeout 120 --timeout-method thread -p no:cacheprovider -k "16 or tmvp or toeplitz or RS16 or kind" \
    > gpurun_out/tw_pytest.log 2>&1 || { tail -30 gpurun_out/tw_pytest.log; exit 1; }
tail -2 gpurun_out/tw_pytest.log
for tw in 0 1; do
  NFEC_RS16_TW=$tw timeout -k 10 200 python3 tools/bench_extra.py --workload rs16 --steps 3 > gpurun_out/tw_rs16_$tw.json 2>&1 || exit 1
  NFEC_RS16_TW=$tw timeout -k 10 300 python3 tools/bench_extra.py --workload c4 --steps 2 > gpurun_out/tw_c4_$tw.json 2>&1 || exit 1
  tail -1 gpurun_out/tw_rs16_$tw.json; tail -1 gpurun_out/tw_c4_$tw.json
done
[ -f norm_amd/_lib/libnfec_diag.so ] || exit 0
for v in 0 1 2 3; do
  NFEC_LIBRARY=$PWD/norm_amd/_lib/libnfec_diag.so NFEC_RS16_TW=1 NFEC_TW_VARIANT=$v timeout -k 10 200 \
      python3 tools/bench_extra.py --workload c4 --blocks 1024 --steps 2 > gpurun_out/tw_probe_$v.json 2>&1 || exit 1
  echo "variant $v: $(tail -1 gpurun_out/tw_probe_$v.json | cut -c1-300)"
done
