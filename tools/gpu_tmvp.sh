#!/bin/bash
# RS16 Toeplitz-split session: its parity tests, the RS16/C4 tests, then C4 with and without
# the split, and a kernel trace of the split.  Every GPU step under its own time limit.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 400 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider \
    tests/test_gpu_tmvp.py tests/test_c4_c5.py -m gpu > gpurun_out/tmvp_tests.log 2>&1
rc=$?; tail -3 gpurun_out/tmvp_tests.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 400 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -p no:cacheprovider \
    tests -m gpu > gpurun_out/tmvp_parity.log 2>&1
rc=$?; tail -2 gpurun_out/tmvp_parity.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python3 tools/bench_extra.py --workload c4 > gpurun_out/c4_tmvp.json 2>&1 || { tail -5 gpurun_out/c4_tmvp.json; exit 5; }
tail -1 gpurun_out/c4_tmvp.json
NFEC_RS16_TMVP=0 timeout -k 10 300 python3 tools/bench_extra.py --workload c4 > gpurun_out/c4_plain.json 2>&1 || { tail -5 gpurun_out/c4_plain.json; exit 6; }
tail -1 gpurun_out/c4_plain.json
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_c4 -o run --output-format csv -- python3 tools/bench_extra.py --workload c4 --steps 2 --warmup 1 > gpurun_out/prof_c4.log 2>&1 || { tail -5 gpurun_out/prof_c4.log; exit 7; }
find gpurun_out/prof_c4 -name '*kernel_stats.csv' | head -1 | xargs -r head -8
