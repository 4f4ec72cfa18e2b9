#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
VARIANTS="0 4 5" bash tools/ab_t3.sh || exit 1
NFEC_T3_VARIANT=4 timeout -k 10 400 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider \
    tests/test_gpu_tmvp.py tests/test_c4_c5.py -m gpu > gpurun_out/t3v4_tests.log 2>&1
rc=$?; tail -2 gpurun_out/t3v4_tests.log; exit $rc
