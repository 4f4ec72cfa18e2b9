#!/bin/bash
# Round check plus A/B of pending variants in one session (boxes are scarce).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=${TAG:-r02g} bash tools/gpu_check.sh || exit $?
VARIANTS="${AB_VARIANTS:-NFEC_FDEC_LANEMAJOR=0 NFEC_FDEC_LANEMAJOR=2 NFEC_FDEC_LANEMAJOR=0 NFEC_FDEC_LANEMAJOR=2}" timeout -k 10 600 bash tools/ab_bench.sh || exit 1
NFEC_FDEC_LANEMAJOR=2 timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -p no:cacheprovider \
    tests/test_gpu_parity.py -m gpu -k "fused or unfused or decode" > gpurun_out/lm2_tests.log 2>&1
rc=$?; tail -2 gpurun_out/lm2_tests.log; exit $rc
