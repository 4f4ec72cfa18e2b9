#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -p no:cacheprovider \
    tests/test_gpu_parity.py tests/test_gpu_tmvp.py -m gpu -k "MDP or mdp or 3- or stream_copy" > gpurun_out/mdp_tests.log 2>&1
rc=$?; tail -2 gpurun_out/mdp_tests.log; [ $rc -ne 0 ] && exit $rc
for i in 1 2; do
timeout -k 10 300 python3 tools/bench_extra.py --workload mdp > gpurun_out/mdp_bench.json 2>&1 || { tail -5 gpurun_out/mdp_bench.json; exit 5; }
tail -1 gpurun_out/mdp_bench.json
done
