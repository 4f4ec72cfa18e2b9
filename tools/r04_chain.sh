#!/bin/bash
# A/B of chained snippet calls in the runtime-coefficient kernel: the diagnostic library built
# with RT_CHAIN=1 (two rows per call/return) against the product library, on the rt GPU tests
# and the RS8 sweep (+ the one-pass (64,32) repair, NFEC_RT_DEC=1) and the MDP repair.
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
cd $R
D=$R/norm_amd/_lib/libnfec_diag.so
NFEC_LIBRARY=$D timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_rt.py > $O/chain_t.log 2>&1
timeout -k 10 300 python3 tools/bench_extra.py --workload rs8sweep > $O/chain_sweep_off.jsonl 2>/dev/null
NFEC_LIBRARY=$D timeout -k 10 300 python3 tools/bench_extra.py --workload rs8sweep > $O/chain_sweep_on.jsonl 2>/dev/null
NFEC_LIBRARY=$D NFEC_RT_DEC=1 timeout -k 10 300 python3 tools/bench_extra.py --workload rs8 --k 64 --m 32 --erasures 16 > $O/chain_6432_on.json 2>/dev/null
timeout -k 10 200 python3 tools/bench_extra.py --workload mdp > $O/chain_mdp_off.json 2>/dev/null
NFEC_LIBRARY=$D timeout -k 10 200 python3 tools/bench_extra.py --workload mdp > $O/chain_mdp_on.json 2>/dev/null
