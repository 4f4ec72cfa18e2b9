#!/bin/bash
# A/B of the runtime-coefficient kernel in per-block launches (the repairs): the GPU tests of the
# rt paths first, then NFEC_RT_GPB = 1, 2, 4 (waves per item group) over the RS8 sweep (with
# NFEC_RT_DEC=1: the one-pass repair for the fixed shapes too) and the MDP repair, and the MDP
# snippet solve (NFEC_MDP_RT=0).  Diagnostic library for the A/B; output under gpurun_out/.
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
mkdir -p $O
cd $R
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread \
    tests/test_gpu_rt.py tests/test_gpu_random.py tests/test_gpu_parity.py > $O/t.log 2>&1
export NFEC_LIBRARY=$R/norm_amd/_lib/libnfec_diag.so
for g in ${GLIST:-1 2 4}; do
    NFEC_RT_DEC=1 NFEC_RT_GPB=$g timeout -k 10 300 python3 tools/bench_extra.py --workload rs8sweep > $O/gab_sweep_g$g.jsonl 2>> $O/gab.err
    NFEC_RT_GPB=$g timeout -k 10 200 python3 tools/bench_extra.py --workload mdp > $O/gab_mdp_g$g.json 2>> $O/gab.err
done
NFEC_MDP_RT=0 timeout -k 10 200 python3 tools/bench_extra.py --workload mdp > $O/gab_mdp_solve.json 2>> $O/gab.err
