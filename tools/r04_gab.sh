#!/bin/bash
# A/B of the runtime-coefficient kernel's waves per item group in per-block launches (the
# repairs): NFEC_RT_GPB = 1, 2, 4 over the RS8 sweep (with NFEC_RT_DEC=1: the one-pass repair for
# the fixed shapes too) and the MDP repair.  Diagnostic library; output under gpurun_out/.
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
mkdir -p $O
cd $R
export NFEC_LIBRARY=$R/norm_amd/_lib/libnfec_diag.so
for g in 1 2 4; do
    NFEC_RT_DEC=1 NFEC_RT_GPB=$g timeout -k 10 300 python3 tools/bench_extra.py --workload rs8sweep > $O/gab_sweep_g$g.jsonl 2>> $O/gab.err
    NFEC_RT_GPB=$g timeout -k 10 200 python3 tools/bench_extra.py --workload mdp > $O/gab_mdp_g$g.json 2>> $O/gab.err
done
