#!/bin/bash
# Round-4 check of the runtime-coefficient paths: GPU tests, the RS8 shape sweep under rocprofv3
# (kernel trace), the (64,32) repair A/B (NFEC_RT_DEC=1: one-pass rt repair instead of the fused
# kernel) and the MDP repair A/B (NFEC_MDP_RT=0: the snippet solve); A/B switches are read by the
# diagnostic library only (make -C norm_amd diag).  Output under gpurun_out/.
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
mkdir -p $O
cd $R
timeout -k 10 500 python -u -m pytest -x -q --timeout 120 --timeout-method thread \
    tests/test_gpu_rt.py tests/test_gpu_random.py tests/test_gpu_parity.py tests/test_npc.py \
    tests/test_gpu_vectors.py > $O/t.log 2>&1
cd /tmp
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_sw2 -o sw -- \
    python3 $R/tools/bench_extra.py --workload rs8sweep > $O/sweep2.jsonl 2> $O/sweep.err
NFEC_LIBRARY=$R/norm_amd/_lib/libnfec_diag.so NFEC_RT_DEC=1 timeout -k 10 300 python3 $R/tools/bench_extra.py --workload rs8sweep > $O/sweep2_rtdec.jsonl 2>> $O/sweep.err
timeout -k 10 200 python3 $R/tools/bench_extra.py --workload mdp > $O/mdp.json 2>> $O/sweep.err
NFEC_LIBRARY=$R/norm_amd/_lib/libnfec_diag.so NFEC_MDP_RT=0 timeout -k 10 200 python3 $R/tools/bench_extra.py --workload mdp > $O/mdp_old.json 2>> $O/sweep.err
