#!/bin/bash
# End-of-round evidence with the final build: PMC traffic of the bench kernels, kernel-trace
# summaries of the secondary workloads, the C5 one-GPU share.  Each GPU step time-limited.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
TAG=${TAG:-r02h} bash tools/pmc.sh || exit 1
WORKLOADS="rs16 mdp c4" bash tools/prof_extra.sh || exit 2
timeout -k 10 400 python3 tools/bench_c5.py > gpurun_out/c5_final.json 2>&1 || { tail -5 gpurun_out/c5_final.json; exit 3; }
tail -1 gpurun_out/c5_final.json
