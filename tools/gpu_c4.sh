#!/bin/bash
# C4 (RS16 k=4096 m=256 vec=1400, 4,096 blocks): bench line with the op roofline, then a kernel trace.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 300 python3 tools/bench_extra.py --workload c4 ${C4_ARGS:-} > gpurun_out/c4_${TAG:-x}.json 2>&1 || { tail -5 gpurun_out/c4_${TAG:-x}.json; exit 5; }
tail -1 gpurun_out/c4_${TAG:-x}.json
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_c4_${TAG:-x} -o run --output-format csv -- python3 tools/bench_extra.py --workload c4 --steps 2 --warmup 1 > gpurun_out/prof_c4_${TAG:-x}.log 2>&1 || { tail -5 gpurun_out/prof_c4_${TAG:-x}.log; exit 7; }
find gpurun_out/prof_c4_${TAG:-x} -name '*kernel_stats.csv' | head -1 | xargs -r head -6
