#!/bin/bash
# Round-4 evidence beside the headline bench: per-call latencies (tools/percall: the drop-in's
# host per-segment Encode, GPU Encode and Decode against the CPU reference restatement), the C4
# tower-kernel PMC passes (tools/pmc_c4.sh -> gpurun_out/pmc_c4/summary.json) and the C4 line
# with its op roofline.  Output under gpurun_out/.
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
mkdir -p $O
cd $R
if [ -z "$SKIP_PERCALL" ]; then
: > $O/percall.jsonl
for args in "rs8 64 32 1408 16 2000" "rs8 64 16 1408 8 2000" "rs8 16 4 1408 4 2000" "rs16 400 100 1400 50 200" "mdp 64 32 1408 16 500"; do
    timeout -k 10 120 tools/percall/_build/percall $args >> $O/percall.jsonl
done
fi
TAG=c4 timeout -k 10 600 bash tools/pmc_c4.sh > $O/pmc_c4.log 2>&1
timeout -k 10 300 python3 tools/bench_extra.py --workload c4 > $O/extra_c4.json 2> $O/extra_c4.err
