#!/bin/bash
# rt kernel with and without HBM reads (NFEC_RT_PROBE=1: every column reads its block's slot 0,
# results wrong): the (64,32) one-pass repair (NFEC_RT_DEC=1) and the (128,32) encode + repair.
# Diagnostic library; lines under gpurun_out/probe_*.json.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export NFEC_LIBRARY=$(pwd)/norm_amd/_lib/libnfec_diag.so
for p in ${PLIST:-0 1}; do
    NFEC_RT_DEC=1 NFEC_RT_PROBE=$p timeout -k 10 120 python3 tools/bench_extra.py --workload rs8 --k 64 --m 32 --erasures 16 > gpurun_out/probe_6432_$p.json 2> gpurun_out/probe_6432_$p.err
    NFEC_RT_PROBE=$p timeout -k 10 120 python3 tools/bench_extra.py --workload rs8 --k 128 --m 32 --erasures 16 > gpurun_out/probe_12832_$p.json 2> gpurun_out/probe_12832_$p.err
done
exit 0
