#!/bin/bash
# RS8 (64, m) encode / 16-erasure repair for NORM's usual parity counts (m = 32, 16, 8; m = 8
# repairs 8 erasures), vec 1400 and 1408, 65,536 blocks.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for m in 32 16 8; do
  e=16; [ $m -lt 16 ] && e=$m
  for v in 1400 1408; do
    timeout -k 10 300 python3 tools/bench_extra.py --workload rs8 --m $m --erasures $e --vec $v > gpurun_out/rs8_${m}_${v}.json 2>&1 || { tail -5 gpurun_out/rs8_${m}_${v}.json; exit 1; }
    tail -1 gpurun_out/rs8_${m}_${v}.json
  done
done
