#!/bin/bash
# Builder timing probe (NFEC_T3_VARIANT=1): per-phase shader clocks of workgroup 0.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export NFEC_T3_VARIANT=1
timeout -k 10 200 python3 tools/bench_extra.py --workload c4 --steps 1 --warmup 0 > gpurun_out/t3t_c4.log 2>&1 || exit 1
grep "t3 builder" gpurun_out/t3t_c4.log | sort | uniq -c | head -8
for m in 20 44; do
  NFEC_RS16_TMVP=0 timeout -k 10 200 python3 tools/bench_extra.py --workload c4 --k 4096 --m $m --blocks 1024 --erasures 0 --steps 1 --warmup 0 > gpurun_out/t3t_$m.log 2>&1 || exit 2
  grep "t3 builder" gpurun_out/t3t_$m.log | sort | uniq -c | head -4
  tail -1 gpurun_out/t3t_$m.log | cut -c1-200
done
