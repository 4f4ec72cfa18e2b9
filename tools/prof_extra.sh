#!/bin/bash
# rocprofv3 kernel-trace summaries of the secondary workloads (tools/bench_extra.py), one pass
# per workload in WORKLOADS; summaries under gpurun_out/profx_<workload>/.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
for w in ${WORKLOADS:-rs16 mdp}; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/profx_$w -o run --output-format csv -- \
      python3 tools/bench_extra.py --workload $w --steps 2 --warmup 1 > gpurun_out/profx_$w.log 2>&1 || { echo "$w failed"; tail -5 gpurun_out/profx_$w.log; exit 1; }
  tail -1 gpurun_out/profx_$w.log
  find gpurun_out/profx_$w -name '*kernel_stats.csv' | head -1 | xargs -r head -12 | cut -c1-160
done
