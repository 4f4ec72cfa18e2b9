#!/bin/bash
# A/B of diagnostic-library switches on the bench workload: for each entry of VARIANTS
# ("NAME=VALUE[,NAME=VALUE]" or "base"), one bench.py run with the diagnostic library loaded;
# prints encode / decode kernel ms.  Each run under its own time limit; a failure ends the script.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export NFEC_LIBRARY=$PWD/norm_amd/_lib/libnfec_diag.so
for rep in ${REPS:-1 2}; do
for v in ${VARIANTS:-base}; do
  envs=""
  [ "$v" != "base" ] && envs=$(echo "$v" | tr ',' ' ')
  env $envs timeout -k 10 180 python3 bench.py --steps ${STEPS:-20} --warmup 3 --no-cpu-baseline --host-steps 0 ${BENCH_ARGS:-} \
      > gpurun_out/ab_${TAG:-x}_${rep}_$v.log 2>&1 || { echo "variant $v failed"; tail -5 gpurun_out/ab_${TAG:-x}_${rep}_$v.log; exit 1; }
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], d['value'], d['kernels_ms'])" \
      gpurun_out/ab_${TAG:-x}_${rep}_$v.log "$v"
done
done
