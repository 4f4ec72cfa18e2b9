#!/bin/bash
# A/B the kernel variants in one GPU session: prints value + per-kernel ms for each setting.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for v in ${VARIANTS:-"NFEC_BS_VARIANT=0" "NFEC_BS_VARIANT=1"}; do
  env $v timeout -k 10 300 python3 bench.py --no-cpu-baseline ${BENCH_ARGS:-} > gpurun_out/ab_$(echo $v | tr '=' '_').log 2>&1 || { echo "$v failed"; tail -5 gpurun_out/ab_$(echo $v | tr '=' '_').log; exit 1; }
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], d['value'], d['kernels_ms'], d['roofline']['frac'])" gpurun_out/ab_$(echo $v | tr '=' '_').log "$v"
done
