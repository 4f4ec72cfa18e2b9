#!/bin/bash
# A/B the kernel variants in one GPU session: prints value + per-kernel ms for each setting.
# VARIANTS: space-separated settings; a setting is comma-separated VAR=VALUE pairs.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for v in ${VARIANTS:-"NFEC_BS_VARIANT=0"}; do
  log=gpurun_out/ab_$(echo "$v" | tr '=,' '__').log
  env ${v//,/ } timeout -k 10 300 python3 bench.py --no-cpu-baseline --host-steps 0 --verify ${BENCH_ARGS:-} > "$log" 2>&1 || { echo "$v failed"; tail -5 "$log"; exit 1; }
  python3 -c 'import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], d["value"], d["kernels_ms"], d["roofline"]["frac"], "verified=%s" % d.get("verified"))' "$log" "$v"
done
