#!/bin/bash
# A/B the shared-table builder variants (NFEC_T3_VARIANT) on C4 and on RS16(400,100) encode.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for v in ${VARIANTS:-0 1 2 3}; do
  for w in c4 rs16; do
    NFEC_T3_VARIANT=$v timeout -k 10 300 python3 tools/bench_extra.py --workload $w --erasures 0 > gpurun_out/t3_${v}_${w}.json 2>&1 || { tail -5 gpurun_out/t3_${v}_${w}.json; exit 1; }
    python3 -c 'import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], sys.argv[3], d["encode_ms"])' gpurun_out/t3_${v}_${w}.json $v $w
  done
done
