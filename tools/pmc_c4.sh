#!/bin/bash
# PMC passes of the C4 RS16 encode (tools/bench_extra.py --workload c4): the tower-field product
# kernel's instruction mix (VALU / SALU / branch / LDS / SMEM), wave states, cycles and HBM bytes,
# one counter group per rocprofv3 run (tools/pmc_r03.sh).  The summary gets the workload's shape
# under "_workload" so bench_extra.py's op roofline can find it (profiles/r0N/pmc_tw_c4_summary.json).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=${TAG:-c4}
export PMC_SCRIPT=tools/bench_extra.py
export PMC_ARGS="--workload c4 --steps 1 --warmup 1"
export PMC_GROUPS="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_BRANCH SQ_INSTS_LDS SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR;SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA;GRBM_GUI_ACTIVE GRBM_COUNT;FETCH_SIZE;WRITE_SIZE"
TAG=$TAG bash tools/pmc_r03.sh > /dev/null || exit 1
python3 - gpurun_out/pmc_$TAG/summary.json <<'PY'
import json, sys
p = sys.argv[1]
d = json.load(open(p))
d["_workload"] = {"workload": "c4", "k": 4096, "m": 256, "vec": 1400, "blocks": 4096, "encodes": 2,
                  "counters": "rocprofv3 --pmc, one group per pass (tools/pmc_c4.sh); per-launch averages"}
json.dump(d, open(p, "w"), indent=1, sort_keys=True)
print(json.dumps({k: {c: v.get(c) for c in ("SQ_INSTS_VALU", "SQ_INSTS_SALU", "SQ_INSTS_BRANCH", "GRBM_GUI_ACTIVE")}
                  for k, v in d.items() if "gf16" in k or "tmvp" in k}, indent=1))
PY
