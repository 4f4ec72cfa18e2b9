#!/bin/bash
# One PMC pass of SQ issue/wait counters over a short bench run (per-kernel rows).
# Usage: TAG=x [ENV settings exported] tools/pmc_sq.sh ; output gpurun_out/sq_$TAG/
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=${TAG:-sq}
OUT=gpurun_out/sq_$TAG
mkdir -p $OUT
export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_ACTIVE_INST_ANY \
  --output-format csv -d $OUT -o pmc -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --host-steps 0 > $OUT/run.log 2>&1 || { echo "pmc failed"; tail -5 $OUT/run.log; exit 1; }
python3 - "$OUT" <<'PY'
import csv, glob, sys, collections
f = glob.glob(sys.argv[1] + "/**/*counter_collection.csv", recursive=True)[0]
agg = collections.defaultdict(lambda: collections.defaultdict(float))
n = collections.Counter()
for r in csv.DictReader(open(f)):
    k = r["Kernel_Name"][:60]
    agg[k][r["Counter_Name"]] += float(r["Counter_Value"])
    n[(k, r["Counter_Name"])] += 1
for k, d in agg.items():
    if "rs8" not in k and "solve" not in k:
        continue
    wc = d.get("SQ_WAVE_CYCLES", 1)
    print(k, {c: round(v / max(1, n[(k, c)]) * 1.0, 0) for c, v in d.items()},
          "wait_any=%.2f wait_inst=%.2f active=%.2f" % (d.get("SQ_WAIT_ANY", 0) / wc, d.get("SQ_WAIT_INST_ANY", 0) / wc,
                                                       d.get("SQ_ACTIVE_INST_ANY", 0) / wc))
PY
