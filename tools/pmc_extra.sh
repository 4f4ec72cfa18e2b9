#!/bin/bash
# SQ counters of a secondary workload (tools/bench_extra.py), one counter group per rocprofv3
# pass; per-dispatch averages of the kernels matching KERNEL on stdout.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
W=${WORKLOAD:-c4}
OUT=gpurun_out/pmcx_$W
mkdir -p $OUT
i=0
for grp in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_ACTIVE_INST_ANY" \
           "SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_INSTS_SALU SQ_INSTS_SMEM SQ_ACTIVE_INST_SCA SQ_INSTS_VMEM_RD" \
           "GRBM_GUI_ACTIVE GRBM_COUNT"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $grp --output-format csv -d $OUT/p$i -o pmc -- python3 tools/bench_extra.py --workload $W ${EXTRA_ARGS:-} > $OUT/p$i.log 2>&1 || { echo "pass $i failed"; tail -5 $OUT/p$i.log; exit 1; }
done
python3 - "$OUT" "${KERNEL:-gf16_t3}" <<'PY'
import csv, glob, sys, collections
agg = collections.defaultdict(float); disp = collections.defaultdict(set)
for f in glob.glob(sys.argv[1] + "/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if sys.argv[2] not in r["Kernel_Name"]:
            continue
        agg[r["Counter_Name"]] += float(r["Counter_Value"])
        disp[r["Counter_Name"]].add(r.get("Dispatch_Id", r.get("Correlation_Id", "")))
per = {c: v / max(1, len(disp[c])) for c, v in agg.items()}
print({c: "%.4g" % v for c, v in sorted(per.items())})
wc = per.get("SQ_WAVE_CYCLES", 1)
print("wait_any/wave_cycles=%.3f wait_inst_any=%.3f active_any=%.3f wait_inst_lds=%.3f" % (
    per.get("SQ_WAIT_ANY", 0) / wc, per.get("SQ_WAIT_INST_ANY", 0) / wc, per.get("SQ_ACTIVE_INST_ANY", 0) / wc,
    per.get("SQ_WAIT_INST_LDS", 0) / wc))
PY
