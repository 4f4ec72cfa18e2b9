#!/bin/bash
# SQ issue/wait counters + GRBM_GUI_ACTIVE (effective clock = GUI_ACTIVE / 8 XCDs / kernel time)
# for each setting in VARIANTS (comma-separated VAR=VALUE pairs), one counter group per
# rocprofv3 pass.  Output: gpurun_out/pmcab_<setting>/, summary lines on stdout.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
for v in ${VARIANTS:-"NFEC_Q4_VARIANT=0"}; do
  OUT=gpurun_out/pmcab_$(echo "$v" | tr '=,' '__')
  mkdir -p $OUT
  i=0
  for grp in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_ACTIVE_INST_ANY" \
             "GRBM_GUI_ACTIVE GRBM_COUNT" "SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_VMEM"; do
    i=$((i+1))
    env ${v//,/ } timeout -s KILL 120 rocprofv3 --pmc $grp --output-format csv -d $OUT/p$i -o pmc -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --host-steps 0 > $OUT/p$i.log 2>&1 || { echo "$v pass $i failed"; tail -5 $OUT/p$i.log; exit 1; }
  done
  python3 - "$OUT" "$v" <<'PY'
import csv, glob, sys, collections
agg = collections.defaultdict(lambda: collections.defaultdict(float))
disp = collections.defaultdict(set)
for f in glob.glob(sys.argv[1] + "/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"]
        if "rs8" not in k:
            continue
        k = k.split("(")[0].split("::")[-1]
        agg[k][r["Counter_Name"]] += float(r["Counter_Value"])
        disp[(k, r["Counter_Name"])].add(r.get("Dispatch_Id", r.get("Correlation_Id", "")))
for k, d in agg.items():
    per = {c: v / max(1, len(disp[(k, c)])) for c, v in d.items()}
    wc = per.get("SQ_WAVE_CYCLES", 1)
    print(sys.argv[2], k, "per-dispatch:", {c: "%.4g" % v for c, v in sorted(per.items())},
          "wait_any=%.3f wait_inst=%.3f active=%.3f" % (per.get("SQ_WAIT_ANY", 0) / wc, per.get("SQ_WAIT_INST_ANY", 0) / wc,
                                                       per.get("SQ_ACTIVE_INST_ANY", 0) / wc))
PY
done
