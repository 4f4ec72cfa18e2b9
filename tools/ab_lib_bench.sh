#!/bin/bash
# A/B of whole library builds on the headline workload, on one box: bench.py (no CPU baseline,
# no host leg) under a rocprofv3 kernel trace with the product library and each of AB_LIBS
# (';'-separated paths, loaded through NFEC_LIBRARY), alternating AB_REPS times (default 2).
# One JSON line per run in gpurun_out/$TAG/ab_lib.jsonl: the line's value and the average
# duration of every nfec kernel.
#   TAG=r06x AB_LIBS="norm_amd/_lib/libnfec_old.so" bash tools/ab_lib_bench.sh
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$(pwd)
O=$R/gpurun_out/${TAG:-ab_lib}
mkdir -p "$O"
export TMPDIR=/tmp
IFS=';' read -ra LIBS <<< "product;$AB_LIBS"
: > "$O/ab_lib.jsonl"
for i in $(seq 1 "${AB_REPS:-2}"); do
    for j in "${!LIBS[@]}"; do
        lib=${LIBS[j]}
        n="lib${j}_r$i"
        envs=()
        [ "$lib" != product ] && envs=(NFEC_LIBRARY="$R/$lib")
        (cd /tmp && env "${envs[@]}" timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv \
            -d "$O/prof_$n" -o "$n" -- python3 "$R/bench.py" --no-cpu-baseline --host-steps 0 --no-verify) \
            > "$O/$n.json" 2> "$O/$n.err" || { echo "ab_lib: $lib failed"; tail -5 "$O/$n.err"; exit 1; }
        python3 - "$O/$n.json" "$lib" "$O/prof_$n" "$O/ab_lib.jsonl" <<'PY'
import csv, glob, json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
st = glob.glob(sys.argv[3] + "/**/*_kernel_stats.csv", recursive=True)
ks = {}
if st:
    for r in csv.DictReader(open(st[0])):
        if "nfec" in r["Name"]:
            ks[r["Name"].replace("nfec::(anonymous namespace)::", "").split("(")[0]] = round(float(r["AverageNs"]) / 1e3, 1)
out = {"lib": sys.argv[2], "value": d["value"], "kernels_ms": d["kernels_ms"], "kernels_us": ks}
open(sys.argv[4], "a").write(json.dumps(out) + "\n")
print(json.dumps(out))
PY
    done
done
