#!/bin/bash
# A/B of diag_knob switches on one box: the knob library (tools/ab_build.sh with
# AB_FLAGS=-DNFEC_KNOBS) under each environment setting of AB_ENVS (';'-separated, e.g.
# "NFEC_TMVP_SH=0;NFEC_TMVP_SH=1"), alternating AB_REPS times (default 2), each run of
# tools/bench_extra.py $AB_ARGS under a rocprofv3 kernel trace; one JSON line per run plus its
# kernel stats under gpurun_out/$TAG/.
#   TAG=r06e AB_LIB=norm_amd/_lib/libnfec_knobs.so AB_ENVS="A=0;A=1" AB_ARGS="--workload rs16" bash tools/ab_env.sh
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$(pwd)
O=$R/gpurun_out/${TAG:-ab_env}
mkdir -p "$O"
export TMPDIR=/tmp
IFS=';' read -ra ENVS <<< "$AB_ENVS"
: > "$O/ab_env.jsonl"
for i in $(seq 1 "${AB_REPS:-2}"); do
    for j in "${!ENVS[@]}"; do
        e=${ENVS[j]}
        n="env${j}_r$i"
        (cd /tmp && env $e NFEC_LIBRARY=$R/$AB_LIB timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv \
            -d "$O/prof_$n" -o "$n" -- python3 "$R/tools/bench_extra.py" $AB_ARGS) > "$O/$n.json" 2> "$O/$n.err" \
            || { echo "ab_env: $e failed"; tail -5 "$O/$n.err"; exit 1; }
        python3 - "$O/$n.json" "$e" "$O/prof_$n" "$O/ab_env.jsonl" <<'PY'
import csv, glob, json, sys
d = json.load(open(sys.argv[1]))
st = glob.glob(sys.argv[3] + "/**/*_kernel_stats.csv", recursive=True)
ks = {}
if st:
    for r in csv.DictReader(open(st[0])):
        ks[r["Name"].replace("nfec::(anonymous namespace)::", "").replace("void ", "").split("(")[0]] = round(float(r["AverageNs"]) / 1e3, 1)
d = {"env": sys.argv[2], "encode_ms": d.get("encode_ms"), "decode_ms": d.get("decode_ms"), "verified": d.get("verified"),
     "kernels_us": {k: v for k, v in ks.items() if "tmvp" in k or "gf16" in k or "rs8" in k}}
open(sys.argv[4], "a").write(json.dumps(d) + "\n")
print(json.dumps(d))
PY
    done
done
