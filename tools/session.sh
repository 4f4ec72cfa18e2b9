#!/bin/bash
# The one GPU session script (round 5 on): each named task runs under its own time limit and the
# first failure ends the script (no retries).  Output under gpurun_out/$TAG/; the summaries that
# are judged get copied into profiles/r0N/ by hand afterwards.
#
#   TAG=r05a bash tools/session.sh suite bench rs16 ...
#
# tasks
#   suite      pytest -m gpu (the whole GPU suite; PYTEST_K narrows it with a -k expression)
#   bench      bench.py line, then rocprofv3 --kernel-trace --stats of bench.py --steps 10
#   rs16       RS16(400,100) 50-erasure repair per 16k blocks under rocprofv3 kernel traces:
#              source loss, uniform loss over all k + m segments, shortened batches (numData in
#              [k/2, k]), accumulate, and vec 1460 (vec % 8 != 0); one JSON line each
#   c4         C4 RS16(4096,256) encode line (with its op roofline) under a kernel trace
#   short      shortened batches (numData in {k, k-1} and in [k/2, k]) beside unshortened ones for
#              RS16(400,100), C4 and RS8(64,32)/(64,16), under kernel traces
#   pmc_rs16   PMC passes of the RS16(400,100) encode (tools/pmc_r03.sh; instruction mix, cycles,
#              HBM bytes) -> pmc_tw_rs16_summary.json, which bench_extra's op roofline reads
#   pmc_c4     PMC passes of C4 (tools/pmc_c4.sh)
#   pmc_bench  PMC passes of the headline workload (tools/pmc_r03.sh: HBM bytes for bench.py)
#   mdp        MDP(64,32) encode + 16-erasure repair line under a kernel trace
#   rs8sweep   RS8 shape sweep (tools/bench_extra.py --workload rs8sweep) under a kernel trace
#   c5         tools/bench_c5.py --steps 2 (the C5 mix's one-GPU share)
#   percall    tools/percall per-call latencies (needs tools/percall/_build/percall)
#   tmvp_levels RS16 encode with the Toeplitz split forced at 0..2 levels on four shapes
#   ab_mdp     MDP(64,32) encode + repair lines from the product library and each of AB_LIBS,
#              alternating on one box (AB_REPS rounds, default 3)
#   ab         A/B of the product library against AB_LIBS (other builds of the same sources, e.g.
#              tools/ab_build.sh with a generator option, loaded through NFEC_LIBRARY): the RS16 GPU
#              tests on each (AB_K: a -k expression, e.g. to skip the split-level expectations of a
#              build with another row count), then rs16 and c4 lines from all, alternating,
#              AB_REPS times (default 2)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$(pwd)
TAG=${TAG:-r05}
O=$R/gpurun_out/$TAG
mkdir -p "$O"
export TMPDIR=/tmp

die() { echo "session: $1 failed (rc $2)"; exit "$2"; }

# rocprofv3 kernel trace + stats of one python command: $1 = name, rest = script and arguments
prof() {
    local name=$1; shift
    (cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/prof_$name" -o "$name" -- \
        python3 "$@") > "$O/$name.json" 2> "$O/$name.err" || return $?
    local st
    st=$(find "$O/prof_$name" -name "${name}_kernel_stats.csv" -print -quit)
    [ -n "$st" ] && cp "$st" "$O/${name}_kernel_stats.csv"
    cat "$O/$name.json"
}

for task in "$@"; do
    case $task in
    suite)
        timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
            -p no:cacheprovider ${PYTEST_K:+-k "$PYTEST_K"} > "$O/pytest_gpu.log" 2>&1
        rc=$?
        tail -n 5 "$O/pytest_gpu.log"
        [ $rc -eq 0 ] || die suite $rc ;;
    bench)
        timeout -k 10 300 python3 bench.py > "$O/bench.json" 2> "$O/bench.err" || die bench $?
        cat "$O/bench.json"
        prof bench_k "$R/bench.py" --steps 10 --no-cpu-baseline --host-steps 0 > /dev/null || die bench_prof $? ;;
    rs16)
        X=$R/tools/bench_extra.py
        prof rs16_source "$X" --workload rs16 || die rs16_source $?
        prof rs16_uniform "$X" --workload rs16 --loss uniform || die rs16_uniform $?
        prof rs16_short "$X" --workload rs16 --shortened || die rs16_short $?
        prof rs16_short_uniform "$X" --workload rs16 --shortened --loss uniform || die rs16_short_uniform $?
        prof rs16_acc "$X" --workload rs16 --accumulate || die rs16_acc $?
        prof rs16_vec1460 "$X" --workload rs16 --vec 1460 || die rs16_vec1460 $?
        prof rs16_vec1460_uniform "$X" --workload rs16 --vec 1460 --loss uniform || die rs16_vec1460_uniform $? ;;
    c4)
        prof c4 "$R/tools/bench_extra.py" --workload c4 || die c4 $? ;;
    short)
        # shortened batches on the fast kernels (round 6): per shape the unshortened encode beside
        # numData in {k, k - 1} (RFC 5052 large / small blocks) and numData over [k/2, k]; the lines
        # carry encode_GiBps per source byte and the encode path that took the batches
        X=$R/tools/bench_extra.py
        prof short_rs16_full "$X" --workload rs16 --erasures 0 || die short $?
        prof short_rs16_rfc "$X" --workload rs16 --erasures 0 --shortened --nd-dist rfc || die short $?
        prof short_rs16_half "$X" --workload rs16 --shortened || die short $?
        prof short_rs16_rfc_dec "$X" --workload rs16 --shortened --nd-dist rfc --loss uniform || die short $?
        prof short_c4_full "$X" --workload c4 || die short $?
        prof short_c4_rfc "$X" --workload c4 --shortened --nd-dist rfc || die short $?
        prof short_rs8_full "$X" --workload rs8 || die short $?
        prof short_rs8_rfc "$X" --workload rs8 --shortened --nd-dist rfc || die short $?
        prof short_rs8_half "$X" --workload rs8 --shortened || die short $?
        prof short_rs8_16_full "$X" --workload rs8 --m 16 --erasures 8 || die short $?
        prof short_rs8_16_rfc "$X" --workload rs8 --m 16 --erasures 8 --shortened --nd-dist rfc || die short $? ;;
    pmc_rs16)
        # the encode alone (--erasures 0), so the tower kernel's counters are the encode's
        PMC_SCRIPT=tools/bench_extra.py PMC_ARGS="--workload rs16 --erasures 0 --steps 1 --warmup 1" \
        PMC_GROUPS="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_BRANCH SQ_INSTS_LDS SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR;SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA;GRBM_GUI_ACTIVE GRBM_COUNT;FETCH_SIZE;WRITE_SIZE" \
        TAG=${TAG}_rs16 timeout -k 10 900 bash tools/pmc_r03.sh > "$O/pmc_rs16.log" 2>&1 || die pmc_rs16 $?
        python3 - "$R/gpurun_out/pmc_${TAG}_rs16/summary.json" "$O/pmc_tw_rs16_summary.json" <<'PY' || die pmc_rs16 $?
import json, sys
d = json.load(open(sys.argv[1]))
d["_workload"] = {"workload": "rs16", "k": 400, "m": 100, "vec": 1400, "blocks": 16384, "encodes": 2,
                  "counters": "rocprofv3 --pmc, one group per pass (tools/session.sh pmc_rs16); encode only; per-launch averages"}
json.dump(d, open(sys.argv[2], "w"), indent=1, sort_keys=True)
PY
        ;;
    pmc_c4)
        TAG=${TAG}_c4 timeout -k 10 900 bash tools/pmc_c4.sh > "$O/pmc_c4.log" 2>&1 || die pmc_c4 $?
        cp "$R/gpurun_out/pmc_${TAG}_c4/summary.json" "$O/pmc_c4_summary.json" ;;
    pmc_bench)
        TAG=${TAG}_bench timeout -k 10 900 bash tools/pmc_r03.sh > "$O/pmc_bench.log" 2>&1 || die pmc_bench $?
        cp "$R/gpurun_out/pmc_${TAG}_bench/summary.json" "$O/pmc_bench_summary.json" ;;
    mdp)
        prof mdp "$R/tools/bench_extra.py" --workload mdp || die mdp $? ;;
    rs8sweep)
        prof rs8sweep "$R/tools/bench_extra.py" --workload rs8sweep || die rs8sweep $? ;;
    c5)
        timeout -k 10 600 python3 tools/bench_c5.py --steps 2 > "$O/c5.json" 2> "$O/c5.err" || die c5 $?
        cat "$O/c5.json" ;;
    percall)
        : > "$O/percall.jsonl"
        for args in "rs8 64 32 1408 16 2000" "rs8 64 16 1408 8 2000" "rs8 16 4 1408 4 2000" "rs16 400 100 1400 50 200" "mdp 64 32 1408 16 500"; do
            timeout -k 10 120 tools/percall/_build/percall $args >> "$O/percall.jsonl" || die percall $?
        done ;;
    tmvp_levels)
        # the Toeplitz split forced at 0 / 1 / 2 Karatsuba levels (NFEC_OPT_* 2 / 20 / 4) on
        # shapes where the level choice is close, encode only; one JSON line each
        : > "$O/tmvp_levels.jsonl"
        for shape in "128 32 51200" "256 64 25600" "512 128 12800" "4096 256 4096"; do
            set -- $shape
            for opt in 2 20 4; do
                timeout -k 10 300 python3 tools/bench_extra.py --workload rs16 --k $1 --m $2 --blocks $3 --erasures 0 \
                    --options $opt >> "$O/tmvp_levels.jsonl" || die tmvp_levels $?
            done
        done
        python3 -c "import json,sys; [print(d['k'], d['m'], d['toeplitz_levels'], d['encode_ms']) for d in map(json.loads, open(sys.argv[1]))]" "$O/tmvp_levels.jsonl" ;;
    ab)
        [ -n "$AB_LIBS" ] || die "ab (AB_LIBS unset)" 2
        for L in $AB_LIBS; do
            n=$(basename "$L" .so)
            NFEC_LIBRARY=$R/$L timeout -k 10 600 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread \
                -p no:cacheprovider tests/test_gpu_rs16_tw.py tests/test_gpu_rs16_kernels.py tests/test_gpu_tmvp.py \
                tests/test_c4_c5.py -m gpu ${AB_K:+-k "$AB_K"} > "$O/pytest_$n.log" 2>&1 || { tail -n 20 "$O/pytest_$n.log"; die ab_tests_$n 1; }
            echo "$n: $(tail -n 1 "$O/pytest_$n.log")"
        done
        for i in $(seq 1 "${AB_REPS:-2}"); do
            for w in rs16 c4; do
                timeout -k 10 300 python3 tools/bench_extra.py --workload $w > "$O/${w}_product_$i.json" || die ab $?
                for L in $AB_LIBS; do
                    n=$(basename "$L" .so)
                    NFEC_LIBRARY=$R/$L timeout -k 10 300 python3 tools/bench_extra.py --workload $w > "$O/${w}_${n}_$i.json" || die ab $?
                done
            done
        done
        for f in "$O"/rs16_*_[0-9].json "$O"/c4_*_[0-9].json; do
            python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[1].rsplit('/',1)[1], d.get('encode_ms'), d.get('decode_ms'))" "$f"
        done ;;
    ab_mdp)
        # MDP(64,32) encode + 16-erasure repair on the product library and each of AB_LIBS,
        # alternating on one box, AB_REPS times (default 3): one JSON line per run
        [ -n "$AB_LIBS" ] || die "ab_mdp (AB_LIBS unset)" 2
        : > "$O/ab_mdp.jsonl"
        for i in $(seq 1 "${AB_REPS:-3}"); do
            timeout -k 10 300 python3 tools/bench_extra.py --workload mdp --steps 10 | sed 's/^{/{"lib": "product", /' >> "$O/ab_mdp.jsonl" || die ab_mdp $?
            for L in $AB_LIBS; do
                n=$(basename "$L" .so)
                NFEC_LIBRARY=$R/$L timeout -k 10 300 python3 tools/bench_extra.py --workload mdp --steps 10 \
                    | sed "s/^{/{\"lib\": \"$n\", /" >> "$O/ab_mdp.jsonl" || die ab_mdp $?
            done
        done
        python3 -c "import json,sys; [print(d['lib'], d['encode_ms'], d['decode_ms'], d['verified']) for d in map(json.loads, open(sys.argv[1]))]" "$O/ab_mdp.jsonl" ;;
    *)
        echo "session: unknown task $task"; exit 2 ;;
    esac
done
