#!/bin/bash
# Round-3 GPU session: -m gpu suite, smoke, bench, rocprofv3 kernel summary.  Each GPU step runs
# under its own time limit and a failure ends the script (no retries).
#   TAG=a bash tools/gpu_r03.sh            everything
#   TAG=b bash tools/gpu_r03.sh tests bench  a subset (tests smoke bench prof percall, or tools/<x>.py)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
TAG=${TAG:-a}
STEPS=${*:-tests smoke bench prof}
export TMPDIR=/tmp
for step in $STEPS; do
  case $step in
    tests)
      timeout -k 10 ${PYTEST_TIMEOUT:-600} python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
          -p no:cacheprovider ${PYTEST_K:+-k "$PYTEST_K"} > gpurun_out/pytest_$TAG.log 2>&1
      rc=$?; tail -6 gpurun_out/pytest_$TAG.log
      [ $rc -eq 0 ] || { echo "pytest rc=$rc"; exit 2; } ;;
    smoke)
      timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$TAG.log 2>&1 \
          || { echo smoke failed; tail -20 gpurun_out/smoke_$TAG.log; exit 3; }
      tail -1 gpurun_out/smoke_$TAG.log ;;
    bench)
      timeout -k 10 600 python3 bench.py ${BENCH_ARGS:-} > gpurun_out/bench_$TAG.log 2>&1 \
          || { echo bench failed; tail -20 gpurun_out/bench_$TAG.log; exit 4; }
      tail -1 gpurun_out/bench_$TAG.log ;;
    prof)
      timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$TAG -o run --output-format csv \
          -- python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline --host-steps 0 > gpurun_out/prof_$TAG.log 2>&1 \
          || { echo rocprof failed; tail -20 gpurun_out/prof_$TAG.log; exit 5; }
      find gpurun_out/prof_$TAG -name '*kernel_stats.csv' | head -1 | xargs -r head -8 ;;
    percall)
      : > gpurun_out/percall_$TAG.jsonl
      for shape in "rs8 64 32 1408 16 2000" "rs8 64 32 1400 16 2000" "rs8 64 16 1408 8 2000" "rs8 16 4 1408 4 2000" \
                   "rs16 400 100 1400 50 200" "rs16 400 20 1400 10 500" "mdp 64 32 1408 16 500" \
                   "rs8 128 127 1408 100 200" "mdp 128 127 1408 100 200" "rs8 128 127 8192 100 50" \
                   "mdp 128 127 8192 100 50" "rs8 200 55 1408 55 200"; do
        timeout -k 10 120 tools/percall/_build/percall $shape >> gpurun_out/percall_$TAG.jsonl \
            2>> gpurun_out/percall_$TAG.err || { echo "percall $shape failed"; tail -5 gpurun_out/percall_$TAG.err; exit 7; }
      done
      cat gpurun_out/percall_$TAG.jsonl ;;
    *)
      # any other word: a python script under tools/ with its args in ARGS_<word>
      var="ARGS_$step"
      timeout -k 10 ${TOOL_TIMEOUT:-600} python3 -u tools/$step.py ${!var} > gpurun_out/${step}_$TAG.log 2>&1 \
          || { echo "$step failed"; tail -20 gpurun_out/${step}_$TAG.log; exit 6; }
      tail -3 gpurun_out/${step}_$TAG.log ;;
  esac
done
