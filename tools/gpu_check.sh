#!/bin/bash
# One GPU session: parity tests, smoke, bench, rocprofv3 kernel trace.  Every GPU step has
# its own time limit; a crash/timeout (exit >= 2 for pytest, != 0 otherwise) ends the script.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
TAG=${TAG:-r01}
timeout -k 10 ${PYTEST_TIMEOUT:-900} python3 -m pytest tests -m gpu -q -p no:cacheprovider ${PYTEST_ARGS:-} > gpurun_out/pytest_gpu_$TAG.log 2>&1
rc=$?
tail -5 gpurun_out/pytest_gpu_$TAG.log
if [ $rc -ge 2 ]; then echo "pytest crashed/timed out rc=$rc"; exit $rc; fi
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$TAG.log 2>&1 || { echo smoke failed; cat gpurun_out/smoke_$TAG.log | tail -20; exit 3; }
tail -1 gpurun_out/smoke_$TAG.log
timeout -k 10 600 python3 bench.py ${BENCH_ARGS:-} > gpurun_out/bench_$TAG.log 2>&1 || { echo bench failed; tail -20 gpurun_out/bench_$TAG.log; exit 4; }
tail -1 gpurun_out/bench_$TAG.log
if [ -n "${PROFILE:-1}" ]; then
  export TMPDIR=/tmp
  timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$TAG -o run --output-format csv -- python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline --host-steps 0 > gpurun_out/prof_$TAG.log 2>&1 || { echo rocprof failed; tail -20 gpurun_out/prof_$TAG.log; exit 5; }
  find gpurun_out/prof_$TAG -name '*kernel_stats.csv' | head -1 | xargs -r head -20
fi
exit $rc
