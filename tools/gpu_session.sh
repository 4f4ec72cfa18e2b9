#!/bin/bash
# One GPU session for A/B work: the -m gpu suite (PYTEST_K, a -k expression, narrows it), then tools/ab_bench.sh
# over VARIANTS.  Every GPU step has its own time limit; a crash/timeout ends the script.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
if [ -z "${SKIP_TESTS:-}" ]; then
  timeout -k 10 300 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
      -p no:cacheprovider ${PYTEST_K:+-k "$PYTEST_K"} > gpurun_out/pt_${TAG:-ab}.log 2>&1
  rc=$?
  tail -15 gpurun_out/pt_${TAG:-ab}.log
  if [ $rc -ge 2 ]; then echo "pytest rc=$rc"; exit $rc; fi
fi
if [ -n "${VARIANTS:-}" ]; then bash tools/ab_bench.sh; exit $?; fi
