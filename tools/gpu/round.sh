#!/bin/bash
# GPU box script: parity tests, then the default bench line, then the rocprofv3 passes of
# tools/profile.sh.  Every GPU step has its own time limit and the chain stops at the first failure.
#   TAG=r02a [SKIP_TESTS=1] [SKIP_PROF=1] [PYTEST_ARGS=...] [BENCH_ARGS=...] bash tools/gpu_round.sh
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${TAG:-r02}
if [ -z "$SKIP_TESTS" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 180 --timeout-method thread ${PYTEST_ARGS} > gpurun_out/gpu_tests_$TAG.log 2>&1
  rc=$?; echo "pytest rc=$rc"; tail -15 gpurun_out/gpu_tests_$TAG.log
  [ $rc -eq 0 ] || [ -n "$CONTINUE_ON_FAIL" ] || exit $rc
fi
if [ -z "$SKIP_BENCH" ]; then
  timeout -k 10 600 python bench.py ${BENCH_ARGS} > gpurun_out/bench_$TAG.log 2>&1
  rc=$?; echo "bench rc=$rc"; tail -c 3000 gpurun_out/bench_$TAG.log
  [ $rc -eq 0 ] || exit $rc
fi
if [ -z "$SKIP_PROF" ]; then
  TAG=$TAG bash tools/profile.sh
fi
