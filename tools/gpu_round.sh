#!/bin/bash
# One gpurun call: GPU parity tests, smoke, default bench, and optionally the
# S=28 headline bench; every GPU step under its own time limit, chained so the
# first abort / fault / timeout ends the call.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
TAG=${TAG:-r02}
TESTS=${TESTS:-tests}
if [ "${SKIP_TESTS:-0}" != 1 ]; then
  timeout -k 10 600 python -u -m pytest $TESTS -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider \
    > gpurun_out/pytest_gpu_$TAG.log 2>&1
  rc=$?; echo "pytest rc=$rc"; tail -5 gpurun_out/pytest_gpu_$TAG.log
  [ $rc -eq 0 ] || exit $rc
fi
if [ "${SKIP_BENCH:-0}" != 1 ]; then
  timeout -k 10 400 python -u bench.py ${BENCH_ARGS:-} > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.log
  rc=$?; echo "bench rc=$rc"; cat gpurun_out/bench_$TAG.json; tail -6 gpurun_out/bench_$TAG.log
  [ $rc -eq 0 ] || exit $rc
fi
if [ -n "${S28:-}" ]; then
  timeout -k 10 600 python -u bench.py --scale 28 --p-gen 8 --steps 3 --warmup 1 --cpu-baseline off \
    > gpurun_out/bench28_$TAG.json 2> gpurun_out/bench28_$TAG.log
  rc=$?; echo "bench28 rc=$rc"; cat gpurun_out/bench28_$TAG.json; tail -8 gpurun_out/bench28_$TAG.log
  [ $rc -eq 0 ] || exit $rc
fi
exit 0
