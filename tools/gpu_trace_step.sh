#!/bin/bash
# Parity subset, then a kernel trace of a short S=28 bench (per-step timeline).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${TAG:-trace}
TESTS=${TESTS:-tests/test_gpu_parity.py}
if [ "${SKIP_TESTS:-0}" != 1 ]; then
  timeout -k 10 400 python -u -m pytest $TESTS -m gpu -x -q --timeout 200 --timeout-method thread -p no:cacheprovider \
    > gpurun_out/pytest_$TAG.log 2>&1
  rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_$TAG.log
  [ $rc -eq 0 ] || exit $rc
fi
PM_LINES_NOCOOP=1 timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_$TAG -o run -- \
  python3 bench.py --steps 3 --warmup 1 --cpu-baseline off --c3 off --fixture-check off > gpurun_out/prof_$TAG.json 2> gpurun_out/prof_$TAG.log
rc=$?; echo "rocprof rc=$rc"; cat gpurun_out/prof_$TAG.json; tail -2 gpurun_out/prof_$TAG.log
exit $rc
