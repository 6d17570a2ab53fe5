#!/bin/bash
# Iteration loop on one GPU call: a parity subset, superstep-0 variant timing
# and a short S=28 bench; each GPU step under its own limit, chained.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
TAG=${TAG:-iter}
TESTS=${TESTS:-tests/test_gpu_parity.py}
timeout -k 10 400 python -u -m pytest $TESTS -m gpu -x -q --timeout 200 --timeout-method thread -p no:cacheprovider \
  > gpurun_out/pytest_$TAG.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_$TAG.log
[ $rc -eq 0 ] || exit $rc
if [ -n "${VARIANTS:-}" ]; then
  timeout -k 10 200 python3 tools/k1_variants.py 28 8 $VARIANTS > gpurun_out/var_$TAG.log 2>&1
  rc=$?; echo "variants rc=$rc"; cat gpurun_out/var_$TAG.log | grep variant
  [ $rc -eq 0 ] || exit $rc
fi
if [ "${BENCH:-1}" = 1 ]; then
  timeout -k 10 300 python3 bench.py --steps 5 --warmup 2 --cpu-baseline off > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.log
  rc=$?; echo "bench rc=$rc"; cat gpurun_out/bench_$TAG.json; tail -2 gpurun_out/bench_$TAG.log
  [ $rc -eq 0 ] || exit $rc
fi
exit 0
