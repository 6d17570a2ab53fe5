#!/bin/bash
# Superstep-0 kernel iteration: GPU parity tests, then the S=28 ablation and a short bench.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
TAG=${TAG:-k1}
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 250 --timeout-method thread -p no:cacheprovider \
  --deselect tests/test_gpu_configs.py > gpurun_out/pytest_$TAG.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -5 gpurun_out/pytest_$TAG.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -u tools/ubench.py 28 8 ${VARIANTS:-0,1,8,2,4} > gpurun_out/ubench_$TAG.log 2>&1
rc=$?; cat gpurun_out/ubench_$TAG.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py --scale 28 --p-gen 8 --steps 10 --warmup 3 --cpu-baseline off > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.log
rc=$?; cat gpurun_out/bench_$TAG.json; tail -3 gpurun_out/bench_$TAG.log
exit $rc
