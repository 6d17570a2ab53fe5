#!/bin/bash
# One gpurun call: GPU parity tests, smoke, and a short bench; every GPU step
# under its own time limit; stops at the first abort / fault / timeout.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
SCALE=${SCALE:-20}
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -5 gpurun_out/pytest_gpu.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
rc=$?; echo "smoke rc=$rc"; tail -3 gpurun_out/smoke.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 600 python bench.py --scale $SCALE --steps 3 --warmup 1 > gpurun_out/bench_s$SCALE.json 2> gpurun_out/bench_s$SCALE.log
rc=$?; echo "bench rc=$rc"; cat gpurun_out/bench_s$SCALE.json; tail -5 gpurun_out/bench_s$SCALE.log
exit $rc
