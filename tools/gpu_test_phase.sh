#!/bin/bash
# GPU parity tests, then the phase timing of the default bench (cached graph).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp PM_GRAPH_CACHE=/tmp/pmgraph
TAG=${TAG:-r01}
timeout -k 10 800 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider \
  > gpurun_out/pytest_$TAG.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -4 gpurun_out/pytest_$TAG.log
[ $rc -ne 0 ] && exit $rc
PM_PHASE_TIMES=1 timeout -k 10 300 python3 bench.py --steps 5 --warmup 2 --cpu-baseline off \
  > gpurun_out/phase_$TAG.json 2> gpurun_out/phase_$TAG.log
rc=$?; echo "phase rc=$rc"; grep "\[pm\]" gpurun_out/phase_$TAG.log | tail -6; cat gpurun_out/phase_$TAG.json
exit $rc
