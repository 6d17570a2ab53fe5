#!/bin/bash
# rocprofv3 kernel trace of a short default bench (per-kernel timeline of a step).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp PM_GRAPH_CACHE=/tmp/pmgraph
TAG=${TAG:-trace}
SCALE=${SCALE:-24}
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_$TAG -o run -- \
  python3 bench.py --scale $SCALE --steps 3 --warmup 1 --cpu-baseline off > gpurun_out/prof_$TAG.json 2> gpurun_out/prof_$TAG.log
rc=$?; echo "rocprof rc=$rc"; cat gpurun_out/prof_$TAG.json
exit $rc
