#!/bin/bash
# rocprofv3 kernel-trace + stats of one bench configuration (no PMC here).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
SCALE=${SCALE:-22}
TAG=${TAG:-s$SCALE}
export TMPDIR=/tmp
timeout -k 10 900 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_$TAG -o run -- \
  python3 bench.py --scale $SCALE --steps 5 --warmup 1 --cpu-baseline off > gpurun_out/prof_$TAG.json 2> gpurun_out/prof_$TAG.log
rc=$?; echo "rocprof rc=$rc"; cat gpurun_out/prof_$TAG.json
find gpurun_out/prof_$TAG -name "*stats*" | head
exit $rc
