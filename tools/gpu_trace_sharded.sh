#!/bin/bash
# rocprofv3 kernel trace of the sharded bench path on one GPU (one rank, no launcher).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp RANK=0 WORLD_SIZE=1 LOCAL_RANK=0 MASTER_ADDR=127.0.0.1 MASTER_PORT=29561
TAG=${TAG:-trace_sh}
SCALE=${SCALE:-24}
timeout -k 10 600 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d gpurun_out/prof_$TAG -o run -- \
  python3 bench.py --sharded --scale $SCALE --steps 3 --warmup 1 --cpu-baseline off > gpurun_out/prof_$TAG.json 2> gpurun_out/prof_$TAG.log
rc=$?; echo "rocprof rc=$rc"; cat gpurun_out/prof_$TAG.json
exit $rc
