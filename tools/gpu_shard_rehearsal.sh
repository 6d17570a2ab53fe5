#!/bin/bash
# Sharded bench path on one GPU (one rank: RCCL, owner partitioning, exchanges).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
SCALE=${SCALE:-24}
timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 \
  --master-port 29533 bench.py ${EXTRA:-} --sharded --scale $SCALE --steps 5 --warmup 2 \
  > gpurun_out/shard1_s$SCALE.json 2> gpurun_out/shard1_s$SCALE.log
rc=$?; echo "sharded bench rc=$rc"; cat gpurun_out/shard1_s$SCALE.json; grep "rank 0" gpurun_out/shard1_s$SCALE.log
exit $rc
