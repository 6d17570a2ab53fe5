#!/bin/bash
# GPU box, round evidence, each step under its own limit and chained: the -m gpu suite, the default bench line
# (and the sharded N=1 rehearsal), the in-process shard scaling of config C5 (tools/shard_scaling.py).
# usage: TAG=x [SKIP_TESTS=1] [SKIP_SCALING=1] tools/gpu_round.sh
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
TAG=${TAG:-r04}
if [ "${SKIP_TESTS:-0}" != 1 ]; then
  TAG=$TAG LIMIT=1300 bash tools/gpu_tests.sh || exit 1
fi
bash tools/gpu_bench.sh $TAG || exit 1
if [ "${SKIP_SCALING:-0}" != 1 ]; then
  timeout -k 10 500 python3 tools/shard_scaling.py --config c5 --out gpurun_out/shards_c5_$TAG.json \
    > /dev/null 2> gpurun_out/shards_c5_$TAG.err || { tail -5 gpurun_out/shards_c5_$TAG.err; exit 1; }
  cat gpurun_out/shards_c5_$TAG.err
fi
