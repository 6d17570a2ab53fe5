#!/bin/bash
# GPU box: the default bench line, then the sharded path at N = 1 (rehearsal), logs under gpurun_out/.
set -o pipefail
mkdir -p gpurun_out
TAG=${1:-r04}
timeout -k 10 400 python3 bench.py --steps 20 --warmup 5 > gpurun_out/bench_${TAG}.json 2> gpurun_out/bench_${TAG}.err || exit $?
tail -3 gpurun_out/bench_${TAG}.err
timeout -k 10 400 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 \
    --master-port 29533 bench.py --gpus 1 --sharded --steps 20 --warmup 5 --cpu-baseline off \
    > gpurun_out/bench_${TAG}_sharded.json 2> gpurun_out/bench_${TAG}_sharded.err
rc=$?
tail -3 gpurun_out/bench_${TAG}_sharded.err
exit $rc
