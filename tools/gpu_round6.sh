#!/bin/bash
# GPU box, round-6 closing evidence, each step under its own limit and chained:
#   1. the default bench line (what the driver runs) and the N=1 sharded launch through torch.distributed.run
#      (the shards report of an N-GPU line, one rank);
#   2. rocprofv3 --kernel-trace --stats of a short bench (per-step timeline, kernel statistics);
#   3. the PMC passes of k_lcc_first and k_lcc_step (tools/gpu_profile.sh, SKIP_STATS: step 2 did it).
# usage: TAG=r06 bash tools/gpu_round6.sh
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${TAG:-r06}
timeout -k 10 400 python3 bench.py --steps 20 --warmup 5 > gpurun_out/bench_${TAG}.json 2> gpurun_out/bench_${TAG}.err \
  || { tail -5 gpurun_out/bench_${TAG}.err; exit 1; }
tail -4 gpurun_out/bench_${TAG}.err
timeout -k 10 300 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 \
    --master-port 29533 bench.py --gpus 1 --sharded --steps 20 --warmup 5 --cpu-baseline off --c3 off --nlcc off --sharded-n1 off \
    > gpurun_out/bench_${TAG}_sharded.json 2> gpurun_out/bench_${TAG}_sharded.err \
  || { tail -5 gpurun_out/bench_${TAG}_sharded.err; exit 1; }
tail -2 gpurun_out/bench_${TAG}_sharded.err
PM_LINES_NOCOOP=1 timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_$TAG -o run -- \
  python3 bench.py --steps 5 --warmup 2 --cpu-baseline off --fixture-check off --c3 off --nlcc off --sharded-n1 off \
  > gpurun_out/prof_$TAG.json 2> gpurun_out/prof_$TAG.log || { tail -5 gpurun_out/prof_$TAG.log; exit 1; }
python3 tools/step_timeline.py gpurun_out/prof_$TAG > gpurun_out/timeline_$TAG.txt && tail -3 gpurun_out/timeline_$TAG.txt
SKIP_STATS=1 TAG=$TAG bash tools/gpu_profile.sh
