#!/bin/bash
# GPU box: a build's parity subset, the default bench line and a rocprofv3 kernel trace of a short bench (step
# timeline), each step under its own limit and chained.
# usage: TAG=x bash tools/gpu_r6b.sh
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${TAG:-r6b}
LIMIT=500 TAG=$TAG bash tools/gpu_tests.sh tests/test_gpu_parity.py tests/test_gpu_tds.py tests/test_gpu_selected.py \
  tests/test_gpu_directed.py tests/test_gpu_shards.py || exit 1
timeout -k 10 400 python3 bench.py --steps 20 --warmup 5 --cpu-baseline off --sharded-n1 off \
  > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err || { tail -5 gpurun_out/bench_$TAG.err; exit 1; }
tail -3 gpurun_out/bench_$TAG.err
PM_LINES_NOCOOP=1 timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_$TAG -o run -- \
  python3 bench.py --steps 5 --warmup 2 --cpu-baseline off --fixture-check off --c3 off --nlcc off --sharded-n1 off \
  > gpurun_out/prof_$TAG.json 2> gpurun_out/prof_$TAG.log || { tail -5 gpurun_out/prof_$TAG.log; exit 1; }
python3 tools/step_timeline.py gpurun_out/prof_$TAG > gpurun_out/timeline_$TAG.txt && cat gpurun_out/timeline_$TAG.txt | cut -c1-110
