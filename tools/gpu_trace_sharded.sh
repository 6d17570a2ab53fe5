#!/bin/bash
# GPU box: kernel trace of the sharded path at N = 1 (RCCL with one rank, bench.py --sharded, no launcher: the
# process is its own rank 0), for the per-step timeline of the sharded search (tools/step_timeline.py).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp RANK=0 LOCAL_RANK=0 WORLD_SIZE=1 MASTER_ADDR=127.0.0.1 MASTER_PORT=29541
TAG=${TAG:-sharded}
PM_LINES_NOCOOP=1 timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_$TAG -o run -- \
  python3 bench.py --sharded --steps 3 --warmup 1 --cpu-baseline off --c3 off --nlcc off --fixture-check off \
  > gpurun_out/prof_$TAG.json 2> gpurun_out/prof_$TAG.log
rc=$?; echo "rocprof rc=$rc"; tail -2 gpurun_out/prof_$TAG.log
[ $rc -eq 0 ] && python3 tools/step_timeline.py gpurun_out/prof_$TAG > gpurun_out/timeline_$TAG.txt && tail -60 gpurun_out/timeline_$TAG.txt
exit $rc
