#!/bin/bash
# Default bench (C2, S=24) + rocprofv3 kernel-trace/stats of the same command.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${TAG:-r01}
timeout -k 10 900 python3 bench.py > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.log
rc=$?; echo "bench rc=$rc"; cat gpurun_out/bench_$TAG.json; tail -4 gpurun_out/bench_$TAG.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 900 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_$TAG -o run -- \
  python3 bench.py --cpu-baseline off > gpurun_out/prof_$TAG.json 2> gpurun_out/prof_$TAG.log
rc=$?; echo "rocprof rc=$rc"; cat gpurun_out/prof_$TAG.json
exit $rc
