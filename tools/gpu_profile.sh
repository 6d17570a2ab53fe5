#!/bin/bash
# Round profile: default bench line, rocprofv3 kernel-trace --stats of the same
# bench command, and the k_lcc_first PMC passes; every GPU step under its own limit.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${TAG:-r02}
timeout -k 10 500 python3 -u bench.py > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.log
rc=$?; echo "bench rc=$rc"; cat gpurun_out/bench_$TAG.json; tail -4 gpurun_out/bench_$TAG.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_$TAG -o run -- \
  python3 -u bench.py --cpu-baseline off > gpurun_out/prof_$TAG.json 2> gpurun_out/prof_$TAG.log
rc=$?; echo "rocprof rc=$rc"; cat gpurun_out/prof_$TAG.json; [ $rc -eq 0 ] || exit $rc
TAG=pmc_$TAG bash tools/gpu_pmc_k1.sh
