#!/bin/bash
# Round-3 final evidence on one GPU box, each step under its own limit: the -m gpu suite, the default bench line,
# the sharded N=1 line, rocprofv3 stats + PMC passes (tools/gpu_profile_r03.sh), a kernel trace of the step.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${TAG:-fin}
timeout -k 10 900 python3 -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread -p no:cacheprovider \
  > gpurun_out/pytest_gpu_$TAG.log 2>&1 || { tail -30 gpurun_out/pytest_gpu_$TAG.log; exit 1; }
tail -1 gpurun_out/pytest_gpu_$TAG.log
bash tools/gpu_bench_r03.sh $TAG || exit 1
TAG=$TAG SKIP_VARIANTS=1 bash tools/gpu_profile_r03.sh || exit 1
python3 tools/parse_pmc_step.py gpurun_out $TAG gpurun_out/pmc_step_$TAG.json || exit 1
PM_LINES_NOCOOP=1 timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/trace_$TAG -o run -- \
  python3 bench.py --steps 3 --warmup 1 --cpu-baseline off --fixture-check off > gpurun_out/trace_$TAG.json 2> gpurun_out/trace_$TAG.log || exit 1
python3 tools/step_timeline.py gpurun_out/trace_$TAG > gpurun_out/timeline_$TAG.txt && cut -c1-100 gpurun_out/timeline_$TAG.txt
