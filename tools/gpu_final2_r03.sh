#!/bin/bash
# Round-3 closing check on one GPU box: the whole -m gpu suite, smoke(), then the default bench line and the
# sharded N=1 line (tools/gpu_bench_r03.sh), each under its own limit.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
TAG=${TAG:-fin2}
timeout -k 10 900 python3 -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread -p no:cacheprovider \
  > gpurun_out/pytest_gpu_$TAG.log 2>&1 || { tail -30 gpurun_out/pytest_gpu_$TAG.log; exit 1; }
tail -1 gpurun_out/pytest_gpu_$TAG.log
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" || exit 1
bash tools/gpu_bench_r03.sh $TAG
