#!/bin/bash
# GPU box: the -m gpu suite, then the default bench line (and the sharded N=1 rehearsal); logs under gpurun_out/.
set -o pipefail
mkdir -p gpurun_out
TAG=${1:-r03}
timeout -k 10 900 python3 -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread \
    > gpurun_out/pytest_gpu_${TAG}.log 2>&1 || { tail -20 gpurun_out/pytest_gpu_${TAG}.log; exit 1; }
tail -2 gpurun_out/pytest_gpu_${TAG}.log
bash tools/gpu_bench_r03.sh ${TAG}
