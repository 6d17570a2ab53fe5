#!/bin/bash
# GPU box: the -m gpu suite (log under gpurun_out/), then optional extra steps.
set -o pipefail
mkdir -p gpurun_out
TAG=${1:-r03}
timeout -k 10 1100 python3 -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread ${PYTEST_ARGS} \
    > gpurun_out/pytest_gpu_${TAG}.log 2>&1
rc=$?
tail -5 gpurun_out/pytest_gpu_${TAG}.log
exit $rc
