#!/bin/bash
# GPU box: selected -m gpu tests (args: tag, pytest paths / -k ...), log under gpurun_out/.
set -o pipefail
mkdir -p gpurun_out
TAG=$1; shift
timeout -k 10 1100 python3 -u -m pytest -m gpu -v --timeout 300 --timeout-method thread "$@" \
    > gpurun_out/pytest_gpu_${TAG}.log 2>&1
rc=$?
tail -5 gpurun_out/pytest_gpu_${TAG}.log
exit $rc
