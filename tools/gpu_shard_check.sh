#!/bin/bash
# Sharded path check: the in-process shard parity tests, then the RCCL one-rank probe.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_gpu_shards.py -m gpu -x -v --timeout 250 --timeout-method thread \
  -p no:cacheprovider > gpurun_out/pytest_shards.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -15 gpurun_out/pytest_shards.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python3 -u tools/rccl_probe.py > gpurun_out/rccl_probe.log 2>&1; echo "rccl rc=$?"; cat gpurun_out/rccl_probe.log
exit 0
