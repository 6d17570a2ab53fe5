#!/bin/bash
# Whole GPU test suite (the BASELINE-config cases excluded unless CONFIGS=1), then the RCCL one-rank probe.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
TAG=${TAG:-suite}
DESEL="--deselect tests/test_gpu_configs.py"
[ "${CONFIGS:-0}" = 1 ] && DESEL=""
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread -p no:cacheprovider $DESEL \
  > gpurun_out/pytest_$TAG.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "FAILED|ERROR|passed|failed" gpurun_out/pytest_$TAG.log | tail -15
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
if [ "${PROBE:-1}" = 1 ]; then
  timeout -k 10 400 python3 -u tools/rccl_probe.py > gpurun_out/rccl_probe.log 2>&1; echo "rccl rc=$?"; cat gpurun_out/rccl_probe.log
fi
exit $rc
