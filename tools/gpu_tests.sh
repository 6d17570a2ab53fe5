#!/bin/bash
# GPU box: pytest over the given test paths / node ids (default: the whole -m gpu suite), log under gpurun_out/.
# usage: TAG=x [LIMIT=seconds] tools/gpu_tests.sh [pytest args ...]
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
TAG=${TAG:-run}
LIMIT=${LIMIT:-1100}
[ $# -eq 0 ] && set -- tests
timeout -k 10 "$LIMIT" python3 -u -m pytest "$@" -m gpu -x -v -s --timeout 600 --timeout-method thread -p no:cacheprovider \
  > gpurun_out/pytest_gpu_$TAG.log 2>&1
rc=$?
grep -E "PASSED|FAILED|ERROR|passed|failed" gpurun_out/pytest_gpu_$TAG.log | tail -40
exit $rc
