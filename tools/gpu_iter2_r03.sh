#!/bin/bash
# GPU box, one iteration: parity subset (every step under its own limit), then the bench A/B over env settings
# given as arguments ("NAME=VALUE", tools/gpu_ab_env.sh), then one phase-times step.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
TESTS=${TESTS:-tests/test_gpu_parity.py tests/test_gpu_configs.py::test_c4_s28_tree_one_gpu}
timeout -k 10 600 python3 -u -m pytest $TESTS -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider \
  > gpurun_out/pytest_iter.log 2>&1 || { tail -30 gpurun_out/pytest_iter.log; exit 1; }
tail -2 gpurun_out/pytest_iter.log
bash tools/gpu_ab_env.sh "$@" || exit 1
PM_PHASE_TIMES=1 timeout -k 10 300 python3 -u bench.py --steps 3 --warmup 2 --cpu-baseline off --fixture-check off \
  > gpurun_out/phase_iter.json 2> gpurun_out/phase_iter.log || exit 1
grep -E "^\[pm\] (run_beta|host|line 4)" gpurun_out/phase_iter.log | tail -3
