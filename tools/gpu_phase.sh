#!/bin/bash
# One S=28 search step with PM_PHASE_TIMES=1 (per-phase host times, NLC line
# phase stamps) and the kernel trace of the same command: where the step's
# time goes outside k_lcc_first.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${TAG:-phase}
PM_PHASE_TIMES=1 timeout -k 10 300 python3 -u bench.py --steps 2 --warmup 1 --cpu-baseline off \
  > gpurun_out/$TAG.json 2> gpurun_out/$TAG.log
rc=$?
echo "phase rc=$rc"
grep -E "^\[pm\]" gpurun_out/$TAG.log | tail -40
exit $rc
