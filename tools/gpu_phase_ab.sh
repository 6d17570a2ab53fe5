#!/bin/bash
# GPU box: per-superstep device times (PM_PHASE_TIMES, fine timing) of the S=28 search under each env setting
# given as an argument (the first run: defaults).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for e in PM_AB=0 "$@"; do
  env $e PM_PHASE_TIMES=1 timeout -k 10 300 python3 -u bench.py --steps 3 --warmup 2 --cpu-baseline off --fixture-check off \
    > gpurun_out/pab.json 2> gpurun_out/pab.log || { tail -5 gpurun_out/pab.log; exit 1; }
  echo "== $e"; grep -E "^\[pm\] (LP itr 0 superstep [0-3]|run_beta|line 4)" gpurun_out/pab.log | tail -6
done
