#!/bin/bash
# Where one S=28 step's time goes: PM_PHASE_TIMES host phases, then a rocprofv3 kernel trace of a short bench
# (k_lines on an ordinary launch: PM_LINES_NOCOOP=1) and the last step's kernel timeline (tools/step_timeline.py).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${TAG:-step}
PM_PHASE_TIMES=1 timeout -k 10 300 python3 -u bench.py --steps 3 --warmup 2 --cpu-baseline off --fixture-check off \
  > gpurun_out/phase_$TAG.json 2> gpurun_out/phase_$TAG.log
rc=$?; echo "phase rc=$rc"; grep -E "^\[pm\]" gpurun_out/phase_$TAG.log | tail -24
[ $rc -eq 0 ] || exit $rc
PM_LINES_NOCOOP=1 timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/trace_$TAG -o run -- \
  python3 bench.py --steps 3 --warmup 1 --cpu-baseline off --fixture-check off > gpurun_out/trace_$TAG.json 2> gpurun_out/trace_$TAG.log
rc=$?; echo "trace rc=$rc"
[ $rc -eq 0 ] || exit $rc
python3 tools/step_timeline.py gpurun_out/trace_$TAG > gpurun_out/timeline_$TAG.txt; cat gpurun_out/timeline_$TAG.txt | cut -c1-110
