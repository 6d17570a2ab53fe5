#!/bin/bash
# GPU box: S=28 bench line phase times (PM_PHASE_TIMES) with the single-block threshold of the NLC line kernel
# at its default and at the values in SMALLS (0: every line on the whole grid).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for sm in default ${SMALLS:-0 256}; do
  if [ "$sm" = default ]; then unset PM_SMALL_LINE; else export PM_SMALL_LINE=$sm; fi
  PM_PHASE_TIMES=1 timeout -k 10 200 python3 bench.py --steps 5 --warmup 2 --cpu-baseline off --fixture-check off --c3 off --nlcc off --sharded-n1 off \
    > gpurun_out/lines_small_$sm.json 2> gpurun_out/lines_small_$sm.err || { tail -5 gpurun_out/lines_small_$sm.err; exit 1; }
  echo "small_line=$sm: $(python3 -c "import json;print(json.loads(open('gpurun_out/lines_small_$sm.json').read().strip().splitlines()[-1])['ms_per_step'])") ms/step"
  grep "line 4" gpurun_out/lines_small_$sm.err | tail -1
  grep -A1 "line 4" gpurun_out/lines_small_$sm.err | tail -1
done
