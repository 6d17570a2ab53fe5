#!/bin/bash
# GPU box: the S=28 bench with cooperative launches (default) and with ordinary ones (PM_LINES_NOCOOP=1: k_lines and
# the list compaction's scan), alternating on one box, each run under its own limit.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
B="python3 bench.py --steps 30 --warmup 5 --cpu-baseline off --c3 off --nlcc off --sharded-n1 off --fixture-check off"
for i in 1 2; do
  for mode in coop nocoop; do
    if [ $mode = nocoop ]; then export PM_LINES_NOCOOP=1; else unset PM_LINES_NOCOOP; fi
    timeout -k 10 240 $B > gpurun_out/coop_ab_${mode}_$i.json 2> gpurun_out/coop_ab_${mode}_$i.err || { tail -3 gpurun_out/coop_ab_${mode}_$i.err; exit 1; }
    echo "$mode $i: $(python3 -c "import json;print(json.loads(open('gpurun_out/coop_ab_${mode}_$i.json').read().strip().splitlines()[-1])['ms_per_step'])") ms"
  done
done
