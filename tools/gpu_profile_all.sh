#!/bin/bash
# Phase timing + rocprofv3 kernel stats + PMC passes of the default bench (C2, S=24).
# The generated graph is cached under /tmp so only the first run pays for it.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp PM_GRAPH_CACHE=/tmp/pmgraph
TAG=${TAG:-r01}
PM_PHASE_TIMES=1 timeout -k 10 300 python3 bench.py --steps 3 --warmup 1 --cpu-baseline off \
  > gpurun_out/phase_$TAG.json 2> gpurun_out/phase_$TAG.log
rc=$?; echo "phase rc=$rc"; grep "\[pm\]" gpurun_out/phase_$TAG.log | tail -12
[ $rc -ne 0 ] && exit $rc
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_$TAG -o run -- \
  python3 bench.py --cpu-baseline off > gpurun_out/prof_$TAG.json 2> gpurun_out/prof_$TAG.log
rc=$?; echo "rocprof rc=$rc"; cat gpurun_out/prof_$TAG.json
[ $rc -ne 0 ] && exit $rc
i=0
for ctr in "FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum"; do
  i=$((i+1))
  timeout -k 10 -s KILL 300 rocprofv3 --pmc $ctr --kernel-include-regex "k_lcc_first" --output-format csv \
    -d gpurun_out/pmc_${TAG}_$i -o run -- python3 bench.py --steps 2 --warmup 0 --cpu-baseline off \
    > gpurun_out/pmc_${TAG}_$i.json 2> gpurun_out/pmc_${TAG}_$i.log
  rc=$?; echo "pmc pass $i ($ctr) rc=$rc"
  if [ $rc -ne 0 ]; then tail -5 gpurun_out/pmc_${TAG}_$i.log; exit $rc; fi
done
python3 tools/parse_pmc.py gpurun_out pmc_${TAG} 24
