#!/bin/bash
# PMC passes for the dominant kernel (k_lcc_first), each counter group in its
# own rocprofv3 run with --kernel-trace only (no sys/runtime traces with --pmc).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
SCALE=${SCALE:-24}
TAG=${TAG:-s$SCALE}
export TMPDIR=/tmp
i=0
for ctr in "FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum"; do
  i=$((i+1))
  timeout -k 10 600 rocprofv3 --pmc $ctr --kernel-include-regex "k_lcc_first" --output-format csv \
    -d gpurun_out/pmc_${TAG}_$i -o run -- python3 bench.py --scale $SCALE --steps 2 --warmup 0 --cpu-baseline off \
    > gpurun_out/pmc_${TAG}_$i.json 2> gpurun_out/pmc_${TAG}_$i.log
  rc=$?; echo "pmc pass $i ($ctr) rc=$rc"
  if [ $rc -ne 0 ]; then tail -5 gpurun_out/pmc_${TAG}_$i.log; exit $rc; fi
done
python3 tools/parse_pmc.py gpurun_out pmc_${TAG} $SCALE
