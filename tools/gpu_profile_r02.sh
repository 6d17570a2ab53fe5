#!/bin/bash
# Round-2 evidence at the S=28 headline: rocprofv3 kernel stats of the bench
# command, then the PMC passes of k_lcc_first (one rocprofv3 run per counter
# group, --kernel-trace only), each GPU step under its own limit.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${TAG:-r02}
SCALE=${SCALE:-28}
PGEN=${PGEN:-8}
if [ "${SKIP_STATS:-0}" != 1 ]; then
  timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_$TAG -o run -- \
    python3 bench.py --steps 5 --warmup 2 --cpu-baseline off > gpurun_out/prof_$TAG.json 2> gpurun_out/prof_$TAG.log
  rc=$?; echo "rocprof stats rc=$rc"; cat gpurun_out/prof_$TAG.json; tail -3 gpurun_out/prof_$TAG.log
  [ $rc -eq 0 ] || exit $rc
fi
i=0
for ctr in ${PMC_GROUPS:-"FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum" "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA" "SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_LDS_BANK_CONFLICT SQ_INSTS_SMEM SQ_WAIT_INST_LDS"}; do
  i=$((i+1))
  timeout -s KILL 150 rocprofv3 --kernel-trace --pmc $ctr --kernel-include-regex "k_lcc_first" --output-format csv \
    -d gpurun_out/pmc_${TAG}_$i -o run -- python3 tools/k1_harness.py $SCALE $PGEN 3 > gpurun_out/pmc_${TAG}_$i.log 2>&1
  rc=$?; echo "pmc pass $i ($ctr) rc=$rc"; tail -1 gpurun_out/pmc_${TAG}_$i.log
  [ $rc -eq 0 ] || exit $rc
done
python3 tools/parse_pmc.py gpurun_out pmc_${TAG} $SCALE $PGEN gpurun_out/pmc_${TAG}.json
