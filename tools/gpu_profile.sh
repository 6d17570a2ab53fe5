#!/bin/bash
# Profiling evidence at the S=28 headline (one GPU step per command, each under its own limit):
#   1. rocprofv3 --kernel-trace --stats of the bench command (k_lines on an ordinary launch: PM_LINES_NOCOOP=1,
#      the cooperative queue crashes rocprofv3's teardown);
#   2. the PMC passes of k_lcc_first (tools/k1_harness.py) and of the later supersteps (k_lcc_step, the bench);
#   3. the superstep-0 ablation variants (libpm_diag.so).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${TAG:-r04}
SCALE=${SCALE:-28}
PGEN=${PGEN:-8}
if [ "${SKIP_STATS:-0}" != 1 ]; then
  PM_LINES_NOCOOP=1 timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_$TAG -o run -- \
    python3 bench.py --steps 5 --warmup 2 --cpu-baseline off --fixture-check off --c3 off --nlcc off --sharded-n1 off > gpurun_out/prof_$TAG.json 2> gpurun_out/prof_$TAG.log
  rc=$?; echo "rocprof stats rc=$rc"; tail -2 gpurun_out/prof_$TAG.log
  [ $rc -eq 0 ] || exit $rc
fi
G1="FETCH_SIZE"
G2="WRITE_SIZE"
G3="TCC_HIT_sum TCC_MISS_sum"
G4="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA"
G5="SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_LDS_BANK_CONFLICT SQ_INSTS_SMEM SQ_WAIT_INST_LDS"
if [ "${SKIP_K1:-0}" != 1 ]; then
  i=0
  for ctr in "$G1" "$G2" "$G3" "$G4" "$G5"; do
    i=$((i+1))
    timeout -s KILL 150 rocprofv3 --kernel-trace --pmc $ctr --kernel-include-regex "k_lcc_first" --output-format csv \
      -d gpurun_out/pmc_${TAG}_$i -o run -- python3 tools/k1_harness.py $SCALE $PGEN 3 > gpurun_out/pmc_${TAG}_$i.log 2>&1
    rc=$?; echo "pmc pass $i ($ctr) rc=$rc"; tail -1 gpurun_out/pmc_${TAG}_$i.log
    [ $rc -eq 0 ] || exit $rc
  done
  python3 tools/parse_pmc.py gpurun_out pmc_${TAG} $SCALE $PGEN gpurun_out/pmc_${TAG}.json
fi
if [ "${SKIP_STEP:-0}" != 1 ]; then
  i=0
  for ctr in "$G1" "$G2" "$G4" "$G5"; do
    i=$((i+1))
    PM_LINES_NOCOOP=1 timeout -s KILL 200 rocprofv3 --kernel-trace --pmc $ctr --kernel-include-regex "k_lcc_step" --output-format csv \
      -d gpurun_out/pmcstep_${TAG}_$i -o run -- python3 bench.py --steps 1 --warmup 1 --cpu-baseline off --fixture-check off --c3 off --nlcc off --sharded-n1 off \
      > gpurun_out/pmcstep_${TAG}_$i.log 2>&1
    rc=$?; echo "k_lcc_step pmc pass $i ($ctr) rc=$rc"
    [ $rc -eq 0 ] || exit $rc
  done
fi
if [ "${SKIP_VARIANTS:-0}" != 1 ]; then
  timeout -k 10 200 python3 tools/k1_variants.py $SCALE $PGEN ${VARIANTS:-0 1024 2048 4096 7168 8 16} > gpurun_out/k1_variants_${TAG}.log 2>&1
  echo "variants rc=$?"; cat gpurun_out/k1_variants_${TAG}.log | tail -8
fi
