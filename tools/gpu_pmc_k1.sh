#!/bin/bash
# PMC passes of the superstep-0 kernel, one rocprofv3 run per counter group
# (--kernel-trace only, no other trace domains), each under its own limit.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${TAG:-pmc}
SCALE=${SCALE:-28}
PGEN=${PGEN:-8}
timeout -k 10 60 rocprofv3 --list-avail > gpurun_out/${TAG}_avail.txt 2>&1 || true
i=0
for ctr in ${GROUPS_OVERRIDE:-"SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS" "SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_LDS_BANK_CONFLICT SQ_INSTS_SMEM SQ_WAIT_INST_LDS" "FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum"}; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $ctr --kernel-include-regex "k_lcc_first" --output-format csv \
    -d gpurun_out/${TAG}_$i -o run -- python3 tools/k1_harness.py $SCALE $PGEN 3 > gpurun_out/${TAG}_$i.log 2>&1
  rc=$?; echo "pass $i ($ctr) rc=$rc"; tail -2 gpurun_out/${TAG}_$i.log
  [ $rc -eq 0 ] || exit $rc
done
exit 0
