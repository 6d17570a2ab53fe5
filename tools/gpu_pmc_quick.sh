#!/bin/bash
# GPU box: SQ instruction / wait counters of the product k_lcc_first (k1_harness, S=28), one pass per group.
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-q}
G4="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA"
G5="SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_LDS_BANK_CONFLICT SQ_INSTS_SMEM SQ_WAIT_INST_LDS"
G2="WRITE_SIZE"
i=0
for ctr in "$G5" "$G4" ${EXTRA:+"$EXTRA"}; do
  i=$((i+1))
  timeout -s KILL 150 rocprofv3 --kernel-trace --pmc $ctr --kernel-include-regex "k_lcc_first" --output-format csv \
    -d gpurun_out/pmcq_${TAG}_$i -o run -- python3 tools/k1_harness.py 28 8 3 > gpurun_out/pmcq_${TAG}_$i.log 2>&1
  rc=$?; echo "pass $i rc=$rc"; tail -1 gpurun_out/pmcq_${TAG}_$i.log
  [ $rc -eq 0 ] || exit $rc
done
python3 tools/parse_pmc.py gpurun_out pmcq_${TAG} 28 8 gpurun_out/pmcq_${TAG}.json > /dev/null
python3 -c "
import json; d=json.load(open('gpurun_out/pmcq_${TAG}.json'))['counters']
for k in sorted(d): print(f'{k:24s} {d[k]:.4g}')"
