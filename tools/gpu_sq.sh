#!/bin/bash
# SQ counters of the superstep-0 kernel (one --pmc group per rocprofv3 run).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
SCALE=${SCALE:-22}
VAR=${VAR:-0}
i=0
for ctr in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY" "SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SALU SQ_LDS_BANK_CONFLICT" "TCP_TCC_READ_REQ_sum TCC_HIT_sum TCC_MISS_sum TA_BUSY_avr" "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $ctr --kernel-include-regex "k_lcc_first" --output-format csv \
    -d gpurun_out/sq_$i -o run -- python3 tools/ubench.py $SCALE $VAR > gpurun_out/sq_$i.log 2>&1
  rc=$?; echo "pass $i rc=$rc"; if [ $rc -ne 0 ]; then tail -5 gpurun_out/sq_$i.log; exit $rc; fi
done
python3 - <<'PY'
import csv, glob
agg = {}
for f in glob.glob("gpurun_out/sq_*/**/*counter_collection*.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        agg.setdefault(r["Counter_Name"], {}).setdefault(r["Dispatch_Id"], 0.0)
        agg[r["Counter_Name"]][r["Dispatch_Id"]] += float(r["Counter_Value"])
for k, v in sorted(agg.items()):
    print(f"{k:28s} per-dispatch avg {sum(v.values())/len(v):.4g}  ({len(v)} dispatches)")
PY
