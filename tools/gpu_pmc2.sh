#!/bin/bash
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 --list-avail > gpurun_out/list_avail.txt 2>&1; echo "list rc=$?"
EXTRA="FETCH_SIZE" bash tools/gpu_pmc_quick.sh s1 > gpurun_out/pmcq_s1.out 2>&1; echo "pmc rc=$?"
tail -25 gpurun_out/pmcq_s1.out
timeout -s KILL 150 rocprofv3 --kernel-trace --pmc WRITE_SIZE --kernel-include-regex "k_lcc_first" --output-format csv -d gpurun_out/pmcq_s1_9 -o run -- python3 tools/k1_harness.py 28 8 3 > gpurun_out/pmcq_s1_9.log 2>&1; echo "write rc=$?"
python3 tools/parse_pmc.py gpurun_out pmcq_s1 28 8 gpurun_out/pmcq_s1.json
