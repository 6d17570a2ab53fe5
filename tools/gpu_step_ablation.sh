#!/bin/bash
# GPU box: the first later superstep (k_lcc_step's first dispatch after superstep 0) at S=28 under timing
# variants -- PM_DIAG_STEP bits (1 no neighbour-T_pub gathers, 2 no survivor row moves, 4 no entry stores; results
# are wrong, timing only), environment settings (STEP_ENVS) and other builds (STEP_LIBS) -- each run under
# rocprofv3 --kernel-trace.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp PM_LINES_NOCOOP=1
for d in ${STEP_DIAGS:-0 1 2 4 7}; do
  PM_DIAG_STEP=$d timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/stepab_d$d -o run -- \
    python3 bench.py --steps 3 --warmup 1 --cpu-baseline off --fixture-check off --c3 off --nlcc off --sharded-n1 off \
    > gpurun_out/stepab_d$d.json 2> gpurun_out/stepab_d$d.log || { tail -5 gpurun_out/stepab_d$d.log; exit 1; }
done
for e in ${STEP_ENVS:-}; do  # VAR=VALUE settings, one run each
  ( export "$e"; timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/stepab_$e -o run -- \
    python3 bench.py --steps 3 --warmup 1 --cpu-baseline off --fixture-check off --c3 off --nlcc off --sharded-n1 off \
    > gpurun_out/stepab_$e.json 2> gpurun_out/stepab_$e.log ) || { tail -5 gpurun_out/stepab_$e.log; exit 1; }
done
for lib in ${STEP_LIBS:-}; do
  PM_LIB=fuzzypatternmatching_amd/lib/$lib timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/stepab_$lib -o run -- \
    python3 bench.py --steps 3 --warmup 1 --cpu-baseline off --fixture-check off --c3 off --nlcc off --sharded-n1 off \
    > gpurun_out/stepab_$lib.json 2> gpurun_out/stepab_$lib.log || { tail -5 gpurun_out/stepab_$lib.log; exit 1; }
done
python3 tools/step_first_dispatch.py gpurun_out/stepab_*
