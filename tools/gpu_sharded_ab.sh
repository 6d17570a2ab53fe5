#!/bin/bash
# GPU box: the sharded path at N = 1 (bench.py --sharded under torch.distributed.run) with the settings in
# SETTINGS (VAR=VALUE, one run each; "none" = defaults), ms/step of each.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for e in ${SETTINGS:-none}; do
  ( [ "$e" != none ] && export "$e"; timeout -k 10 300 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 1 \
      --master-addr 127.0.0.1 --master-port 29535 bench.py --gpus 1 --sharded --steps 20 --warmup 5 --cpu-baseline off \
      --fixture-check off > gpurun_out/shab_$e.json 2> gpurun_out/shab_$e.err ) || { tail -5 gpurun_out/shab_$e.err; exit 1; }
  echo "$e: $(python3 -c "import json;print(json.loads(open('gpurun_out/shab_$e.json').read().strip().splitlines()[-1])['ms_per_step'])") ms"
done
