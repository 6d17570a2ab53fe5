#!/bin/bash
# GPU box: the default bench against the same bench under each environment setting given as an argument
# ("NAME=VALUE"), alternating, steps 20; prints ms/step per run.
mkdir -p gpurun_out
run() {
  env "$@" timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 --cpu-baseline off --fixture-check off \
    > gpurun_out/ab.json 2> gpurun_out/ab.err || { tail -3 gpurun_out/ab.err; exit 1; }
  python3 -c "import json; d=json.loads(open('gpurun_out/ab.json').read().strip().splitlines()[-1]); print('$*', d['ms_per_step'], d['roofline']['avg_launch_ms'])"
}
for rep in 1 2; do
  run PM_AB=0
  for e in "$@"; do run $e; done
done
