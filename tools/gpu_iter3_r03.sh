#!/bin/bash
# GPU box: parity subset (one GPU, shards, S=28 fixture), the default bench line, then config C5 at size.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
TAG=${TAG:-i3}
TESTS=${TESTS:-tests/test_gpu_parity.py tests/test_gpu_shards.py tests/test_gpu_configs.py::test_c4_s28_tree_one_gpu}
timeout -k 10 700 python3 -u -m pytest $TESTS -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider \
  > gpurun_out/pytest_$TAG.log 2>&1 || { tail -30 gpurun_out/pytest_$TAG.log; exit 1; }
tail -1 gpurun_out/pytest_$TAG.log
timeout -k 10 400 python3 bench.py --steps 20 --warmup 5 --cpu-baseline off > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err \
  || { tail -5 gpurun_out/bench_$TAG.err; exit 1; }
python3 -c "import json; d=json.loads(open('gpurun_out/bench_$TAG.json').read().strip().splitlines()[-1]); print('bench', d['ms_per_step'], d['roofline']['avg_launch_ms'], d['fixture'])"
if [ "${SKIP_C5:-0}" != 1 ]; then
  timeout -k 10 300 python3 -u tools/c5_at_size.py --scale 20 --oracle --out gpurun_out/c5_s20.json \
    2> gpurun_out/c5_s20.log || { tail -20 gpurun_out/c5_s20.log; exit 1; }
  tail -2 gpurun_out/c5_s20.log
  timeout -k 10 900 python3 -u tools/c5_at_size.py --scale 27 --oracle --out gpurun_out/c5_s27.json \
    2> gpurun_out/c5_s27.log
  rc=$?; tail -12 gpurun_out/c5_s27.log; exit $rc
fi
