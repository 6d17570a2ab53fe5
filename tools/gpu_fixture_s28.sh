#!/bin/bash
# GPU box: make the S=28 oracle fixture, then check the GPU headline path against it, then bench.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 1000 python3 -u tests/golden/make_rmat_fixture.py --scale 28 --p-gen 8 \
    --out gpurun_out/rmat_s28_p8_tree.json > gpurun_out/fixture_s28.log 2>&1 || exit $?
cp gpurun_out/rmat_s28_p8_tree.json tests/golden/rmat_s28_p8_tree.json
timeout -k 10 300 python3 -u -m pytest -x -v --timeout 240 --timeout-method thread tests/test_gpu_configs.py \
    -k s28 > gpurun_out/pytest_s28.log 2>&1 || exit $?
timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 --cpu-baseline off > gpurun_out/bench_r03a.json 2> gpurun_out/bench_r03a.err
