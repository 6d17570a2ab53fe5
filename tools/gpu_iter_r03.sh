#!/bin/bash
# GPU box, one iteration of a kernel change: superstep-0 variant timings (libpm_diag.so),
# then the parity suites named in $TESTS (default: parity + S=28 fixture), then a short bench.
set -o pipefail
mkdir -p gpurun_out
TAG=${1:-it}
if [ "${SKIP_VARIANTS:-0}" != 1 ]; then
  timeout -k 10 240 python3 tools/k1_variants.py 28 8 ${VARIANTS:-0 8 16 32 128 1} > gpurun_out/k1v_${TAG}.log 2>&1 \
    || { tail -5 gpurun_out/k1v_${TAG}.log; exit 1; }
  cat gpurun_out/k1v_${TAG}.log | grep variant
fi
timeout -k 10 900 python3 -u -m pytest ${TESTS:-tests/test_gpu_parity.py tests/test_gpu_configs.py} -m gpu -x -q \
    --timeout 300 --timeout-method thread > gpurun_out/pytest_${TAG}.log 2>&1 || { tail -30 gpurun_out/pytest_${TAG}.log; exit 1; }
tail -2 gpurun_out/pytest_${TAG}.log
timeout -k 10 400 python3 bench.py --steps 20 --warmup 5 --cpu-baseline off > gpurun_out/bench_${TAG}.json 2> gpurun_out/bench_${TAG}.err \
    || { tail -5 gpurun_out/bench_${TAG}.err; exit 1; }
tail -1 gpurun_out/bench_${TAG}.err
python3 -c "
import json; d=json.loads(open('gpurun_out/bench_${TAG}.json').read().strip().splitlines()[-1])
print('value', d['value']/1e9, 'ms/step', d['ms_per_step'], 'k1 ms', d['roofline']['avg_launch_ms'], 'frac', d['roofline']['frac'], 'fixture', (d.get('fixture') or {}).get('match'), d.get('invalid'))"
