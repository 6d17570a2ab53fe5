timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_directed.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_ms.log 2>&1; echo "pytest rc=$?"; tail -2 gpurun_out/pytest_ms.log
TAG=trace_ms bash tools/gpu_trace_step.sh || exit 1
for sl in 16384 1024 64 0; do
  PM_SMALL_LINE=$sl PM_PHASE_TIMES=1 timeout -k 10 300 python3 -u bench.py --cpu-baseline off --steps 3 --warmup 1 > gpurun_out/phase_$sl.json 2> gpurun_out/phase_$sl.log || exit 1
  echo "small_line=$sl"; grep "line 4:" gpurun_out/phase_$sl.log | tail -1; python3 -c "import json;print(json.load(open('gpurun_out/phase_$sl.json'))['ms_per_step'])"
done
