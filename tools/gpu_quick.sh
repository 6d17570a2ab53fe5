# Parity subset (one-GPU parity, directed, C2 at S=24) then the default bench line
mkdir -p gpurun_out
TAG=${TAG:-quick}
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_directed.py tests/test_gpu_configs.py -k "not c3 and not c5 and not c4" -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_$TAG.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_$TAG.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 -u bench.py --cpu-baseline off ${BENCH_ARGS:-} > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.log
rc=$?; echo "bench rc=$rc"; cat gpurun_out/bench_$TAG.json; tail -1 gpurun_out/bench_$TAG.log; exit $rc
