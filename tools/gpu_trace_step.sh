# Kernel trace of the default bench (2 warm-up + 2 timed steps) for a per-step breakdown
mkdir -p gpurun_out; export TMPDIR=/tmp
TAG=${TAG:-trace}
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/$TAG -o run -- \
  python3 -u bench.py --cpu-baseline off --steps 2 --warmup 2 ${BENCH_ARGS:-} > gpurun_out/$TAG.json 2> gpurun_out/$TAG.log
rc=$?; echo "trace rc=$rc"; cat gpurun_out/$TAG.json; exit $rc
