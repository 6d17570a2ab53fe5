mkdir -p gpurun_out; export TMPDIR=/tmp
PM_DUMP_MAPS=1 timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/rpa -o run -- python3 -u bench.py --scale 20 --p-gen 4 --steps 2 --warmup 1 --cpu-baseline off > gpurun_out/rpa.json 2> gpurun_out/rpa.log; echo "a rc=$?"; ls gpurun_out/rpa | head -3
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/rpb -o run -- python3 -u tools/k1_harness.py 20 4 2 > gpurun_out/rpb.log 2>&1; echo "b rc=$?"; ls gpurun_out/rpb | head -3

timeout -k 10 400 python3 -u tools/rccl_probe.py > gpurun_out/rccl_probe.log 2>&1; echo "rccl rc=$?"; cat gpurun_out/rccl_probe.log
exit 0
