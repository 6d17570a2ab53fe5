mkdir -p gpurun_out
timeout -k 10 300 python -u tools/ubench.py 28 8 0,1,8,2,4 > gpurun_out/ubench28.log 2>&1; rc=$?; cat gpurun_out/ubench28.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u -m pytest tests/test_gpu_configs.py -m gpu -x -v -s --timeout 380 --timeout-method thread -p no:cacheprovider -k c5 > gpurun_out/pytest_c5.log 2>&1; rc=$?; tail -6 gpurun_out/pytest_c5.log; [ $rc -eq 0 ] || exit $rc
PM_BIG=1 timeout -k 10 600 python -u -m pytest tests/test_gpu_configs.py -m gpu -x -v -s --timeout 580 --timeout-method thread -p no:cacheprovider -k c4 > gpurun_out/pytest_c4.log 2>&1; rc=$?; tail -8 gpurun_out/pytest_c4.log; exit $rc
