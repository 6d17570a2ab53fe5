# GPU box: superstep-0 variants (head vs working tree), the gather floor of the first later superstep with its
# FETCH_SIZE / L2 passes, and the S=28 line phase times.
mkdir -p gpurun_out && export TMPDIR=/tmp && \
PM_LIB=fuzzypatternmatching_amd/lib/libpm_head_diag.so timeout -k 10 200 python3 -u tools/ubench.py 28 8 0,5 > gpurun_out/ub_head.txt 2>&1 && \
PM_LIB=fuzzypatternmatching_amd/lib/libpm_diag.so timeout -k 10 300 python3 -u tools/ubench.py 28 8 0,13,21,25,29,33,37 > gpurun_out/ub_nt.txt 2>&1 && \
timeout -k 10 300 python3 -u tools/gather_floor.py 28 8 > gpurun_out/gf.json 2> gpurun_out/gf.err && \
GF_ROUNDS=1 timeout -s KILL 200 rocprofv3 --kernel-trace --pmc FETCH_SIZE --kernel-include-regex "k_gather_floor" --output-format csv -d gpurun_out/pmc_gf1 -o run -- python3 tools/gather_floor.py 28 8 > gpurun_out/pmc_gf1.log 2>&1 && \
GF_ROUNDS=1 timeout -s KILL 200 rocprofv3 --kernel-trace --pmc TCC_HIT_sum TCC_MISS_sum --kernel-include-regex "k_gather_floor" --output-format csv -d gpurun_out/pmc_gf2 -o run -- python3 tools/gather_floor.py 28 8 > gpurun_out/pmc_gf2.log 2>&1 && \
PM_PHASE_TIMES=1 timeout -k 10 200 python3 bench.py --steps 2 --warmup 1 --cpu-baseline off --fixture-check off --c3 off --nlcc off --sharded-n1 off > gpurun_out/tds_pos.json 2> gpurun_out/tds_pos.err
rc=$?; grep -A1 "line 4" gpurun_out/tds_pos.err | tail -4; tail -3 gpurun_out/ub_head.txt; tail -9 gpurun_out/ub_nt.txt; cat gpurun_out/gf.json; exit $rc
