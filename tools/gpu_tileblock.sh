#!/bin/bash
mkdir -p gpurun_out
for lib in libpm_diag libpm_tb8 libpm_tb16 libpm_diag; do
  PM_LIB=fuzzypatternmatching_amd/lib/$lib.so timeout -k 10 200 python3 tools/k1_variants.py 28 8 0 0 > gpurun_out/tb_$lib.log 2>&1 || exit 1
  echo "$lib: $(grep variant gpurun_out/tb_$lib.log | tr '\n' ' ')"
done
