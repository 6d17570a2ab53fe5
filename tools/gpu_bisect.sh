mkdir -p gpurun_out
for v in HEAD KEEP STORE WPE; do
  if [ $v = HEAD ]; then L=""; else L=alt/libpm_$v.so; fi
  PM_LIB=$L timeout -k 10 200 python3 -u bench.py --cpu-baseline off --steps 1 --warmup 0 > gpurun_out/bis_$v.json 2> gpurun_out/bis_$v.log || exit 1
  echo "$v: $(grep -o 'final |S|=[0-9]* |M|=[0-9]*' gpurun_out/bis_$v.log)"
done
