set -o pipefail
mkdir -p gpurun_out
PM_HOST_PROBES=1 timeout -k 10 300 python3 bench.py --steps 20 --warmup 3 --cpu-baseline off --c3 off --nlcc off --fixture-check off > gpurun_out/probe_bench.json 2> gpurun_out/probe_bench.err || exit 1
tail -4 gpurun_out/probe_bench.err
for s in 22 23 24 25; do
  timeout -k 10 240 python3 tools/nlcc_phase_times.py --scale $s --alphabet 64 > gpurun_out/c5a64_s$s.json 2> gpurun_out/c5a64_s$s.err || { echo "S=$s failed/timeout"; tail -3 gpurun_out/c5a64_s$s.err; exit 0; }
  python3 -c "import json; d=json.loads(open('gpurun_out/c5a64_s$s.json').read().splitlines()[-1]); print($s, d['seconds'], d['lcc_edges']+d['nlcc_edges']+d['tds_edges'], d['walks'])"
done
