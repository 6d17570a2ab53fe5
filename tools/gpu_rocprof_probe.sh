# rocprofv3 exit behaviour of one search through the library (tools/rp_exit.py MODE);
# a fatal signal prints a native backtrace into the log.  Modes chained with &&.
mkdir -p gpurun_out; export TMPDIR=/tmp
run() {
  timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/rp_$1 -o run -- \
    python3 -u tools/rp_exit.py $1 > gpurun_out/rp_$1.log 2>&1
  rc=$?; echo "$1 rc=$rc"; return $rc
}
run ${1:-beta} && run ${2:-lcc}
