#!/bin/bash
# GPU box: kernel traces of one C5-shaped search (S=27 hash-256 4-cycle, tools/nlcc_phase_times.py) with the
# product library and the builds named in LIBS, and the k_lcc_step dispatch durations of each, side by side.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp PM_LINES_NOCOOP=1
for L in libpm.so ${LIBS:-}; do
  PM_LIB=fuzzypatternmatching_amd/lib/$L timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/c5ab_$L -o run -- \
    python3 tools/nlcc_phase_times.py --repeat 2 > gpurun_out/c5ab_$L.json 2> gpurun_out/c5ab_$L.log || { tail -5 gpurun_out/c5ab_$L.log; exit 1; }
done
python3 - <<'PY'
import csv, glob, os
for d in sorted(glob.glob("gpurun_out/c5ab_*/")):
    rows = []
    for f in glob.glob(d + "**/*kernel_trace.csv", recursive=True):
        rows += list(csv.DictReader(open(f)))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    tot = {}
    seq = []
    for r in rows:
        n = r["Kernel_Name"].split("(")[0][-40:]
        dur = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
        tot[n] = tot.get(n, 0) + dur
        if "k_lcc_step" in n:
            seq.append(round(dur))
    top = sorted(tot.items(), key=lambda x: -x[1])[:16]
    print(os.path.basename(d.rstrip("/")), "k_lcc_step:", seq)
    print("   top:", [(k, round(v)) for k, v in top])
PY
