"""Per-kernel breakdown of the last search step in a rocprofv3 kernel trace
(tools/gpu_trace_step.sh): kernels from the last k_lcc_first launch on, with
the gaps between them.

usage: step_breakdown.py TRACE_DIR [N_AFTER]
"""
import csv
import glob
import sys

f = glob.glob(sys.argv[1] + "/**/*kernel_trace.csv", recursive=True)[0]
rows = sorted(csv.DictReader(open(f)), key=lambda r: int(r["Start_Timestamp"]))
first = [i for i, r in enumerate(rows) if "k_lcc_first" in r["Kernel_Name"]][-1]
n_after = int(sys.argv[2]) if len(sys.argv) > 2 else 60
prev = None
tot = 0.0
for r in rows[first:first + n_after]:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    gap = (s - prev) / 1000 if prev else 0.0
    prev = e
    tot += (e - s) / 1000
    name = r["Kernel_Name"].split("(")[0].replace("void ", "")[-48:]
    print(f"{name:48s} {(e - s) / 1000:9.1f} us  gap {gap:7.1f} us  grid {r['Grid_Size_X']}")
print(f"kernel time {tot:.1f} us over {len(rows[first:first + n_after])} launches")
