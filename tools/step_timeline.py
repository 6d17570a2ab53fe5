"""Per-step kernel timeline of a rocprofv3 --kernel-trace run of bench.py.

usage: step_timeline.py TRACE_DIR  (the last complete step: from the last but one
k_lcc_first launch to the last one)
"""
import csv
import glob
import sys

rows = []
for f in glob.glob(sys.argv[1] + "/**/*kernel_trace.csv", recursive=True):
    rows += list(csv.DictReader(open(f)))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
idx = [i for i, r in enumerate(rows) if "k_lcc_first" in r["Kernel_Name"]]
i0, i1 = idx[-2], idx[-1]
t0 = int(rows[i0]["Start_Timestamp"])
for r in rows[i0:i1]:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    print(f"{(s - t0) / 1e3:9.1f} {(e - s) / 1e3:8.1f}  {r['Kernel_Name'][:100]}")
print(f"step: {(int(rows[i1]['Start_Timestamp']) - t0) / 1e3:.1f} us")
