"""Durations of the first later superstep (the first k_lcc_step dispatch after each k_lcc_first) and of
k_lcc_first in rocprofv3 kernel-trace directories.  usage: step_first_dispatch.py DIR [DIR ...]"""
import csv
import glob
import os
import statistics
import sys

for d in sys.argv[1:]:
    files = glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True)
    if not files:
        continue
    rows = []
    for f in files:
        rows += list(csv.DictReader(open(f)))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    first, step = [], []
    after = False
    for r in rows:
        name = r["Kernel_Name"]
        dur = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
        if "k_lcc_first" in name:
            first.append(dur)
            after = True
        elif "k_lcc_step" in name and after:
            step.append(dur)
            after = False
    if step:
        print(f"{os.path.basename(d)}: first later superstep median {statistics.median(step):.1f} us "
              f"(n={len(step)}, {', '.join(f'{x:.0f}' for x in step)}); k_lcc_first median {statistics.median(first):.1f} us")
