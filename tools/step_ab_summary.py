"""Last-step timelines of several rocprofv3 --kernel-trace runs of bench.py side by side (tools/gpu_step_ablation.sh
output dirs): per run the step length and the durations of the LCC kernels in launch order.

usage: step_ab_summary.py DIR [DIR ...]
"""
import csv
import glob
import os
import sys

for d in sys.argv[1:]:
    rows = []
    for f in glob.glob(d + "/**/*kernel_trace.csv", recursive=True):
        rows += list(csv.DictReader(open(f)))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    idx = [i for i, r in enumerate(rows) if "k_lcc_first" in r["Kernel_Name"]]
    if len(idx) < 2:
        print(os.path.basename(d), "no complete step")
        continue
    i0, i1 = idx[-2], idx[-1]
    t0 = int(rows[i0]["Start_Timestamp"])
    seq = []
    for r in rows[i0:i1]:
        n = r["Kernel_Name"]
        short = ("step" if "k_lcc_step<" in n else "pieces" if "k_lcc_step_pieces" in n else "pack" if "k_long_pack" in n
                 else "first" if "k_lcc_first" in n else "lines" if "k_lines" in n else None)
        if short:
            seq.append(f"{short}:{(int(r['End_Timestamp']) - int(r['Start_Timestamp'])) / 1e3:.0f}")
    print(f"{os.path.basename(d):28s} step {(int(rows[i1]['Start_Timestamp']) - t0) / 1e3:7.1f} us  " + " ".join(seq))
