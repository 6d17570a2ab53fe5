"""Prints the kernel timeline of the last pattern-search step of a rocprofv3 kernel trace."""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
# last step = from the last k_lcc_first to the end
idx = max(i for i, r in enumerate(rows) if "k_lcc_first" in r["Kernel_Name"])
start = idx
while start > 0 and "fillBuffer" in rows[start - 1]["Kernel_Name"]:
    start -= 1
t0 = int(rows[start]["Start_Timestamp"])
busy = 0
for r in rows[start:]:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    busy += e - s
    print(f"{(s - t0) / 1e3:9.1f} {(e - s) / 1e3:8.2f}  {r['Kernel_Name'][:70]}")
end = int(rows[-1]["End_Timestamp"])
print(f"span {(end - t0) / 1e3:.1f} us, busy {busy / 1e3:.1f} us")
