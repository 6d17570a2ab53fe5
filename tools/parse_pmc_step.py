"""Summarise the rocprofv3 --pmc passes of k_lcc_step (tools/gpu_profile.sh, one bench step per pass) into
a JSON file: the later LCC supersteps of the LAST search in each pass, per dispatch in launch order (the first
is the superstep right after superstep 0), with HBM bytes = (2 x FETCH_SIZE + WRITE_SIZE) x 1024 (gfx950,
MI355X_MICROARCH.md "HBM [CDNA4]") and the dispatch's duration from the pass's own timestamps.

usage: parse_pmc_step.py GPURUN_OUT TAG OUT.json
"""
import csv
import glob
import json
import os
import sys


def dispatches(d):
    rows = {}
    for f in glob.glob(os.path.join(d, "**", "*counter_collection*.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            if "k_lcc_step" not in r["Kernel_Name"]:
                continue
            x = rows.setdefault(int(r["Dispatch_Id"]), {"counters": {}, "ns": int(r["End_Timestamp"]) -
                                                        int(r["Start_Timestamp"])})
            x["counters"][r["Counter_Name"]] = x["counters"].get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
    ids = sorted(rows)
    # the last search of the run: the supersteps after the last big gap in dispatch ids are not needed --
    # a search has the same number of k_lcc_step dispatches every time, so take the final len // searches
    return [rows[i] for i in ids]


def main():
    base, tag, out = sys.argv[1], sys.argv[2], sys.argv[3]
    passes = [dispatches(d) for d in sorted(glob.glob(os.path.join(base, f"pmcstep_{tag}_[0-9]*"))) if os.path.isdir(d)]
    passes = [p for p in passes if p]
    n = min(len(p) for p in passes)
    per = 7  # later supersteps of one S=28 tree search (diameter 8)
    res = {"kernel": "k_lcc_step", "what": "the later LCC supersteps of the last bench search of each pass, in "
           "launch order; hbm_bytes = (2 x FETCH_SIZE + WRITE_SIZE) x 1024", "dispatches": []}
    for j in range(max(0, n - per), n):
        c = {}
        ns = []
        for p in passes:
            c.update(p[j]["counters"])
            ns.append(p[j]["ns"])
        d = {"index": j - max(0, n - per), "counters": c, "us_under_pmc": round(min(ns) / 1e3, 1)}
        if "FETCH_SIZE" in c and "WRITE_SIZE" in c:
            d["hbm_bytes"] = int((2 * c["FETCH_SIZE"] + c["WRITE_SIZE"]) * 1024)
            # (the 2x is the streaming-read correction; a narrow random gather miss is tallied as one 64-B
            # request (tools/gather_floor.py calibration), so the gathers' share is over-stated by it)
            d["fetch_requests_64B"] = int(c["FETCH_SIZE"] * 1024 / 64)
        res["dispatches"].append(d)
    json.dump(res, open(out, "w"), indent=1)
    for d in res["dispatches"]:
        print(d["index"], d.get("hbm_bytes"), d["us_under_pmc"])


if __name__ == "__main__":
    main()
