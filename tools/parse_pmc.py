"""Summarise rocprofv3 --pmc passes of k_lcc_first into profiles/<round>_pmc_lcc_first.json.

HBM bytes per launch follow MI355X_MICROARCH.md section HBM / cdna_hip_programming.md 7:
FETCH_SIZE and WRITE_SIZE are in KiB; on gfx950 FETCH_SIZE counts 64 B per
TCC_EA0_RDREQ, i.e. half of a 128-B request, so reads are doubled:
    hbm_bytes = (2 * FETCH_SIZE + WRITE_SIZE) * 1024
(the doc calls the x2 exact for 16-B-per-lane streams and uncalibrated for
other widths; both raw and corrected values are recorded).
"""
import csv
import glob
import json
import os
import sys


def counters(d):
    out = {}
    for f in glob.glob(os.path.join(d, "**", "*counter_collection*.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            name = r.get("Counter_Name")
            val = float(r.get("Counter_Value", 0))
            disp = r.get("Dispatch_Id")
            out.setdefault(name, {}).setdefault(disp, 0.0)
            out[name][disp] += val
    return {k: sum(v.values()) / max(1, len(v)) for k, v in out.items()}


def main():
    base, tag, scale = sys.argv[1], sys.argv[2], int(sys.argv[3])
    vals = {}
    for i in (1, 2, 3):
        vals.update(counters(os.path.join(base, f"{tag}_{i}")))
    fetch = vals.get("FETCH_SIZE")
    write = vals.get("WRITE_SIZE")
    res = {"kernel": "k_lcc_first", "scale": scale, "p_gen": 4, "pattern": "rmat_log2_tree_pattern",
           "fetch_size_kib": fetch, "write_size_kib": write,
           "tcc_hit": vals.get("TCC_HIT_sum"), "tcc_miss": vals.get("TCC_MISS_sum")}
    if fetch is not None and write is not None:
        res["hbm_bytes_per_launch"] = int((2 * fetch + write) * 1024)
        res["hbm_bytes_per_launch_raw"] = int((fetch + write) * 1024)
    if res["tcc_hit"] is not None and res["tcc_miss"]:
        res["l2_hit_rate"] = res["tcc_hit"] / (res["tcc_hit"] + res["tcc_miss"])
    os.makedirs("profiles", exist_ok=True)
    out = os.path.join(base, f"{tag}_summary.json")
    json.dump(res, open(out, "w"), indent=1)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
