"""Split NLC lines, strong scaling of the token passing over in-process shards (one GPU).

BASELINE config C3 (R-MAT S=26, P_gen=4, the 4-cycle pattern: the NLCC stress) searched by
pm_run_rmat_local_shards with N = 1, 2, 4 shards driven by threads of this process on one device: the shards
take turns on the chip, so shard 0's NLC-line device time (pm_run_stats.nlcc_seconds) is the time of its
1/N of the sources.  Prints one JSON line: per N the shard-0 line time, lines run split, and the result
counters (which must not depend on N).

usage: python3 tools/split_lines_scaling.py [--scale 26] [--p-gen 4] [--shards 1 2 4] [--out FILE]
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import fuzzypatternmatching_amd as pm  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--scale", type=int, default=26)
    ap.add_argument("--p-gen", type=int, default=4)
    ap.add_argument("--pattern", default="rmat_log2_cycle4_pattern")
    ap.add_argument("--shards", type=int, nargs="+", default=[1, 2, 4])
    ap.add_argument("--out", default=None)
    args = ap.parse_args()
    pattern = os.path.join(ROOT, "patterns", args.pattern)
    res = {"what": f"R-MAT S={args.scale} P_gen={args.p_gen} {args.pattern}, N in-process shards on one GPU: "
                   "shard 0's NLC-line device time (its 1/N of the split lines' sources)", "runs": []}
    keys = ("iterations", "lcc_edges", "nlcc_edges", "tds_edges", "walks", "final_vertices", "final_edges")
    ref = None
    for n in args.shards:
        t = time.time()
        st = pm.run_rmat_local_shards(args.scale, args.p_gen, pattern, n, "", max_iterations=64)
        row = {"shards": n, "shard0_nlcc_ms": round(st["nlcc_seconds"] * 1e3, 3),
               "shard0_search_ms": round(st["seconds"] * 1e3, 3), "split_lines": st["split_lines"],
               "wall_s": round(time.time() - t, 2)}
        row.update({k: st[k] for k in keys})
        if ref is None:
            ref = {k: st[k] for k in keys}
        row["same_result_as_first"] = all(st[k] == ref[k] for k in keys)
        res["runs"].append(row)
        print(json.dumps(row), file=sys.stderr, flush=True)
    line = json.dumps(res)
    print(line)
    if args.out:
        with open(args.out, "w") as f:
            f.write(line + "\n")
    return 0 if all(r["same_result_as_first"] for r in res["runs"]) else 3


if __name__ == "__main__":
    sys.exit(main())
