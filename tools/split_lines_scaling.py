"""Split NLC lines, strong scaling of the token passing over in-process shards (one GPU).

An R-MAT graph (default S=22, P_gen=4) with hash labels (default alphabet 64: the C5 label shape, whose NLC
lines have tens of thousands of sources -- with the degree labels of C3 the lines find a few thousand and none
is split) and the 4-cycle pattern, searched by pm_run_beta_local_shards with N = 1, 2, 4 shards driven by
threads of this process on one device: the shards take turns on the chip, so shard 0's NLC-line device time
(pm_run_stats.nlcc_seconds) is the time of its 1/N of the sources.  --labels degree runs the generated graph
with its degree labels (pm_run_rmat_local_shards).  Prints one JSON line: per N the shard-0 line time, lines
run split, and the result counters (which must not depend on N).

usage: python3 tools/split_lines_scaling.py [--scale 22] [--p-gen 4] [--labels hash|degree] [--alphabet 64]
                                            [--shards 1 2 4] [--split-min N] [--out FILE]
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))

import fuzzypatternmatching_amd as pm  # noqa: E402
import pmtest  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--scale", type=int, default=22)
    ap.add_argument("--labels", choices=["hash", "degree"], default="hash")
    ap.add_argument("--alphabet", type=int, default=64)
    ap.add_argument("--p-gen", type=int, default=4)
    ap.add_argument("--pattern", default="rmat_log2_cycle4_pattern")
    ap.add_argument("--shards", type=int, nargs="+", default=[1, 2, 4])
    ap.add_argument("--split-min", type=int, default=None, help="PM_SPLIT_LINES (source census from which a line splits)")
    ap.add_argument("--out", default=None)
    args = ap.parse_args()
    if args.split_min is not None:
        os.environ["PM_SPLIT_LINES"] = str(args.split_min)
    pattern = os.path.join(ROOT, "patterns", args.pattern)
    lab = f"hash32(v ^ 5) % {args.alphabet} labels" if args.labels == "hash" else "degree-log2 labels"
    res = {"what": f"R-MAT S={args.scale} P_gen={args.p_gen} {lab}, {args.pattern}, N in-process shards on one "
                   "GPU: shard 0's NLC-line device time (its 1/N of the split lines' sources)", "runs": []}
    g = labels = None
    if args.labels == "hash":
        g = pm.rmat_graph(args.scale, args.p_gen, device=0)
        labels = pmtest.hash_labels(g.n, args.alphabet, salt=5)
    keys = ("iterations", "lcc_edges", "nlcc_edges", "tds_edges", "walks", "final_vertices", "final_edges")
    ref = None
    for n in args.shards:
        t = time.time()
        if g is None:
            st = pm.run_rmat_local_shards(args.scale, args.p_gen, pattern, n, "", max_iterations=64)
        else:
            st = pm.run_beta_local_shards(g, pattern, n, "", max_iterations=64, labels=labels)
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
