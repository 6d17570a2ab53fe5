"""One search sharded over N in-process shards (one GPU), N = 1, 2, 4, 8: every shard's statistics.

pm_run_rmat_local_shards2 generates the R-MAT graph shard by shard on the device (each shard its generator
ranks' streams, the entries routed to their owners), sets the labels, and runs the search `repeats` times;
the shards take turns on the chip (ThreadComm), so each shard's device times are its own work, with no
contention from the others.  Per N the tool records, for every shard: the superstep-0 kernel time, the
device time of the sharded part (search start -> replica hand-off, less the collectives' host time), the
NLC-line device time (split lines: its share of the sources), edges held, collectives and bytes -- and
checks the result directory against the oracle's fixture when one exists (results must not depend on N).

    python3 tools/shard_scaling.py --config c5 --out gpurun_out/shards_c5.json     # S=27, hash-256, 4-cycle
    python3 tools/shard_scaling.py --config c4 --out gpurun_out/shards_c4.json     # S=28, degree, tree
"""
import argparse
import json
import os
import shutil
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))

import fuzzypatternmatching_amd as pm  # noqa: E402
import pmtest  # noqa: E402

CONFIGS = {
    # (scale, P_gen, pattern, labels: None = degree | (alphabet, salt), fixture)
    "c5": (27, 8, "rmat_log2_cycle4_pattern", (256, 5), "rmat_s27_p8_cycle4_hash256.json"),
    "c4": (28, 8, "rmat_log2_tree_pattern", None, "rmat_s28_p8_tree.json"),
    "small": (20, 4, "rmat_log2_cycle4_pattern", (64, 0), None),
}
KEYS = ("seconds", "device_seconds", "lcc_first_kernel_ms", "shard_sharded_ms", "nlcc_seconds", "split_lines",
        "line_overflows", "exact_lines", "shard_entries", "shard_rows", "shard_hub_entries", "shard_hubs_controlled",
        "shard_ss0_entries", "shard_ss0_survivors", "comm_calls", "comm_bytes", "comm_seconds", "replica_rows",
        "replica_entries")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", choices=sorted(CONFIGS), default="c5")
    ap.add_argument("--shards", type=int, nargs="+", default=[1, 2, 4, 8])
    ap.add_argument("--repeats", type=int, default=3)
    ap.add_argument("--split-min", type=int, default=None, help="PM_SPLIT_LINES (first-position tokens)")
    ap.add_argument("--handoff", type=int, default=None, help="PM_HANDOFF (superstep of the replica hand-off)")
    ap.add_argument("--out", default=None)
    args = ap.parse_args()
    if args.split_min is not None:
        os.environ["PM_SPLIT_LINES"] = str(args.split_min)
    if args.handoff is not None:
        os.environ["PM_HANDOFF"] = str(args.handoff)
    scale, p_gen, pattern, lab, fixture = CONFIGS[args.config]
    pdir = os.path.join(ROOT, "patterns", pattern)
    labels = None if lab is None else pmtest.hash_labels(1 << scale, lab[0], salt=lab[1])
    fx = json.load(open(os.path.join(ROOT, "tests", "golden", fixture))) if fixture else None
    out = {"config": args.config, "scale": scale, "p_gen": p_gen, "pattern": pattern,
           "labels": "degree" if lab is None else f"hash32(v ^ {lab[1]}) % {lab[0]}", "repeats": args.repeats,
           "split_min": os.environ.get("PM_SPLIT_LINES"), "handoff": os.environ.get("PM_HANDOFF"), "runs": {}}
    for n in args.shards:
        td = tempfile.mkdtemp(prefix="pmshards")
        t0 = time.time()
        each = pm.run_rmat_local_shards_each(scale, p_gen, pdir, n, td, max_iterations=64, labels=labels,
                                             repeats=args.repeats)
        wall = time.time() - t0
        run = {"wall_s_incl_generation": round(wall, 2), "per_shard": {k: [s[k] for s in each] for k in KEYS},
               "result": {k: each[0][k] for k in ("iterations", "lcc_edges", "nlcc_edges", "tds_edges", "walks",
                                                  "final_vertices", "final_edges", "hubs")}}
        if fx:
            diffs = pmtest.digest_diffs(fx["digest"], pmtest.result_digest(td, fx["nranks"]))
            for k_g, k_o in (("final_vertices", "final_vertices"), ("final_edges", "final_edges"),
                             ("lcc_edges", "lcc_edges"), ("nlcc_edges", "nlcc_edges"), ("tds_edges", "tds_edges"),
                             ("walks", "paths")):
                if each[0][k_g] != fx["stats"][k_o]:
                    diffs.append(f"{k_g}: {each[0][k_g]} != {fx['stats'][k_o]}")
            run["fixture_match"] = not diffs
            run["fixture_diffs"] = diffs[:4]
        shutil.rmtree(td, ignore_errors=True)
        ps = run["per_shard"]
        print(f"N={n}: lcc_first max {max(ps['lcc_first_kernel_ms']):.3f} ms, sharded part max "
              f"{max(ps['shard_sharded_ms']):.3f} ms, lines max {max(ps['nlcc_seconds']) * 1e3:.3f} ms "
              f"(split {ps['split_lines'][0]}), device {max(ps['device_seconds']) * 1e3:.3f} ms, "
              f"fixture {run.get('fixture_match')}", file=sys.stderr, flush=True)
        out["runs"][str(n)] = run
    s = json.dumps(out)
    if args.out:
        with open(args.out, "w") as f:
            f.write(s + "\n")
    print(s)


if __name__ == "__main__":
    main()
