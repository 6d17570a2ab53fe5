"""Config C5's search with small alphabets, measured on the GPU (verdict r5 item 8: the 256-letter choice rested
on an extrapolation of the oracle's S=20-22 counts).  For each alphabet and scale: the S-scale R-MAT graph
(P_gen = 8, GPU generator), labels hash32(v ^ 5) % alphabet, the 4-cycle pattern (4 cycle-check lines + the TDS
line), one complete search without result files; then (if the search took at most a third of --budget) the
same search with the TDS enumeration capped at --cap walks per level chunk (the exact path's chunked
enumeration), whose counters must be identical (chunk invariance).  Where the search traversed at most
--oracle-edges edges the oracle runs it too and its counters must match.  One JSON line per (alphabet, scale)
on stdout; a search past --budget seconds ends the alphabet's sweep, and the whole sweep stops once
--total-budget seconds have passed.

usage: python3 tools/c5_alphabet_growth.py [--alphabets 64 8] [--scales 12 ... 27] [--cap 1048576]
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
sys.path.insert(0, os.path.join(ROOT, "oracle"))

import fuzzypatternmatching_amd as pm  # noqa: E402
import pmtest  # noqa: E402

KEYS = ("iterations", "terminated", "final_vertices", "final_edges", "lcc_edges", "nlcc_edges", "tds_edges", "walks")


def heartbeat():
    import threading

    def beat():
        t0 = time.time()
        while True:
            time.sleep(30)
            print(f"[c5 growth] {time.time() - t0:.0f}s", file=sys.stderr, flush=True)
    threading.Thread(target=beat, daemon=True).start()


def watched(fn, limit, what):
    """fn() with a watchdog: past `limit` seconds a line says so and the process exits (status 5)."""
    import threading
    done = threading.Event()

    def dog():
        if not done.wait(limit):
            print(json.dumps(dict(what, skipped=f"search still running after {limit:.0f} s")), flush=True)
            os._exit(5)
    threading.Thread(target=dog, daemon=True).start()
    try:
        return fn()
    finally:
        done.set()


def main():
    heartbeat()
    ap = argparse.ArgumentParser()
    ap.add_argument("--alphabets", type=int, nargs="+", default=[64, 8])
    ap.add_argument("--scales", type=int, nargs="+", default=list(range(12, 28)))
    ap.add_argument("--cap", type=int, default=1 << 20)
    ap.add_argument("--budget", type=float, default=150.0, help="seconds of one search beyond which the sweep stops")
    ap.add_argument("--oracle-edges", type=float, default=2e9, help="the oracle checks searches up to this many edges")
    ap.add_argument("--total-budget", type=float, default=700.0)
    ap.add_argument("--p-gen", type=int, default=8)
    ap.add_argument("--no-capped", action="store_true", help="skip the capped rerun (timing runs)")
    ap.add_argument("--search-limit", type=float, default=400.0,
                    help="a search still running after this many seconds ends the run (one line says so)")
    args = ap.parse_args()
    cyc = os.path.join(ROOT, "patterns", "rmat_log2_cycle4_pattern")
    t_start = time.time()
    for alphabet in args.alphabets:
        prev = None
        for scale in args.scales:
            if time.time() - t_start > args.total_budget:
                print(json.dumps({"alphabet": alphabet, "scale": scale, "skipped": "total budget spent"}), flush=True)
                return
            m, gen_s = pm.rmat_matcher(scale, args.p_gen, cyc, device=0)
            m.set_labels(pmtest.hash_labels(1 << scale, alphabet, salt=5))
            t0 = time.perf_counter()
            a = watched(lambda: m.run_beta("", 64), args.search_limit, {"alphabet": alphabet, "scale": scale})
            ta = time.perf_counter() - t0
            b, tb = None, None
            if ta <= args.budget / 3 and not args.no_capped:
                os.environ["PM_TDS_CAP"] = str(args.cap)
                t0 = time.perf_counter()
                b = m.run_beta("", 64)
                tb = time.perf_counter() - t0
                del os.environ["PM_TDS_CAP"]
            m.close()
            edges = a["lcc_edges"] + a["nlcc_edges"] + a["tds_edges"]
            row = {"alphabet": alphabet, "scale": scale, "seconds": round(ta, 3), "edges": edges,
                   "edges_per_s": round(edges / ta, 1), "walks": a["walks"], "tds_edges": a["tds_edges"],
                   "path_cycle_edges": a["nlcc_edges"], "lcc_edges": a["lcc_edges"],
                   "final_vertices": a["final_vertices"], "exact_lines": a["exact_lines"],
                   "line_overflows": a["line_overflows"], "path_batches": a["path_batches"],
                   "split_lines": a["split_lines"], "tds_chunks": a["tds_chunks"],
                   "gen_s": round(gen_s, 3)}
            if b is not None:
                row.update({"capped_seconds": round(tb, 3), "capped_tds_chunks": b["tds_chunks"],
                            "cap_invariant": all(a[k] == b[k] for k in KEYS)})
            if edges <= args.oracle_edges:
                import oracle
                t0 = time.perf_counter()
                g = pm.rmat_graph(scale, args.p_gen, device=0)
                so = oracle.run(g.off, g.col, cyc, None, labels=pmtest.hash_labels(g.n, alphabet, salt=5),
                                max_iterations=64, threads=oracle.default_threads())
                row["oracle_match"] = all(a[k] == so["paths" if k == "walks" else k] for k in KEYS)
                row["oracle_seconds"] = round(time.perf_counter() - t0, 2)
            # the next scale's search, predicted from this scale's growth, past twice the budget: the sweep ends
            nxt = ta * (ta / prev) if prev and ta > 1.0 else 0.0
            row["next_scale_predicted_s"] = round(nxt, 1)
            print(json.dumps(row), flush=True)
            prev = ta
            if ta > args.budget or nxt > 2 * args.budget:
                break


if __name__ == "__main__":
    main()
