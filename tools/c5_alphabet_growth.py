"""Config C5's search with small alphabets, measured on the GPU (verdict r5 item 8: the 256-letter choice rested
on an extrapolation of the oracle's S=20-22 counts).  For each alphabet and scale: the S-scale R-MAT graph
(P_gen = 8, GPU generator), labels hash32(v ^ 5) % alphabet, the 4-cycle pattern (4 cycle-check lines + the TDS
line), one complete search without result files; then the same search with the TDS enumeration capped at
--cap walks per level chunk (the exact path's chunked enumeration), whose counters must be identical (chunk
invariance).  At --oracle-max scale and below the oracle runs the same search and its counters must match.
One JSON line per (alphabet, scale) on stdout; a run past --budget seconds ends the alphabet's sweep.

usage: python3 tools/c5_alphabet_growth.py [--alphabets 64 8] [--scales 22 23 24 25 26 27] [--cap 1048576]
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


def main():
    heartbeat()
    ap = argparse.ArgumentParser()
    ap.add_argument("--alphabets", type=int, nargs="+", default=[64, 8])
    ap.add_argument("--scales", type=int, nargs="+", default=[22, 23, 24, 25, 26, 27])
    ap.add_argument("--cap", type=int, default=1 << 20)
    ap.add_argument("--budget", type=float, default=150.0, help="seconds of one search beyond which the sweep stops")
    ap.add_argument("--oracle-max", type=int, default=20)
    ap.add_argument("--p-gen", type=int, default=8)
    args = ap.parse_args()
    cyc = os.path.join(ROOT, "patterns", "rmat_log2_cycle4_pattern")
    for alphabet in args.alphabets:
        for scale in args.scales:
            m, gen_s = pm.rmat_matcher(scale, args.p_gen, cyc, device=0)
            m.set_labels(pmtest.hash_labels(1 << scale, alphabet, salt=5))
            t0 = time.perf_counter()
            a = m.run_beta("", 64)
            ta = time.perf_counter() - t0
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
                   "line_overflows": a["line_overflows"], "capped_seconds": round(tb, 3),
                   "capped_tds_chunks": b["tds_chunks"],
                   "cap_invariant": all(a[k] == b[k] for k in KEYS)}
            if scale <= args.oracle_max:
                import oracle
                g = pm.rmat_graph(scale, args.p_gen, device=0)
                so = oracle.run(g.off, g.col, cyc, None, labels=pmtest.hash_labels(g.n, alphabet, salt=5),
                                max_iterations=64, threads=oracle.default_threads())
                row["oracle_match"] = all(a[k] == so["paths" if k == "walks" else k] for k in KEYS)
            print(json.dumps(row), flush=True)
            if ta > args.budget:
                break


if __name__ == "__main__":
    main()
