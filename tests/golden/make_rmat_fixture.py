#!/usr/bin/env python3
"""Makes an R-MAT result fixture with the ORACLE (test infrastructure, never the product).

    python tests/golden/make_rmat_fixture.py --scale 28 --p-gen 8 --pattern rmat_log2_tree_pattern \
        --out gpurun_out/rmat_s28_p8_tree.json

Runs oracle/pm_oracle.cpp (the CPU restatement, all host threads) on the R-MAT graph of
generate_rmat.cpp with P_gen generator ranks (src/generate_rmat.cpp:202-213), degree labels,
and writes pmtest.result_digest() of its result directory (count files, sorted-line-set sha256
of the active vertex / edge / subgraph files; run_pattern_matching_beta.cpp:1370-1425) plus its
counters and timings.  The graph comes from the GPU generator (pm_rmat.hip, bit-identical to the
oracle's own generator: tests/test_gpu_rmat.py), copied to the host; at S=28 the oracle needs
about 100 GB of host memory, so this runs on the GPU box, once.  The committed fixture is
tests/golden/rmat_s<S>_p<P>_<pattern>.json; tests/test_gpu_configs.py and bench.py check the
GPU search against it.
"""
import argparse
import json
import os
import shutil
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
for p in (ROOT, os.path.join(ROOT, "oracle"), os.path.join(ROOT, "tests")):
    sys.path.insert(0, p)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--scale", type=int, required=True)
    ap.add_argument("--p-gen", type=int, required=True)
    ap.add_argument("--pattern", default="rmat_log2_tree_pattern")
    ap.add_argument("--nranks", type=int, default=1)
    ap.add_argument("--labels", default="degree",
                    help="degree (vertex_data_db_degree) or hash:<alphabet>:<salt> (pmtest.hash_labels: config C5's "
                         "explicit labels hash32(v ^ salt) % alphabet)")
    ap.add_argument("--timing-runs", type=int, default=2, help="extra oracle runs without result files (baseline)")
    ap.add_argument("--max-iterations", type=int, default=64)
    ap.add_argument("--out", required=True)
    a = ap.parse_args()

    import fuzzypatternmatching_amd as pm
    import oracle
    import pmtest

    import threading
    t_start = time.time()

    def beat():  # the GPU runner takes a silent command for a hung one
        while True:
            time.sleep(30)
            print(f"[heartbeat {time.time() - t_start:.0f}s]", flush=True)

    threading.Thread(target=beat, daemon=True).start()
    pattern = os.path.join(ROOT, "patterns", a.pattern)
    t0 = time.time()
    g = pm.rmat_graph(a.scale, a.p_gen, device=0)
    print(f"graph S={a.scale} P_gen={a.p_gen}: V={g.n} E={g.nnz} in {time.time() - t0:.1f}s", flush=True)
    labels = None
    if a.labels != "degree":
        kind, alphabet, salt = a.labels.split(":")
        assert kind == "hash"
        labels = pmtest.hash_labels(g.n, int(alphabet), salt=int(salt))
    threads = oracle.default_threads()
    td = tempfile.mkdtemp(prefix="pmfix")
    try:
        rd = os.path.join(td, "oracle")
        t0 = time.time()
        st = oracle.run(g.off, g.col, pattern, rd, labels=labels, nranks=a.nranks, max_iterations=a.max_iterations,
                        threads=threads)
        print(f"oracle run with result files: {st['seconds']:.2f}s search, {time.time() - t0:.1f}s total", flush=True)
        dig = pmtest.result_digest(rd, a.nranks)
        secs = [st["seconds"]]
        for i in range(a.timing_runs):
            s2 = oracle.run(g.off, g.col, pattern, None, labels=labels, nranks=a.nranks,
                            max_iterations=a.max_iterations, threads=threads)
            secs.append(s2["seconds"])
            assert s2["lcc_edges"] == st["lcc_edges"] and s2["final_vertices"] == st["final_vertices"]
            print(f"oracle timing run {i}: {s2['seconds']:.2f}s", flush=True)
    finally:
        shutil.rmtree(td, ignore_errors=True)
    edges = st["lcc_edges"] + st["nlcc_edges"] + st["tds_edges"]
    med = sorted(secs)[len(secs) // 2]
    out = {
        "what": f"oracle result digest: R-MAT S={a.scale} P_gen={a.p_gen}, {a.labels} labels, {a.pattern}, "
                f"nranks={a.nranks} (tests/golden/make_rmat_fixture.py)",
        "scale": a.scale, "p_gen": a.p_gen, "pattern": a.pattern, "nranks": a.nranks, "labels": a.labels,
        "vertices": g.n, "directed_entries": g.nnz,
        "stats": {k: st[k] for k in ("iterations", "terminated", "lcc_edges", "nlcc_edges", "tds_edges", "paths",
                                     "final_vertices", "final_edges", "lcc_calls", "supersteps")},
        "digest": dig,
        "oracle_timing": {"threads": threads, "seconds": [round(x, 3) for x in secs], "median_s": round(med, 3),
                          "edges_per_s": round(edges / med, 1), "host_cpus": os.cpu_count()},
    }
    os.makedirs(os.path.dirname(os.path.abspath(a.out)), exist_ok=True)
    with open(a.out, "w") as f:
        json.dump(out, f, indent=1)
    print(json.dumps(out["stats"]), flush=True)
    print(json.dumps(out["oracle_timing"]), flush=True)


if __name__ == "__main__":
    main()
