"""BASELINE config C5 at size on one GPU: an R-MAT text edge list of scale S (default 27, P_gen = 8 files,
written from the GPU generator's stream), ingested on the GPU with -u 1 (ingest_edge_list.cpp:164-240,
parallel_edge_list_reader.hpp:242-266), explicit -v label files (vertex_data_db.hpp:137-257) parsed on the GPU,
and the pattern searched with result files.  Labels: --labels hash (default) writes hash32(v ^ 5) % alphabet
(default 256) as -v files; --labels degree writes the degree-log2 labels of the symmetrized graph.  Pattern:
the 4-cycle (default), whose template-driven enumeration runs in chunks of at most --tds-cap walks per level
(run_tds_line; the reference batches its enumeration, tds_batch_1.hpp:1139-1253).  (With 8 or 64 letters the
4-cycle enumeration at S=27 is ~10^13 edges -- it grows ~6x per scale from the oracle's S=20-22 counts -- for
the reference as for this path; 256 letters keep it tractable.)  Checks:
  * the ingested context's result directory equals the GPU-generated graph's (same labels) -- the text path
    builds the same graph;
  * the same search with a small TDS chunk cap gives the same result directory (chunk-size invariance);
  * with --oracle, both equal the oracle's result on the host CSR (~60 GB of host memory at S=27).
tests/test_gpu_configs.py::test_c5_s27_ingested_label_files runs the same checks in the GPU suite.
Prints one JSON line (ingest GB/s, search time, digests, match flags); progress on stderr.

usage: python3 tools/c5_at_size.py [--scale 27] [--p-gen 8] [--dir /dev/shm/c5] [--oracle] [--out FILE]
"""
import argparse
import ctypes
import json
import os
import shutil
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))
sys.path.insert(0, os.path.join(ROOT, "tests"))

import numpy as np  # noqa: E402

import fuzzypatternmatching_amd as pm  # noqa: E402
from fuzzypatternmatching_amd import _abi  # noqa: E402
import pmtest  # noqa: E402

T0 = time.time()


def log(*a):
    print(f"[c5 {time.time() - T0:6.1f}s]", *a, file=sys.stderr, flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--scale", type=int, default=27)
    ap.add_argument("--p-gen", type=int, default=8)
    ap.add_argument("--dir", default=None, help="text files (default: /dev/shm when it has room, else TMPDIR)")
    ap.add_argument("--pattern", default="rmat_log2_cycle4_pattern")
    ap.add_argument("--labels", choices=["degree", "hash"], default="hash")
    ap.add_argument("--tds-cap", type=int, default=1 << 20, help="PM_TDS_CAP of the chunk-invariance rerun")
    ap.add_argument("--alphabet", type=int, default=256)
    ap.add_argument("--nranks", type=int, default=8, help="output ranks of the result files")
    ap.add_argument("--oracle", action="store_true")
    ap.add_argument("--out", default=None)
    args = ap.parse_args()
    lib = _abi.load()
    pattern = os.path.join(ROOT, "patterns", args.pattern)
    n = 1 << args.scale
    base_dir = args.dir
    if base_dir is None:
        need = (n * 16 * 20) + (n * 14)
        shm = shutil.disk_usage("/dev/shm").free if os.path.isdir("/dev/shm") else 0
        base_dir = "/dev/shm" if shm > 1.5 * need else tempfile.gettempdir()
    work = tempfile.mkdtemp(prefix="c5_", dir=base_dir)
    res = {"config": "C5 at size", "scale": args.scale, "p_gen": args.p_gen, "pattern": args.pattern,
           "labels": ("degree-log2 labels of the symmetrized graph" if args.labels == "degree" else
                      f"hash32(v ^ 5) % {args.alphabet}") + ", as -v files", "text_dir": base_dir}
    g = None
    try:
        # 0. the graph's host CSR (the oracle's input; degree labels)
        if args.labels == "degree" or args.oracle:
            g = pm.rmat_graph(args.scale, args.p_gen, device=0)
            log(f"host CSR: V={g.n} E={g.nnz}")
        if args.labels == "degree":
            deg = np.diff(g.off)
            labels = np.zeros(n, np.uint64)
            nz = deg > 0
            labels[nz] = (np.floor(np.log2(deg[nz].astype(np.float64))) + 1).astype(np.uint64)  # bit_width
            del deg, nz
        else:
            labels = pmtest.hash_labels(n, args.alphabet, salt=5)
        # 1. inputs
        t = time.time()
        nb = ctypes.c_uint64()
        if lib.pm_write_rmat_text(args.scale, args.p_gen, 0, os.path.join(work, "edges").encode(), ctypes.byref(nb)):
            raise pm._err()
        files = [os.path.join(work, f"edges.{r}") for r in range(args.p_gen)]
        res["edge_text_bytes"] = nb.value
        log(f"edge text: {nb.value / 1e9:.2f} GB in {args.p_gen} files ({time.time() - t:.1f}s)")
        lb = ctypes.c_uint64()
        if lib.pm_write_label_text(labels.ctypes.data, n, os.path.join(work, "lab").encode(), 4, ctypes.byref(lb)):
            raise pm._err()
        res["label_text_bytes"] = lb.value
        log(f"label text: {lb.value / 1e9:.2f} GB in 4 files")
        # 2. GPU ingest (edges, then labels) -> search with result files
        t = time.time()
        m, ingest_s = pm.edge_list_matcher(files, pattern, undirected=True, device=0, nranks=args.nranks)
        t_ctx = time.time() - t
        t = time.time()
        m.labels_from_files(os.path.join(work, "lab"))
        lab_s = time.time() - t
        res["ingest"] = {"edge_parse_and_csr_s": round(ingest_s, 3),
                         "edge_text_gbs": round(nb.value / ingest_s / 1e9, 2),
                         "context_total_s": round(t_ctx, 3),
                         "labels_s_incl_relayout": round(lab_s, 3),
                         "vertices": m.graph.n, "directed_entries": m.graph.nnz}
        log(f"ingest: {ingest_s:.2f}s ({nb.value / ingest_s / 1e9:.2f} GB/s of text), context {t_ctx:.2f}s, "
            f"labels {lab_s:.2f}s, V={m.graph.n} E={m.graph.nnz}")
        out_i = os.path.join(work, "res_ingested")
        t = time.time()
        si = m.run_beta(out_i, 64)
        res["search_ingested"] = {"seconds_incl_files": round(time.time() - t, 3), "stats": si}
        t = time.time()
        reps = [m.run_beta("", 64)["seconds"] for _ in range(3)]
        res["search_ingested"]["seconds_no_files"] = [round(x, 5) for x in reps]
        edges = si["lcc_edges"] + si["nlcc_edges"] + si["tds_edges"]
        res["search_ingested"]["edges_per_s"] = round(edges / min(reps), 1)
        log(f"search (ingested): {si}, {min(reps) * 1e3:.2f} ms without files")
        os.environ["PM_TDS_CAP"] = str(args.tds_cap)
        out_c = os.path.join(work, "res_capped")
        scap = m.run_beta(out_c, 64)
        del os.environ["PM_TDS_CAP"]
        res["chunk_cap_invariance"] = {"cap": args.tds_cap, "chunks": scap["tds_chunks"],
                                       "chunks_default": si["tds_chunks"],
                                       "same": not pmtest.digest_diffs(pmtest.result_digest(out_i, args.nranks),
                                                                       pmtest.result_digest(out_c, args.nranks))}
        log(f"chunk cap {args.tds_cap}: {scap['tds_chunks']} chunks, same result: "
            f"{res['chunk_cap_invariance']['same']}")
        m.close()
        dig_i = pmtest.result_digest(out_i, args.nranks)
        # 3. the same graph generated on the GPU, same labels
        m2, _ = pm.rmat_matcher(args.scale, args.p_gen, pattern, device=0, nranks=args.nranks)
        m2.set_labels(labels)
        out_g = os.path.join(work, "res_generated")
        sg = m2.run_beta(out_g, 64)
        m2.close()
        dig_g = pmtest.result_digest(out_g, args.nranks)
        d = pmtest.digest_diffs(dig_g, dig_i)
        keys = ("iterations", "terminated", "final_vertices", "final_edges", "lcc_edges", "nlcc_edges", "tds_edges",
                "walks")
        res["ingested_equals_generated"] = not d and all(si[k] == sg[k] for k in keys)
        res["digest"] = dig_i
        log(f"ingested == generated: {res['ingested_equals_generated']} {d[:3]}")
        # 4. the oracle on the host CSR (full size)
        if args.oracle:
            import oracle
            log("oracle ...")
            t = time.time()
            out_o = os.path.join(work, "res_oracle")
            so = oracle.run(g.off, g.col, pattern, out_o, labels=labels, nranks=args.nranks, threads=16)
            res["oracle_s"] = round(time.time() - t, 2)
            del g
            diffs = pmtest.compare_result_dirs(out_o, out_i, args.nranks)
            for k_g, k_o in (("final_vertices", "final_vertices"), ("final_edges", "final_edges"),
                             ("lcc_edges", "lcc_edges"), ("nlcc_edges", "nlcc_edges"), ("tds_edges", "tds_edges"),
                             ("walks", "paths"), ("iterations", "iterations")):
                if si[k_g] != so[k_o]:
                    diffs.append(f"{k_g}: gpu {si[k_g]} != oracle {so[k_o]}")
            res["oracle_match"] = not diffs
            res["oracle_diffs"] = diffs[:5]
            log(f"oracle match: {not diffs} ({res['oracle_s']}s) {diffs[:3]}")
    finally:
        shutil.rmtree(work, ignore_errors=True)
    line = json.dumps(res)
    print(line, flush=True)
    if args.out:
        with open(args.out, "w") as f:
            f.write(line + "\n")
    ok = (res.get("ingested_equals_generated") and res.get("oracle_match", True)
          and res.get("chunk_cap_invariance", {}).get("same", True))
    sys.exit(0 if ok else 3)


if __name__ == "__main__":
    main()
