"""Shared helpers for the parity tests: graph builders and result-dir comparison."""
import os

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

# parity = sorted line sets for vertex / edge / subgraph
# files, exact per-rank line sequences for count files; timing columns and
# message counts are excluded.
SET_DIRS = {"all_ranks_active_vertices", "all_ranks_active_edges", "all_ranks_subgraphs"}
SEQ_DIRS = {"all_ranks_active_vertices_count", "all_ranks_active_edges_count"}


def csr_from_edges(src, dst, n):
    src = np.asarray(src, np.uint64)
    dst = np.asarray(dst, np.uint64)
    o = np.lexsort((dst, src))
    src, dst = src[o], dst[o]
    off = np.zeros(n + 1, np.uint64)
    np.add.at(off, src.astype(np.int64) + 1, 1)
    return np.cumsum(off).astype(np.uint64), dst.astype(np.uint32)


def symmetric_csr(pairs, n):
    src = [a for a, b in pairs] + [b for a, b in pairs]
    dst = [b for a, b in pairs] + [a for a, b in pairs]
    return csr_from_edges(src, dst, n)


def hash_labels(n, alphabet, salt=0):
    """Explicit small-alphabet labels (config C5 style): hash32(v ^ salt) % alphabet."""
    v = (np.arange(n, dtype=np.uint64) ^ np.uint64(salt)).astype(np.uint32)
    a = v.astype(np.uint64)
    m = np.uint64(0xFFFFFFFF)
    a = ((a + np.uint64(0x7ed55d16)) + (a << np.uint64(12))) & m
    a = ((a ^ np.uint64(0xc761c23c)) ^ (a >> np.uint64(19))) & m
    a = ((a + np.uint64(0x165667b1)) + (a << np.uint64(5))) & m
    a = ((a + np.uint64(0xd3a2646c)) ^ (a << np.uint64(9))) & m
    a = ((a + np.uint64(0xfd7046c5)) + (a << np.uint64(3))) & m
    a = ((a ^ np.uint64(0xb55a4f09)) ^ (a >> np.uint64(16))) & m
    return (a % np.uint64(alphabet)).astype(np.uint64)


def _read(path):
    with open(path) as f:
        return [l.rstrip("\n") for l in f]


def _strip_time(lines, keep_cols):
    return [", ".join(l.split(", ")[:keep_cols]) for l in lines]


def compare_result_dirs(a, b, nranks):
    """Returns a list of human-readable differences (empty = parity)."""
    diffs = []
    pa = _read(os.path.join(a, "result_pattern_set"))
    pb = _read(os.path.join(b, "result_pattern_set"))
    cut = lambda ls: [l.split(", ")[:3] + l.split(", ")[4:] for l in ls]
    if cut(pa) != cut(pb):
        diffs.append(f"result_pattern_set: {pa} != {pb}")
    for name, cols in (("result_iteration", 1), ("result_step", 2), ("result_superstep", 3)):
        la = _strip_time(_read(os.path.join(a, "0", name)), cols)
        lb = _strip_time(_read(os.path.join(b, "0", name)), cols)
        if la != lb:
            diffs.append(f"{name}: {la[:6]}... != {lb[:6]}...")
    for r in range(nranks):
        for d in SEQ_DIRS:
            fn = ("active_vertices_" if "vertices" in d else "active_edges_") + str(r)
            la = _read(os.path.join(a, "0", d, fn))
            lb = _read(os.path.join(b, "0", d, fn))
            if la != lb:
                diffs.append(f"{d}/{fn}: {la} != {lb}")
        for d in ("all_ranks_active_vertices", "all_ranks_active_edges"):
            fn = ("active_vertices_" if "vertices" in d else "active_edges_") + str(r)
            la = sorted(_read(os.path.join(a, "0", d, fn)))
            lb = sorted(_read(os.path.join(b, "0", d, fn)))
            if la != lb:
                diffs.append(f"{d}/{fn}: {len(la)} vs {len(lb)} lines; first diff "
                             f"{sorted(set(la) ^ set(lb))[:5]}")
        sg = os.path.join(a, "0", "all_ranks_subgraphs")
        names = sorted(x for x in os.listdir(sg) if x.endswith("_" + str(r)))
        for fn in names:
            la = sorted(_read(os.path.join(a, "0", "all_ranks_subgraphs", fn)))
            pb_ = os.path.join(b, "0", "all_ranks_subgraphs", fn)
            lb = sorted(_read(pb_)) if os.path.exists(pb_) else None
            if la != lb:
                diffs.append(f"subgraphs/{fn}: {None if lb is None else len(lb)} vs {len(la)} lines")
    return diffs
