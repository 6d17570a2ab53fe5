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


def _sha(lines):
    import hashlib
    h = hashlib.sha256()
    for l in lines:
        h.update(l.encode())
        h.update(b"\n")
    return h.hexdigest()


def result_digest(result_dir, nranks):
    """Rank-count-independent digest of a result directory (for fixtures at sizes whose
    result files are too large to commit, e.g. the S=28 headline).

    * result_pattern_set and result_iteration/step/superstep without the timing columns;
    * count files summed over the rank files line by line, as the reference's aggregator
      examples/scripts/total_active_count.py:38-91 does (the tokens of the first file's line
      minus the last one, then the sum of the last tokens over all rank files);
    * vertex / edge / subgraph files: the union over ranks with the rank column dropped,
      as (line count, sha256 of the sorted lines)."""
    d = os.path.join(result_dir, "0")
    out = {}
    ps = _read(os.path.join(result_dir, "result_pattern_set"))
    # ps, P, iterations, seconds, |E_p|, |V_p|, #NLC (beta.cpp:1375-1381): P and seconds dropped
    out["result_pattern_set"] = [", ".join(l.split(", ")[:1] + l.split(", ")[2:3] + l.split(", ")[4:]) for l in ps]
    for name, cols in (("result_iteration", 1), ("result_step", 2), ("result_superstep", 3)):
        out[name] = _strip_time(_read(os.path.join(d, name)), cols)
    for sub, stem in (("all_ranks_active_vertices_count", "active_vertices_"),
                      ("all_ranks_active_edges_count", "active_edges_")):
        tot = None
        for r in range(nranks):
            ls = [l.split(", ") for l in _read(os.path.join(d, sub, stem + str(r)))]
            if tot is None:
                tot = [[", ".join(t[:-1]), int(t[-1])] for t in ls]
            else:
                assert len(ls) == len(tot), f"{sub}: rank files of different length"
                for a, t in zip(tot, ls):
                    a[1] += int(t[-1])
        out[sub] = [f"{a}, {b}" for a, b in (tot or [])]
    for sub, stem in (("all_ranks_active_vertices", "active_vertices_"), ("all_ranks_active_edges", "active_edges_")):
        lines = []
        for r in range(nranks):
            lines += [l.split(", ", 1)[1] for l in _read(os.path.join(d, sub, stem + str(r))) if l]
        lines.sort()
        out[sub] = {"lines": len(lines), "sha256": _sha(lines)}
    sg = os.path.join(d, "all_ranks_subgraphs")
    by_line = {}
    for fn in sorted(os.listdir(sg)):
        pl = fn.split("_")[1]
        by_line.setdefault(pl, [])
        by_line[pl] += [l.split(", ", 1)[1] for l in _read(os.path.join(sg, fn)) if l]
    out["all_ranks_subgraphs"] = {pl: {"lines": len(v), "sha256": _sha(sorted(v))} for pl, v in sorted(by_line.items())}
    return out


def digest_diffs(a, b):
    """Keys on which two result_digest() dicts differ."""
    return [f"{k}: {a.get(k)} != {b.get(k)}" for k in sorted(set(a) | set(b)) if a.get(k) != b.get(k)]


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
