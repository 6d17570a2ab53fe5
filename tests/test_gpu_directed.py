"""Directed inputs and asymmetric active-edge maps (SURVEY A.6 hazards 5, 9, 10): the
push-form later supersteps (k_lcc_push_send / k_lcc_push_verify) and the in-row
superstep 0 against the oracle, which restates the reference's message passing
(sends along out-edges, later supersteps along keys(M[v])) and needs no symmetry."""
import os
import subprocess

import numpy as np
import pytest

import fuzzypatternmatching_amd as pm
import oracle
import pmtest

pytestmark = pytest.mark.gpu

TREE = os.path.join(pmtest.ROOT, "patterns", "rmat_log2_tree_pattern")
CYCLE = os.path.join(pmtest.ROOT, "patterns", "rmat_log2_cycle4_pattern")
BIN = os.path.join(pmtest.ROOT, "fuzzypatternmatching_amd", "csrc", "tools", "bin")


def _directed_rmat(scale, p_gen):
    """The generator's undirected pairs (u, v) taken as directed edges u -> v only."""
    und = [oracle.rmat_rank_edges(scale, p_gen, r) for r in range(p_gen)]
    u = np.concatenate([x[0] for x in und])
    v = np.concatenate([x[1] for x in und])
    off, col = pmtest.csr_from_edges(u, v, 1 << scale)
    return off, col


def _check(off, col, pattern, tmp_path, labels=None, nranks=1, symmetric=False):
    a, b = tmp_path / "oracle", tmp_path / "gpu"
    so = oracle.run(off, col, pattern, str(a), labels=labels, nranks=nranks, threads=oracle.default_threads())
    m = pm.PatternMatcher(pm.Graph(off, col, symmetric, nranks), pattern, labels=labels)
    sg = m.run_beta(str(b))
    m.close()
    assert pmtest.compare_result_dirs(str(a), str(b), nranks) == []
    for k_g, k_o in (("iterations", "iterations"), ("terminated", "terminated"), ("final_vertices", "final_vertices"),
                     ("final_edges", "final_edges"), ("lcc_edges", "lcc_edges"), ("nlcc_edges", "nlcc_edges"),
                     ("tds_edges", "tds_edges"), ("walks", "paths")):
        assert sg[k_g] == so[k_o], (k_g, sg[k_g], so[k_o])
    return sg


@pytest.mark.parametrize("pat,scale,p_gen,alphabet,nranks", [
    ("tree", 12, 2, None, 1), ("tree", 16, 4, None, 3), ("cycle", 14, 4, None, 1),
    ("cycle", 11, 1, 8, 2), ("tree", 10, 1, 16, 1), ("cycle", 16, 4, 64, 1)])
def test_directed_rmat_matches_oracle(pat, scale, p_gen, alphabet, nranks, tmp_path):
    off, col = _directed_rmat(scale, p_gen)
    labels = None if alphabet is None else pmtest.hash_labels(1 << scale, alphabet)
    _check(off, col, TREE if pat == "tree" else CYCLE, tmp_path, labels, nranks)


def test_directed_known_answer(tmp_path):
    # the tree embedding of tests/test_gpu_parity.py with every edge one way only:
    # superstep 0 still builds M from the in-edges, later supersteps follow M back
    pairs = [(0, 1), (1, 2), (1, 3), (3, 5), (4, 5), (5, 6), (2, 1), (6, 5)]
    labels = np.array([3, 4, 7, 2, 3, 5, 7], np.uint64)
    off, col = pmtest.csr_from_edges([a for a, b in pairs], [b for a, b in pairs], 7)
    _check(off, col, TREE, tmp_path, labels)


def test_ingest_directed_edge_list_cli(tmp_path):
    """ingest_edge_list -u 0 (the reference's default, ingest_edge_list.cpp:92,115) -> beta CLI."""
    off, col = _directed_rmat(12, 2)
    src = np.repeat(np.arange(off.shape[0] - 1, dtype=np.uint64), np.diff(off).astype(np.int64))
    txt = tmp_path / "edges.txt"
    np.savetxt(txt, np.stack([src, col.astype(np.uint64)], 1), fmt="%d")
    base = str(tmp_path / "g")
    r = subprocess.run([os.path.join(BIN, "ingest_edge_list"), "-o", base, "-n", "2", str(txt)],
                       capture_output=True, text=True)
    assert r.returncode == 0, r.stderr
    g = pm.read_graph(base)
    assert not g.symmetric
    out = tmp_path / "gpu"
    out.mkdir()
    r = subprocess.run([os.path.join(BIN, "run_pattern_matching_beta"), "-i", base, "-p", TREE, "-o", str(out)],
                       capture_output=True, text=True)
    assert r.returncode == 0, r.stderr
    ora = tmp_path / "oracle"
    oracle.run(g.off, g.col, TREE, str(ora), nranks=2, threads=oracle.default_threads())
    assert pmtest.compare_result_dirs(str(ora), str(out), 2) == []


TRI = os.path.join(pmtest.ROOT, "patterns", "triangle_tail_pattern")


def _triangles(k, extra=()):
    """k disjoint triangles s-b-c (labels 3, 4, 5) plus extra edges."""
    pairs = []
    for t in range(k):
        s, b, c = 3 * t, 3 * t + 1, 3 * t + 2
        pairs += [(s, b), (b, c), (s, c)]
    pairs += list(extra)
    n = 3 * k
    labels = np.array([3, 4, 5] * k, np.uint64)
    off, col = pmtest.symmetric_csr(pairs, n)
    return off, col, labels


@pytest.mark.parametrize("k,extra", [(1, ()), (6, [(1, 7), (4, 10), (2, 5), (9, 9), (12, 16), (13, 3)])])
def test_asymmetric_active_edge_map(k, extra, tmp_path, monkeypatch):
    """patterns/triangle_tail_pattern on triangles: line 0 acks the label-3 vertex s and
    flags M[s][c] (nem_1.hpp:764-770); line 1 leaves s unacked and clears bit 0 of its
    T_pub only; the next LCC call's messages then keep s -> c alive through the flag
    while c drops s (SURVEY A.6 hazards 4, 5, 9; hand-derived in the pattern's README).
    The pull form must detect the asymmetry (PM_FORCE_PULL=1 aborts); the default push
    form matches the oracle."""
    off, col, labels = _triangles(k, extra)
    monkeypatch.setenv("PM_FORCE_PULL", "1")
    m = pm.PatternMatcher(pm.Graph(off, col, True), TRI, labels=labels)
    with pytest.raises(pm.PMError, match="asymmetric"):
        m.run_beta("", 50)
    m.close()
    monkeypatch.delenv("PM_FORCE_PULL")
    sg = _check(off, col, TRI, tmp_path, labels, symmetric=True)
    if k == 1:  # hand-derived: iteration 1 keeps s with both (flagged) entries for one superstep
        lines = open(tmp_path / "gpu/0/all_ranks_active_edges_count/active_edges_0").read().split("\n")
        assert lines[4] == "1, LP, 0, 2" and sg["iterations"] == 2


TDS_TAIL = os.path.join(pmtest.ROOT, "patterns", "triangle_tail_tds_pattern")


@pytest.mark.parametrize("k,extra", [(4, [(1, 3), (7, 10)]), (6, [(1, 7), (4, 10), (2, 5), (9, 9), (12, 16), (13, 3)])])
def test_subgraph_files_rewritten_per_iteration(k, extra, tmp_path):
    """patterns/triangle_tail_tds_pattern: enumeration lines in two iterations, the second
    one truncating subgraphs_4_0 (SURVEY A.6 hazard 6; hand-derived for k = 4 in the
    pattern's README and tests/test_cpu_hazards.py)."""
    off, col, labels = _triangles(k, extra)
    sg = _check(off, col, TDS_TAIL, tmp_path, labels, symmetric=True)
    assert sg["iterations"] == 2
