"""CPU tests: oracle pinned against the reference's own vectors and known-answer graphs."""
import os

import numpy as np
import pytest

import oracle
import pmtest

GOLDEN = os.path.join(pmtest.ROOT, "tests", "golden")


def test_mt19937_known_answer():
    # C++ standard [rand.predef]: 10000th output of default-seeded mt19937.
    assert oracle.mt19937_nth(5489, 10000) == 4123659995


def test_hash_nbits_matches_reference_header():
    # Vectors produced by the reference's own include/havoqgt/detail/hash.hpp
    # (oracle/ref_hash_main.cpp, built in place by `make -C oracle ref`).
    n = 0
    with open(os.path.join(GOLDEN, "hash_nbits_ref.txt")) as f:
        for line in f:
            x, bits, h = (int(t) for t in line.split())
            assert oracle.hash_nbits(x, bits) == h, (x, bits)
            n += 1
    assert n == 132
    # SURVEY.md 8(c) spot values
    assert oracle.hash_nbits(0, 21) == 1996217
    assert oracle.hash_nbits(12345, 28) == 149789864


def test_rmat_stream_properties():
    u, v = oracle.rmat_rank_edges(12, 4, 1)
    assert u.shape[0] == (1 << 12) * 16 // 4
    assert u.max() < (1 << 12) and v.max() < (1 << 12)
    # different ranks use different seeds (5489 + 3 r)
    u0, _ = oracle.rmat_rank_edges(12, 4, 0)
    assert not np.array_equal(u0, u)


def _tree_copy(extra=()):
    # template vertices 0..6 of examples/rmat_log2_tree_pattern as graph vertices
    pairs = [(0, 1), (1, 2), (1, 3), (3, 5), (4, 5), (5, 6)] + list(extra)
    labels = np.array([3, 4, 7, 2, 3, 5, 7], np.uint64)
    return pairs, labels


def test_known_answer_single_embedding(tree_pattern, tmp_path):
    pairs, labels = _tree_copy()
    off, col = pmtest.symmetric_csr(pairs, 7)
    st = oracle.run(off, col, tree_pattern, str(tmp_path), labels=labels)
    assert st["terminated"] == 1 and st["iterations"] == 1
    assert st["final_vertices"] == 7 and st["final_edges"] == 12
    assert st["paths"] == 1
    lines = open(tmp_path / "0/all_ranks_subgraphs/subgraphs_4_0").read().split("\n")
    assert lines[0] == "[0], 0, 1, 2, 1, 3, 5, 4, 5, 6, [6]"
    verts = sorted(open(tmp_path / "0/all_ranks_active_vertices/active_vertices_0").read().split("\n")[:-1])
    assert "0, 0, 0, 3, 0000000000000001" in verts  # T_pub of vertex 0 = {template 0}
    assert "0, 4, 0, 3, 0000000000010000" in verts  # vertex 4 = {template 4}


def test_known_answer_no_embedding(tree_pattern, tmp_path):
    pairs, labels = _tree_copy()
    pairs = [p for p in pairs if p != (5, 6)]  # template 5 loses its label-7 neighbour
    off, col = pmtest.symmetric_csr(pairs, 7)
    st = oracle.run(off, col, tree_pattern, str(tmp_path), labels=labels)
    assert st["final_vertices"] == 0 and st["final_edges"] == 0 and st["paths"] == 0


def test_known_answer_shared_label3_vertex(tree_pattern, tmp_path):
    # One label-3 vertex plays templates 0 and 4: LCC keeps it (both bits have
    # their neighbours) but the path 4-5-3-1-0 can only end on itself, so the
    # NLCC invalidates it and the interleaved LCC cascade removes everything.
    pairs = [(0, 1), (1, 2), (1, 3), (3, 5), (0, 5), (5, 6)]
    labels = np.array([3, 4, 7, 2, 99, 5, 7], np.uint64)  # vertex 4 unused (label 99)
    off, col = pmtest.symmetric_csr(pairs, 7)
    st = oracle.run(off, col, tree_pattern, str(tmp_path), labels=labels)
    assert st["final_vertices"] == 0
    assert st["iterations"] >= 1 and st["terminated"] == 1
    steps = open(tmp_path / "0/result_step").read().split("\n")
    assert len(steps) > 2  # an interleaved LCC ran


def test_known_answer_degree_labels(tree_pattern):
    # The tree embedded with degree-log2 labels: pad every vertex with leaf
    # neighbours (degree 1 -> label 1, matches no template).
    want_deg = {0: 4, 1: 8, 2: 64, 3: 2, 4: 4, 5: 16, 6: 64}
    pairs, _ = _tree_copy()
    deg = {v: 0 for v in want_deg}
    for a, b in pairs:
        deg[a] += 1
        deg[b] += 1
    nxt = 7
    for v, d in want_deg.items():
        for _ in range(d - deg[v]):
            pairs.append((v, nxt))
            nxt += 1
    off, col = pmtest.symmetric_csr(pairs, nxt)
    st = oracle.run(off, col, tree_pattern)
    assert st["final_vertices"] == 7 and st["final_edges"] == 12 and st["paths"] == 1


def test_oracle_partition_invariance(cycle_pattern, tmp_path):
    off, col = oracle.rmat_csr(10, 4)
    labels = pmtest.hash_labels(1 << 10, 8)
    a, b = tmp_path / "p1", tmp_path / "p3"
    s1 = oracle.run(off, col, cycle_pattern, str(a), labels=labels, nranks=1)
    s3 = oracle.run(off, col, cycle_pattern, str(b), labels=labels, nranks=3)
    assert s1["nlcc_edges"] > 0 and s1["paths"] > 0
    assert s1["final_vertices"] == s3["final_vertices"] and s1["final_edges"] == s3["final_edges"]
    cat = lambda d, sub, stem, n: sorted(
        l.split(", ", 1)[1] for r in range(n) for l in open(d / "0" / sub / f"{stem}{r}").read().split("\n") if l)
    assert cat(a, "all_ranks_active_vertices", "active_vertices_", 1) == \
        cat(b, "all_ranks_active_vertices", "active_vertices_", 3)


def test_oracle_selected_vertices_known_answer(tmp_path):
    """patterns/selected_vertices_pattern on hand-built graphs (counts derived by hand, see
    the pattern's README).  A 4-cycle c (label 5) - d (6) - a (3) - b (4) - c, plus
    a2 (3) - b2 (4) - c2 (5) - d hanging off it.  a2 fails the LCC in superstep 0 (no
    label-6 neighbour), b2 in superstep 1; c2 survives the LCC but line 0 never reaches it
    from a through a B, so the selected-vertices line 1 leaves it unconfirmed: bit 2
    cleared, c2 leaves S (its M and d's entry stay until the next LCC call).

    The reference registers a selected vertex when its own init visit runs
    (nem_1.hpp:409-436), and on one rank the init traversal drains every source's tokens
    before the next vertex (visitor_queue.hpp:221-251): a C vertex is confirmed only if
    its id precedes the source's.  With c = 0 < a = 3 the 4-cycle survives; with the ids
    of the cycle reversed (a = 0 < c = 2) c is not yet registered when a's token arrives,
    so it is dropped as well and the whole graph empties."""
    pat = os.path.join(pmtest.ROOT, "patterns", "selected_vertices_pattern")
    rd = lambda d, f: open(tmp_path / "0" / d / f).read().split("\n")[:-1]
    # c=0, d=1, b=2, a=3, c2=4, b2=5, a2=6
    pairs = [(3, 2), (2, 0), (0, 1), (1, 3), (6, 5), (5, 4), (4, 1)]
    labels = np.array([5, 6, 4, 3, 5, 4, 3], np.uint64)
    off, col = pmtest.symmetric_csr(pairs, 7)
    so = oracle.run(off, col, pat, str(tmp_path), labels=labels)
    assert so["iterations"] == 2 and so["terminated"] == 1
    assert so["final_vertices"] == 4 and so["final_edges"] == 8
    assert rd("all_ranks_active_vertices_count", "active_vertices_0") == [
        "0, LP, 0, 6", "0, LP, 1, 5", "0, TP, 0, 5", "0, TP, 1, 4",
        "1, LP, 0, 4", "1, LP, 1, 4"]  # no removal in iteration 1: no token passing
    assert rd("all_ranks_active_edges_count", "active_edges_0") == [
        "0, LP, 0, 13", "0, LP, 1, 11", "0, TP, 0, 11", "0, TP, 1, 9",
        "1, LP, 0, 8", "1, LP, 1, 8"]
    final = sorted(l.split(", ")[1] for l in rd("all_ranks_active_vertices", "active_vertices_0"))
    assert final == ["0", "1", "2", "3"]
    # a = 0, b = 1, c = 2, d = 3: c is registered after a's tokens have passed
    pairs = [(0, 1), (1, 2), (2, 3), (3, 0), (4, 5), (5, 6), (6, 3)]
    labels = np.array([3, 4, 5, 6, 3, 4, 5], np.uint64)
    off, col = pmtest.symmetric_csr(pairs, 7)
    so = oracle.run(off, col, pat, str(tmp_path / "b"), labels=labels)
    assert so["final_vertices"] == 0
    assert open(tmp_path / "b/0/all_ranks_active_vertices_count/active_vertices_0").read().split("\n")[3] == \
        "0, TP, 1, 3"


def test_result_digest_is_rank_count_independent(tmp_path):
    """pmtest.result_digest (the S=28 fixture's digest) sums count files over ranks and drops
    the rank column, so one fixture checks any number of ranks / shards."""
    import pmtest
    off, col = oracle.rmat_csr(13, 4)
    pattern = os.path.join(pmtest.ROOT, "patterns", "rmat_log2_tree_pattern")
    ds = []
    for nr in (1, 3):
        rd = str(tmp_path / f"r{nr}")
        oracle.run(off, col, pattern, rd, nranks=nr)
        ds.append(pmtest.result_digest(rd, nr))
    assert pmtest.digest_diffs(ds[0], ds[1]) == []
    assert ds[0]["all_ranks_active_vertices"]["lines"] > 0
