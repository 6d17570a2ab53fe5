"""GPU parity tests: the HIP path (via the C-ABI) against the CPU oracle on the same inputs."""
import os

import numpy as np
import pytest

import fuzzypatternmatching_amd as pm
import oracle
import pmtest

pytestmark = pytest.mark.gpu

PATTERNS = {
    "tree": os.path.join(pmtest.ROOT, "patterns", "rmat_log2_tree_pattern"),
    "cycle": os.path.join(pmtest.ROOT, "patterns", "rmat_log2_cycle4_pattern"),
}

# (pattern, scale, P_gen, label alphabet or None for degree labels, nranks)
RMAT_CASES = [
    ("tree", 10, 1, None, 1),
    ("tree", 16, 4, None, 1),
    ("tree", 16, 4, None, 4),
    ("cycle", 14, 4, None, 1),
    ("cycle", 10, 1, 8, 1),
    ("cycle", 12, 4, 8, 3),
    ("tree", 10, 1, 16, 1),
    ("tree", 9, 2, 8, 2),
]


def _run_both(off, col, pattern, tmp_path, labels=None, nranks=1, max_iterations=100):
    a, b = tmp_path / "oracle", tmp_path / "gpu"
    so = oracle.run(off, col, pattern, str(a), labels=labels, nranks=nranks, max_iterations=max_iterations)
    g = pm.Graph(off, col, True, nranks)
    m = pm.PatternMatcher(g, pattern, labels=labels)
    sg = m.run_beta(str(b), max_iterations=max_iterations)
    m.close()
    return so, sg, pmtest.compare_result_dirs(str(a), str(b), nranks)


@pytest.mark.parametrize("pat,scale,p_gen,alphabet,nranks", RMAT_CASES)
def test_rmat_matches_oracle(pat, scale, p_gen, alphabet, nranks, tmp_path):
    g = pm.rmat_graph(scale, p_gen)
    labels = None if alphabet is None else pmtest.hash_labels(g.n, alphabet)
    so, sg, diffs = _run_both(g.off, g.col, PATTERNS[pat], tmp_path, labels, nranks)
    assert diffs == []
    assert sg["iterations"] == so["iterations"] and sg["terminated"] == so["terminated"]
    assert sg["final_vertices"] == so["final_vertices"] and sg["final_edges"] == so["final_edges"]
    # edges-traversed counters are defined identically on both sides
    assert sg["lcc_edges"] == so["lcc_edges"]
    assert sg["nlcc_edges"] == so["nlcc_edges"]
    assert sg["tds_edges"] == so["tds_edges"]
    assert sg["walks"] == so["paths"]


@pytest.mark.parametrize("pat,scale,p_gen,alphabet", [("tree", 16, 4, None), ("cycle", 14, 4, None),
                                                     ("cycle", 12, 4, 8)])
def test_repeated_searches_on_one_context(pat, scale, p_gen, alphabet, tmp_path):
    # three searches on one context (as the bench runs them): each must reproduce the oracle.  From the second
    # search on, the first later superstep's kernel is chosen from the previous search's superstep-0 survivors
    # (short rows: 3 entries in flight per lane, else 4), so both instantiations meet the oracle here.
    g = pm.rmat_graph(scale, p_gen)
    labels = None if alphabet is None else pmtest.hash_labels(g.n, alphabet)
    a = tmp_path / "oracle"
    so = oracle.run(g.off, g.col, PATTERNS[pat], str(a), labels=labels, nranks=1)
    m = pm.PatternMatcher(pm.Graph(g.off, g.col, True, 1), PATTERNS[pat], labels=labels)
    try:
        for i in range(3):
            b = tmp_path / f"gpu{i}"
            sg = m.run_beta(str(b))
            assert pmtest.compare_result_dirs(str(a), str(b), 1) == [], i
            assert (sg["lcc_edges"], sg["nlcc_edges"], sg["tds_edges"], sg["walks"]) == \
                (so["lcc_edges"], so["nlcc_edges"], so["tds_edges"], so["paths"]), i
    finally:
        m.close()


@pytest.mark.parametrize("pat,scale,p_gen,alphabet,nranks", [RMAT_CASES[2], RMAT_CASES[5], RMAT_CASES[7]])
def test_exact_count_token_passing_matches_oracle(pat, scale, p_gen, alphabet, nranks, tmp_path, monkeypatch):
    # PM_FUSED_LINES=0: every NLC line through the per-position launch path
    # (the fallback of the fused line kernels on capacity overflow)
    monkeypatch.setenv("PM_FUSED_LINES", "0")
    g = pm.rmat_graph(scale, p_gen)
    labels = None if alphabet is None else pmtest.hash_labels(g.n, alphabet)
    so, sg, diffs = _run_both(g.off, g.col, PATTERNS[pat], tmp_path, labels, nranks)
    assert diffs == []
    assert sg["nlcc_edges"] == so["nlcc_edges"] and sg["tds_edges"] == so["tds_edges"]


@pytest.mark.parametrize("env", [{"PM_PATH_BATCH": "1"}, {"PM_PATH_BATCH": "7"}, {"PM_ARENA_MB": "1"}])
def test_exact_path_lines_in_source_batches(env, tmp_path, monkeypatch):
    """The exact path's path / cycle lines in initiator batches: forced (PM_PATH_BATCH) or because a line's tokens
    do not fit a 1 MiB scratch arena (PM_ARENA_MB=1: the batch that ran out of room is discarded and halved) --
    config C5's S=26 search with 64 letters ran out of the 32 GiB arena before batches existed.  Every result file
    and counter against the oracle."""
    monkeypatch.setenv("PM_FUSED_LINES", "0")
    for k, v in env.items():
        monkeypatch.setenv(k, v)
    g = pm.rmat_graph(12, 4)
    labels = pmtest.hash_labels(g.n, 8)
    so, sg, diffs = _run_both(g.off, g.col, PATTERNS["cycle"], tmp_path, labels, 3)
    assert diffs == []
    assert (sg["lcc_edges"], sg["nlcc_edges"], sg["tds_edges"], sg["walks"]) == \
        (so["lcc_edges"], so["nlcc_edges"], so["tds_edges"], so["paths"])
    print(f"exact lines {sg['exact_lines']}, path batches {sg['path_batches']}")
    assert sg["path_batches"] > sg["exact_lines"]  # (batches did run: more than one per line)


@pytest.mark.parametrize("env,nranks", [({"PM_HASH_SLOTS": "16384", "PM_DEBUG_NOGROW_SHARD": "0"}, 1),
                                         ({"PM_HASH_SLOTS": "16384", "PM_DEBUG_NOGROW_SHARD": "0"}, 3),
                                         ({"PM_FUSED_WCAP": "1048576"}, 1)])
def test_local_split_lines_match_oracle(env, nranks, tmp_path, monkeypatch):
    """One context, a path / cycle line that outgrows the (source, vertex) table with no room to grow it
    (PM_HASH_SLOTS, PM_DEBUG_NOGROW_SHARD=0), or a TDS line that outgrows the fused walk storage (PM_FUSED_WCAP):
    the fused kernel runs the line over its sources in parts, the post-processing once after every part
    (local_split_line), instead of the exact path.  Every result file and counter against the oracle."""
    for k, v in env.items():
        monkeypatch.setenv(k, v)
    g = pm.rmat_graph(13, 4)
    labels = pmtest.hash_labels(g.n, 8)
    so, sg, diffs = _run_both(g.off, g.col, PATTERNS["cycle"], tmp_path, labels, nranks)
    assert diffs == []
    assert (sg["lcc_edges"], sg["nlcc_edges"], sg["tds_edges"], sg["walks"], sg["final_vertices"]) == \
        (so["lcc_edges"], so["nlcc_edges"], so["tds_edges"], so["paths"], so["final_vertices"])
    print(f"overflows {sg['line_overflows']}, local split lines {sg['split_lines']}, exact lines {sg['exact_lines']}")
    assert sg["line_overflows"] > 0 and sg["split_lines"] > 0


@pytest.mark.parametrize("pat,scale,p_gen,alphabet,nranks,shards,pack",
                         [("tree", 16, 4, None, 4, 0, None), ("cycle", 14, 4, None, 1, 0, None),
                          ("cycle", 12, 4, 8, 3, 0, None), ("cycle", 15, 4, 64, 1, 0, None),
                          ("cycle", 15, 4, 64, 1, 0, 3), ("tree", 15, 4, None, 2, 3, None),
                          ("cycle", 13, 4, 8, 1, 2, None)])
def test_pull_long_rows_in_pieces(pat, scale, p_gen, alphabet, nranks, shards, pack, tmp_path, monkeypatch):
    """PM_PULL_LONG=8: every pull-superstep row above 8 entries goes to the long-row list and is worked in pieces by
    k_lcc_step_pieces (the path of C5's hub rows, normally above 4096 entries), its verify by the row's last piece,
    and in the call's last superstep packed by k_long_pack (PM_PACK_PIECES=3: most rows do not fit the scratch and
    are left to the row compaction); three searches per context (from the second on, the pieces launch runs only
    where the previous search listed rows), and the sharded path, against the oracle."""
    monkeypatch.setenv("PM_PULL_LONG", "8")
    if pack:
        monkeypatch.setenv("PM_PACK_PIECES", str(pack))
    g = pm.rmat_graph(scale, p_gen)
    labels = None if alphabet is None else pmtest.hash_labels(g.n, alphabet)
    a = tmp_path / "oracle"
    hub = 64 if shards else pm.DEFAULT_HUB_THRESHOLD  # (sharded: delegates split by target owner)
    so = oracle.run(g.off, g.col, PATTERNS[pat], str(a), labels=labels, nranks=nranks, hub_threshold=hub)
    keys = ("lcc_edges", "nlcc_edges", "tds_edges", "walks", "final_vertices", "final_edges")
    want = tuple(so["paths" if k == "walks" else k] for k in keys)
    if shards:
        b = tmp_path / "gpu_shards"
        sg = pm.run_beta_local_shards(pm.Graph(g.off, g.col, True, nranks, hub_threshold=hub), PATTERNS[pat], shards,
                                      str(b), labels=labels)
        assert pmtest.compare_result_dirs(str(a), str(b), nranks) == []
        assert tuple(sg[k] for k in keys) == want
        return
    m = pm.PatternMatcher(pm.Graph(g.off, g.col, True, nranks), PATTERNS[pat], labels=labels)
    try:
        for i in range(3):
            b = tmp_path / f"gpu{i}"
            sg = m.run_beta(str(b))
            assert pmtest.compare_result_dirs(str(a), str(b), nranks) == [], i
            assert tuple(sg[k] for k in keys) == want, i
    finally:
        m.close()


def _tree_pairs():
    return [(0, 1), (1, 2), (1, 3), (3, 5), (4, 5), (5, 6)], np.array([3, 4, 7, 2, 3, 5, 7], np.uint64)


def test_known_answer_single_embedding(tmp_path):
    pairs, labels = _tree_pairs()
    off, col = pmtest.symmetric_csr(pairs, 7)
    so, sg, diffs = _run_both(off, col, PATTERNS["tree"], tmp_path, labels)
    assert diffs == []
    assert sg["final_vertices"] == 7 and sg["final_edges"] == 12 and sg["walks"] == 1
    lines = open(tmp_path / "gpu/0/all_ranks_subgraphs/subgraphs_4_0").read().split("\n")
    assert lines[0] == "[0], 0, 1, 2, 1, 3, 5, 4, 5, 6, [6]"


def test_known_answer_shared_label3_vertex(tmp_path):
    pairs = [(0, 1), (1, 2), (1, 3), (3, 5), (0, 5), (5, 6)]
    labels = np.array([3, 4, 7, 2, 99, 5, 7], np.uint64)
    off, col = pmtest.symmetric_csr(pairs, 7)
    so, sg, diffs = _run_both(off, col, PATTERNS["tree"], tmp_path, labels)
    assert diffs == []
    assert sg["final_vertices"] == 0


def test_empty_and_isolated_inputs(tmp_path):
    # no edges at all, and a graph whose labels match nothing
    off = np.zeros(9, np.uint64)
    col = np.zeros(0, np.uint32)
    so, sg, diffs = _run_both(off, col, PATTERNS["tree"], tmp_path / "a", np.full(8, 3, np.uint64))
    assert diffs == [] and sg["final_vertices"] == 0
    off2, col2 = pmtest.symmetric_csr([(0, 1), (1, 2), (2, 0), (2, 2)], 3)  # includes a self loop
    so, sg, diffs = _run_both(off2, col2, PATTERNS["cycle"], tmp_path / "b", np.array([3, 4, 5], np.uint64))
    assert diffs == []


def test_duplicate_edges_and_self_loops(tmp_path):
    pairs, labels = _tree_pairs()
    pairs = pairs + [(1, 2), (1, 2), (5, 5), (3, 3), (0, 1)]  # multiplicity + self loops
    off, col = pmtest.symmetric_csr(pairs, 7)
    so, sg, diffs = _run_both(off, col, PATTERNS["tree"], tmp_path, labels)
    assert diffs == []
    assert sg["lcc_edges"] == so["lcc_edges"]


def test_heavy_rows_segment_boundaries(tmp_path):
    # Two hubs of degree > 1024 (split into 1024-entry segments by superstep 0)
    # with duplicate entries straddling the segment boundary, plus rows of
    # 65..1024 entries.  Cycle pattern labels: A=3, leaves 4, C=5, closers 6.
    n_leaf, n_close = 1100, 3
    A, C = 0, 1
    leaves = list(range(2, 2 + n_leaf))
    closers = list(range(2 + n_leaf, 2 + n_leaf + n_close))
    pairs = [(A, v) for v in leaves] + [(C, v) for v in leaves]
    pairs += [(A, v) for v in leaves[1000:1050]] * 2  # multiplicity across entry 1024 of A's row
    pairs += [(C, w) for w in closers] + [(A, w) for w in closers]
    mid = 2 + n_leaf + n_close  # a row of 200 entries (65..1024 class)
    pairs += [(mid, v) for v in leaves[:200]]
    n = mid + 1
    labels = np.zeros(n, np.uint64)
    labels[A], labels[C] = 3, 5
    labels[leaves] = 4
    labels[closers] = 6
    labels[mid] = 3
    off, col = pmtest.symmetric_csr(pairs, n)
    so, sg, diffs = _run_both(off, col, PATTERNS["cycle"], tmp_path, labels)
    assert diffs == []
    assert sg["lcc_edges"] == so["lcc_edges"] and sg["tds_edges"] == so["tds_edges"]
    assert sg["walks"] == so["paths"] and sg["walks"] > 0


def test_step_api_matches_driver():
    g = pm.rmat_graph(12, 4)
    labels = pmtest.hash_labels(g.n, 8)
    m = pm.PatternMatcher(g, PATTERNS["cycle"], labels=labels)
    m.reset()
    s = m.lcc_bsp(True)
    assert s["supersteps"] == 4
    tp = m.token_passing(0)
    assert tp["sources"] > 0 and tp["edges_traversed"] > 0
    m.post_token_passing(0)
    tpub, mdeg, nbrs = m.export_state()
    assert int(mdeg.sum()) == nbrs.shape[0]
    assert np.all(mdeg[tpub == 0] == 0)
    m.close()


def test_tds_walk_sink_matches_subgraph_file(tmp_path):
    """pm_tds hands each kept walk to a callback: iteration 0 of the hand-derived
    patterns/triangle_tail_tds_pattern input (four triangles) through the step API gives the
    lines of the oracle's subgraphs_4_0 after one iteration (tests/test_cpu_hazards.py)."""
    pat = os.path.join(pmtest.ROOT, "patterns", "triangle_tail_tds_pattern")
    pairs = [(3 * t + a, 3 * t + b) for t in range(4) for a, b in ((0, 1), (1, 2), (0, 2))] + [(1, 3), (7, 10)]
    off, col = pmtest.symmetric_csr(pairs, 12)
    labels = np.array([3, 4, 5] * 4, np.uint64)
    oracle.run(off, col, pat, str(tmp_path), labels=labels, max_iterations=1)
    want = sorted(l for l in open(tmp_path / "0" / "all_ranks_subgraphs" / "subgraphs_4_0").read().split("\n") if l)
    m = pm.PatternMatcher(pm.Graph(off, col, True), pat, labels=labels)
    m.reset()
    m.lcc_bsp(True)
    for pl in range(4):
        m.token_passing(pl)
        m.post_token_passing(pl)
    got = []
    st = m.tds(4, lambda rank, v: got.append(f"[{rank}], " + ", ".join(map(str, v)) + f", [{v[-1]}]"))
    m.close()
    assert sorted(got) == want and len(want) == 4 and st["walks"] == 4


def test_iteration_cap_reports_non_termination(tmp_path):
    g = pm.rmat_graph(12, 4)
    labels = pmtest.hash_labels(g.n, 8)
    so, sg, diffs = _run_both(g.off, g.col, PATTERNS["cycle"], tmp_path, labels, max_iterations=1)
    assert sg["iterations"] == so["iterations"] == 1
    assert sg["terminated"] == so["terminated"] == 0
    assert diffs == []


def test_cli_end_to_end_matches_oracle(tmp_path):
    import subprocess
    binp = os.path.join(pmtest.ROOT, "fuzzypatternmatching_amd", "csrc", "tools", "bin")
    base = str(tmp_path / "g")
    assert subprocess.run([os.path.join(binp, "generate_rmat"), "-s", "12", "-n", "4", "-o", base]).returncode == 0
    # -v label files (prefix matching: every file named lab.* in the directory)
    g = pm.read_graph(base)
    labels = pmtest.hash_labels(g.n, 8)
    half = g.n // 2
    with open(tmp_path / "lab.0", "w") as f:
        f.write("".join(f"{v} {labels[v]}\n" for v in range(half)))
    with open(tmp_path / "lab.1", "w") as f:
        f.write("".join(f"{v} {labels[v]}\n" for v in range(half, g.n)))
    out = tmp_path / "gpu"
    out.mkdir()
    r = subprocess.run([os.path.join(binp, "run_pattern_matching_beta"), "-i", base, "-v", str(tmp_path / "lab"),
                        "-p", PATTERNS["cycle"], "-o", str(out)], capture_output=True, text=True)
    assert r.returncode == 0, r.stderr
    ora = tmp_path / "oracle"
    oracle.run(g.off, g.col, PATTERNS["cycle"], str(ora), labels=labels, nranks=4)
    assert pmtest.compare_result_dirs(str(ora), str(out), 4) == []


def test_search_start_clears_tpub():
    """Every nonzero T_pub entry (either ping-pong buffer) sits at an slist entry after a search, and the next
    search's start -- the deferred clear batched into its first launch -- leaves both buffers all zero, after
    full, capped and step-API searches alike (the superstep-0 records path writes nothing for a row the first
    later superstep removes, so it relies on clean buffers)."""
    g = pm.rmat_graph(12, 4)
    labels = pmtest.hash_labels(g.n, 8)
    m = pm.PatternMatcher(g, PATTERNS["cycle"], labels=labels)
    try:
        for cap in (0, 1, 0):
            m.run_beta("", max_iterations=cap)
            c0, c1, outside = m.tpub_census()
            assert c0 + c1 > 0 and outside == 0, (c0, c1, outside)
            assert m.tpub_census(deferred_reset=True) == (0, 0, 0)
        m.reset()
        m.lcc_bsp(True)
        m.token_passing(0)
        m.post_token_passing(0)
        assert m.tpub_census()[2] == 0
        assert m.tpub_census(deferred_reset=True) == (0, 0, 0)
        # and the search after it still matches the oracle
        so = oracle.run(g.off, g.col, PATTERNS["cycle"], None, labels=labels)
        sg = m.run_beta("")
        assert (sg["final_vertices"], sg["final_edges"], sg["walks"]) == (so["final_vertices"], so["final_edges"],
                                                                         so["paths"])
    finally:
        m.close()
