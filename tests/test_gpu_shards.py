"""GPU parity of the sharded search against the CPU oracle.

The shards run as threads of this process on the one device of the test box
(pm_run_beta_local_shards: the partitioning, tiling and exchanges of the
multi-GPU path with an in-process Comm in place of RCCL); the RCCL Comm itself
is exercised with one rank (pm_create_shard).  Results must equal the oracle's
for every shard count."""
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
    # one label on three template vertices: the wide code exchange (64-bit records, T_pub by position)
    "wstar": os.path.join(pmtest.ROOT, "patterns", "wide_star_pattern"),      # diameter 2
    "wspider": os.path.join(pmtest.ROOT, "patterns", "wide_spider_pattern"),  # diameter 3
    # cycle flags that break M's symmetry (push-form later LCC calls, hazards 4, 5, 9)
    "triangle": os.path.join(pmtest.ROOT, "patterns", "triangle_tail_pattern"),
}

# (pattern, scale, P_gen, label alphabet or None, result-file ranks, shards)
SHARD_CASES = [
    ("tree", 14, 4, None, 1, 2),
    ("tree", 16, 4, None, 4, 3),
    ("cycle", 12, 4, 8, 3, 2),
    ("cycle", 14, 4, None, 1, 4),
    ("tree", 10, 1, 16, 1, 4),
    ("cycle", 10, 1, 8, 2, 1),
]


def _check(so, sg):
    assert sg["iterations"] == so["iterations"] and sg["terminated"] == so["terminated"]
    assert sg["final_vertices"] == so["final_vertices"] and sg["final_edges"] == so["final_edges"]
    assert sg["lcc_edges"] == so["lcc_edges"]
    assert sg["nlcc_edges"] == so["nlcc_edges"]
    assert sg["tds_edges"] == so["tds_edges"]
    assert sg["walks"] == so["paths"]


def _run_both(off, col, pattern, tmp_path, shards, labels=None, nranks=1, max_iterations=100,
              hub_threshold=pm.DEFAULT_HUB_THRESHOLD):
    a, b = tmp_path / "oracle", tmp_path / "shards"
    so = oracle.run(off, col, pattern, str(a), labels=labels, nranks=nranks, max_iterations=max_iterations,
                    hub_threshold=hub_threshold)
    g = pm.Graph(off, col, True, nranks, hub_threshold)
    sg = pm.run_beta_local_shards(g, pattern, shards, str(b), max_iterations=max_iterations, labels=labels)
    return so, sg, pmtest.compare_result_dirs(str(a), str(b), nranks)


@pytest.mark.parametrize("pat,scale,p_gen,alphabet,nranks,shards", SHARD_CASES)
def test_sharded_rmat_matches_oracle(pat, scale, p_gen, alphabet, nranks, shards, tmp_path):
    g = pm.rmat_graph(scale, p_gen)
    labels = None if alphabet is None else pmtest.hash_labels(g.n, alphabet)
    so, sg, diffs = _run_both(g.off, g.col, PATTERNS[pat], tmp_path, shards, labels, nranks)
    assert diffs == []
    _check(so, sg)


# delegates: rows of degree >= -d split over the shards by target owner, combined at the controller
# (hub ordinal % shards); small thresholds so that hubs carry pattern labels (tree: label 7 = degree 64..127)
DELEGATE_CASES = [
    ("tree", 16, 4, 64, 4, 4),
    ("tree", 15, 4, 100, 1, 3),
    ("cycle", 13, 4, 16, 2, 2),
    ("tree", 14, 1, 32, 3, 5),
]


@pytest.mark.parametrize("pat,scale,p_gen,thr,nranks,shards", DELEGATE_CASES)
def test_sharded_delegates_match_oracle(pat, scale, p_gen, thr, nranks, shards, tmp_path):
    g = pm.rmat_graph(scale, p_gen)
    assert int((np.diff(g.off) >= thr).sum()) > 0  # some delegates
    so, sg, diffs = _run_both(g.off, g.col, PATTERNS[pat], tmp_path, shards, None, nranks, hub_threshold=thr)
    assert diffs == []
    _check(so, sg)


# labels on three template vertices (xcode_wide): diameters 2 and 3, two and three shards, with delegates
WIDE_CASES = [
    ("wstar", 12, 4, 6, 64, 1, 2),
    ("wstar", 14, 4, 8, 100, 2, 3),
    ("wspider", 12, 4, 6, 48, 1, 3),
    ("wspider", 14, 4, 8, 100, 3, 2),
    ("wstar", 13, 4, 6, pm.DEFAULT_HUB_THRESHOLD, 1, 1),
]


@pytest.mark.parametrize("pat,scale,p_gen,alphabet,thr,nranks,shards", WIDE_CASES)
def test_sharded_wide_codes_match_oracle(pat, scale, p_gen, alphabet, thr, nranks, shards, tmp_path):
    g = pm.rmat_graph(scale, p_gen)
    labels = pmtest.hash_labels(g.n, alphabet)
    so, sg, diffs = _run_both(g.off, g.col, PATTERNS[pat], tmp_path, shards, labels, nranks, hub_threshold=thr)
    assert diffs == []
    _check(so, sg)
    assert so["final_vertices"] > 0 and so["nlcc_edges"] > 0
    if thr < pm.DEFAULT_HUB_THRESHOLD:
        assert sg["hubs"] > 0


@pytest.mark.parametrize("pat", ["wstar", "wspider"])
def test_wide_codes_one_gpu_match_oracle(pat, tmp_path):
    g = pm.rmat_graph(13, 4)
    labels = pmtest.hash_labels(g.n, 6)
    so = oracle.run(g.off, g.col, PATTERNS[pat], str(tmp_path / "oracle"), labels=labels)
    m = pm.PatternMatcher(pm.Graph(g.off, g.col, True), PATTERNS[pat], labels=labels)
    sg = m.run_beta(str(tmp_path / "gpu"), 100)
    assert m.tpub_census()[2] == 0
    m.close()
    assert pmtest.compare_result_dirs(str(tmp_path / "oracle"), str(tmp_path / "gpu"), 1) == []
    _check(so, sg)


# split NLC lines (PM_SPLIT_LINES=1: every line with a source runs split by owner, its effects exchanged):
# (pattern, scale, P_gen, alphabet, result ranks, shards, hub threshold, TDS cap forcing the exact-path rerun)
SPLIT_CASES = [
    ("cycle", 12, 4, 8, 3, 2, pm.DEFAULT_HUB_THRESHOLD, None),
    ("cycle", 14, 4, None, 1, 3, pm.DEFAULT_HUB_THRESHOLD, None),
    ("tree", 16, 4, None, 4, 4, 64, None),
    ("cycle", 13, 4, 16, 2, 2, 16, None),
    ("cycle", 12, 4, 8, 2, 3, pm.DEFAULT_HUB_THRESHOLD, 997),
    ("triangle", 12, 4, 6, 1, 2, pm.DEFAULT_HUB_THRESHOLD, None),
    ("wspider", 12, 4, 6, 1, 2, pm.DEFAULT_HUB_THRESHOLD, None),
]


@pytest.mark.parametrize("pat,scale,p_gen,alphabet,nranks,shards,thr,cap", SPLIT_CASES)
def test_split_lines_match_oracle(pat, scale, p_gen, alphabet, nranks, shards, thr, cap, tmp_path, monkeypatch):
    monkeypatch.setenv("PM_SPLIT_LINES", "1")
    if cap:
        monkeypatch.setenv("PM_TDS_CAP", str(cap))
    g = pm.rmat_graph(scale, p_gen)
    labels = None if alphabet is None else pmtest.hash_labels(g.n, alphabet)
    so, sg, diffs = _run_both(g.off, g.col, PATTERNS[pat], tmp_path, shards, labels, nranks, hub_threshold=thr)
    assert diffs == []
    _check(so, sg)
    assert so["nlcc_edges"] + so["tds_edges"] > 0


@pytest.mark.parametrize("nogrow", [None, 1])
def test_split_line_overflow_agreed(nogrow, tmp_path, monkeypatch):
    """A split line overflows a tiny (source, vertex) table on every shard (the table and the arena have one
    size on every shard), and the shards agree whether to grow it: with room on all of them every shard reruns
    the line fused and split (its collectives); with PM_DEBUG_NOGROW_SHARD=1 shard 1 has no room, so every
    shard takes the exact path (no collectives) -- a shard-local decision hung the split line's all-gathers."""
    monkeypatch.setenv("PM_SPLIT_LINES", "1")
    monkeypatch.setenv("PM_HASH_SLOTS", "1024")
    if nogrow is not None:
        monkeypatch.setenv("PM_DEBUG_NOGROW_SHARD", str(nogrow))
    g = pm.rmat_graph(12, 4)
    labels = pmtest.hash_labels(g.n, 8)
    so, sg, diffs = _run_both(g.off, g.col, PATTERNS["cycle"], tmp_path, 3, labels, 2)
    assert diffs == []
    _check(so, sg)
    assert sg["line_overflows"] > 0
    if nogrow is None:
        assert sg["split_lines"] > 0
    else:
        assert sg["exact_lines"] > 0


def test_sharded_exact_count_lines(tmp_path, monkeypatch):
    monkeypatch.setenv("PM_FUSED_LINES", "0")
    g = pm.rmat_graph(12, 4)
    labels = pmtest.hash_labels(g.n, 8)
    so, sg, diffs = _run_both(g.off, g.col, PATTERNS["cycle"], tmp_path, 3, labels, 3)
    assert diffs == []
    _check(so, sg)


def test_sharded_known_answers(tmp_path):
    # tiny graphs: most shards own no state-map vertex at all
    pairs = [(0, 1), (1, 2), (1, 3), (3, 5), (4, 5), (5, 6)]
    labels = np.array([3, 4, 7, 2, 3, 5, 7], np.uint64)
    off, col = pmtest.symmetric_csr(pairs, 7)
    for shards in (2, 5):
        so, sg, diffs = _run_both(off, col, PATTERNS["tree"], tmp_path / str(shards), shards, labels)
        assert diffs == []
        assert sg["final_vertices"] == 7 and sg["walks"] == 1
    off0 = np.zeros(9, np.uint64)
    so, sg, diffs = _run_both(off0, np.zeros(0, np.uint32), PATTERNS["tree"], tmp_path / "empty", 3,
                              np.full(8, 3, np.uint64))
    assert diffs == [] and sg["final_vertices"] == 0


def test_sharded_non_termination_cap(tmp_path):
    g = pm.rmat_graph(12, 4)
    labels = pmtest.hash_labels(g.n, 8)
    so, sg, diffs = _run_both(g.off, g.col, PATTERNS["cycle"], tmp_path, 2, labels, max_iterations=1)
    assert diffs == []
    assert sg["terminated"] == so["terminated"] == 0


def test_rccl_shard_single_rank(tmp_path):
    # pm_create_shard with one rank: the RCCL communicator carries every
    # exchange of the sharded driver (all-gathers and all-reduces of one rank)
    g = pm.rmat_graph(12, 4)
    deg = np.diff(g.off).astype(np.uint32)
    uid = pm.comm_unique_id()
    assert len(uid) >= 128
    m = pm.ShardedPatternMatcher(g.n, g.off, g.col, deg, PATTERNS["tree"], 1, 0, uid, nranks=2)
    sg = m.run_beta(str(tmp_path / "rccl"), max_iterations=100)
    m.close()
    so = oracle.run(g.off, g.col, PATTERNS["tree"], str(tmp_path / "oracle"), nranks=2, max_iterations=100)
    assert pmtest.compare_result_dirs(str(tmp_path / "oracle"), str(tmp_path / "rccl"), 2) == []
    _check(so, sg)


# the GPU-generated sharded input (pm_run_rmat_local_shards): each shard draws its generator
# ranks' streams on the device, the entries reach their owners (delegates by target) in one
# all-to-all; results equal the oracle's on the one-GPU graph for every shard count
@pytest.mark.parametrize("scale,p_gen,shards,thr,nranks", [(14, 4, 2, pm.DEFAULT_HUB_THRESHOLD, 1),
                                                           (15, 4, 4, 64, 4), (14, 8, 3, 48, 2)])
def test_gpu_generated_shards_match_oracle(scale, p_gen, shards, thr, nranks, tmp_path):
    g = pm.rmat_graph(scale, p_gen)
    a, b = tmp_path / "oracle", tmp_path / "shards"
    so = oracle.run(g.off, g.col, PATTERNS["tree"], str(a), nranks=nranks, hub_threshold=thr, max_iterations=100)
    sg = pm.run_rmat_local_shards(scale, p_gen, PATTERNS["tree"], shards, str(b), max_iterations=100, nranks=nranks,
                                  hub_threshold=thr)
    assert pmtest.compare_result_dirs(str(a), str(b), nranks) == []
    _check(so, sg)


def test_rccl_rmat_shard_single_rank(tmp_path):
    # pm_create_rmat_shard with one RCCL rank: the bench's N-GPU construction path at N = 1
    uid = pm.comm_unique_id()
    m, secs = pm.rmat_shard_matcher(14, 4, PATTERNS["tree"], 1, 0, uid, nranks=2)
    sg = m.run_beta(str(tmp_path / "rccl"), max_iterations=100)
    m.close()
    g = pm.rmat_graph(14, 4)
    so = oracle.run(g.off, g.col, PATTERNS["tree"], str(tmp_path / "oracle"), nranks=2, max_iterations=100)
    assert pmtest.compare_result_dirs(str(tmp_path / "oracle"), str(tmp_path / "rccl"), 2) == []
    _check(so, sg)
