"""SURVEY.md A.6 hazards on the CPU oracle, each checked on its own input.

Hand-derived (expected lines worked out by hand, see the docstrings / pattern READMEs):
  3  M entries to vertices removed in the same verify are counted one superstep
     (tests/test_cpu_oracle.py::test_oracle_selected_vertices_known_answer: "0, LP, 0, 13"
     includes b2's entry for a2, removed in that verify);
  4, 5, 9  the NLCC clear touches T_pub only, TN |= before the edge check, the cycle
     terminal's edge flag survives into the next verify (tests/test_gpu_directed.py
     ::test_asymmetric_active_edge_map, patterns/triangle_tail_pattern/README.md);
  1  exactly D supersteps per LCC call (below).
  6  subgraph files are reopened with truncation in every iteration that runs token
     passing: only the last such iteration's walks survive (below,
     patterns/triangle_tail_tds_pattern/README.md).
Property-checked on small R-MAT inputs found by a bounded search (the GPU path is
compared file by file with the oracle on the same inputs in tests/test_gpu_*.py):
  7  interleaved LCC calls reuse the iteration number in their LP lines;
  11 non-termination is reported by the iteration cap, not hidden.
"""
import os

import numpy as np
import pytest

import fuzzypatternmatching_amd as pm
import oracle
import pmtest

CYCLE = os.path.join(pmtest.ROOT, "patterns", "rmat_log2_cycle4_pattern")
TREE = os.path.join(pmtest.ROOT, "patterns", "rmat_log2_tree_pattern")


def _lines(d, *parts):
    with open(os.path.join(d, *parts)) as f:
        return [l for l in f.read().split("\n") if l]


def test_hazard1_exactly_diameter_supersteps(tmp_path):
    # a single edge whose labels match nothing: every LCC call still runs D = 8 supersteps
    off, col = pmtest.symmetric_csr([(0, 1)], 2)
    oracle.run(off, col, TREE, str(tmp_path), labels=np.array([1, 1], np.uint64))
    lp = [l for l in _lines(tmp_path, "0", "result_superstep") if ", LP, " in l]
    assert [l.split(", ")[2] for l in lp] == [str(i) for i in range(8)]


def _search(pred, patterns=(CYCLE,), scales=(8, 9), alphabets=(6, 8), salts=range(6), max_iterations=100):
    import tempfile
    for pat in patterns:
        for scale in scales:
            g = pm.rmat_graph(scale, 2)
            for alpha in alphabets:
                for salt in salts:
                    labels = pmtest.hash_labels(g.n, alpha, salt=salt)
                    d = tempfile.mkdtemp()
                    so = oracle.run(g.off, g.col, pat, d, labels=labels, max_iterations=max_iterations)
                    if pred(d, so):
                        return d, so
    return None, None


def test_hazard7_interleaved_lcc_reuses_iteration():
    # cycle4 lines have interleave_lp = 1: a deleting line is followed by an LCC call
    # whose LP lines carry the same itr (beta.cpp:1163-1197; global_itr_count unchanged)
    def pred(d, so):
        steps = [l.split(", ")[:2] for l in _lines(d, "0", "result_step")]
        lp = [s[0] for s in steps if s[1] == "LP"]
        return any(lp.count(i) > 1 for i in set(lp))
    d, so = _search(pred)
    assert d, "no interleaved LCC call found"
    steps = [l.split(", ")[:2] for l in _lines(d, "0", "result_step")]
    itrs = [int(s[0]) for s in steps]
    assert itrs == sorted(itrs) and max(itrs) == so["iterations"] - 1


TDS_TAIL = os.path.join(pmtest.ROOT, "patterns", "triangle_tail_tds_pattern")


def test_hazard6_subgraph_files_hold_the_last_iteration(tmp_path):
    # hand-derived in patterns/triangle_tail_tds_pattern/README.md: iteration 0's
    # enumeration (line 4) writes four triangles, line 5 then strips vertices 6 and 9
    # of bit 0, iteration 1 removes their triangles and reopens subgraphs_4_0 with
    # truncation (beta.cpp:713-717): only triangles 0 and 1 are left in the file
    off, col = pmtest.symmetric_csr([(3 * t + a, 3 * t + b) for t in range(4) for a, b in ((0, 1), (1, 2), (0, 2))]
                                    + [(1, 3), (7, 10)], 12)
    labels = np.array([3, 4, 5] * 4, np.uint64)
    tri = lambda ts: sorted(f"[0], {3 * t}, {3 * t + 1}, {3 * t + 2}, {3 * t}, [{3 * t}]" for t in ts)
    first = oracle.run(off, col, TDS_TAIL, str(tmp_path / "a"), labels=labels, max_iterations=1)
    assert first["iterations"] == 1
    assert sorted(_lines(tmp_path / "a", "0", "all_ranks_subgraphs", "subgraphs_4_0")) == tri(range(4))
    full = oracle.run(off, col, TDS_TAIL, str(tmp_path / "b"), labels=labels)
    tp = [l.split(", ")[:3] for l in _lines(tmp_path / "b", "0", "result_superstep") if ", TP, " in l]
    assert ["1", "TP", "4"] in tp and full["iterations"] == 2 and full["final_vertices"] == 6
    assert sorted(_lines(tmp_path / "b", "0", "all_ranks_subgraphs", "subgraphs_4_0")) == tri(range(2))
    assert sorted(_lines(tmp_path / "b", "0", "all_ranks_subgraphs", "subgraphs_5_0")) == \
        ["[0], 0, 1, 3, [3]", "[0], 3, 1, 0, [0]"]


def test_hazard11_non_termination_is_reported(tmp_path):
    # an iteration cap stops a search that would go on and reports terminated = 0
    g = pm.rmat_graph(12, 4)
    labels = pmtest.hash_labels(g.n, 8)
    so = oracle.run(g.off, g.col, CYCLE, str(tmp_path), labels=labels, max_iterations=1)
    assert so["iterations"] == 1 and so["terminated"] == 0
    full = oracle.run(g.off, g.col, CYCLE, None, labels=labels, max_iterations=100)
    assert full["iterations"] > 1


@pytest.mark.skipif(not os.path.exists("/usr/bin/g++") and not os.path.exists("/usr/bin/c++"), reason="no host g++")
def test_oracle_under_asan_ubsan():
    # SURVEY.md section 5 (race / memory checking): the oracle and its CSR driver built
    # with -fsanitize=address,undefined run the tree and 4-cycle patterns, one and four
    # threads, with no report (any finding aborts with a non-zero status)
    import subprocess
    odir = os.path.join(pmtest.ROOT, "oracle")
    r = subprocess.run(["make", "-s", "-C", odir, "sanitize"], capture_output=True, text=True)
    assert r.returncode == 0, r.stderr
    exe = os.path.join(odir, "_san", "oracle_main")
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=1", UBSAN_OPTIONS="halt_on_error=1")
    for args in (["10", "2", TREE, "1"], ["10", "2", TREE, "4"], ["9", "2", CYCLE, "4", "8"]):
        r = subprocess.run([exe] + args, capture_output=True, text=True, env=env, timeout=300)
        assert r.returncode == 0, (args, r.stderr[-2000:])
