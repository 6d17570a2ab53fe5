"""pattern_selected_vertices (NLC field 6; nem_1.hpp:155-170, 409-436, 697-719;
run_pattern_matching_beta.cpp:791-850, 959-1000) on the GPU against the oracle:
token-source sets carried from the previous line, the verified vertices' bit
cleared when unconfirmed.  patterns/selected_vertices_pattern (README there)."""
import os

import numpy as np
import pytest

import fuzzypatternmatching_amd as pm
import oracle
import pmtest

pytestmark = pytest.mark.gpu

SV = os.path.join(pmtest.ROOT, "patterns", "selected_vertices_pattern")


def _check(off, col, tmp_path, labels, nranks=1, shards=0):
    a, b = tmp_path / "oracle", tmp_path / "gpu"
    so = oracle.run(off, col, SV, str(a), labels=labels, nranks=nranks, threads=oracle.default_threads())
    g = pm.Graph(off, col, True, nranks)
    if shards:
        sg = pm.run_beta_local_shards(g, SV, shards, str(b), labels=labels)
    else:
        m = pm.PatternMatcher(g, SV, labels=labels)
        sg = m.run_beta(str(b))
        m.close()
    assert pmtest.compare_result_dirs(str(a), str(b), nranks) == []
    for k_g, k_o in (("iterations", "iterations"), ("final_vertices", "final_vertices"),
                     ("final_edges", "final_edges"), ("lcc_edges", "lcc_edges"), ("nlcc_edges", "nlcc_edges")):
        assert sg[k_g] == so[k_o], (k_g, sg[k_g], so[k_o])
    return sg


def test_selected_vertices_known_answers(tmp_path):
    # tests/test_cpu_oracle.py::test_oracle_selected_vertices_known_answer, hand-derived there
    pairs = [(3, 2), (2, 0), (0, 1), (1, 3), (6, 5), (5, 4), (4, 1)]
    off, col = pmtest.symmetric_csr(pairs, 7)
    sg = _check(off, col, tmp_path / "a", np.array([5, 6, 4, 3, 5, 4, 3], np.uint64))
    assert sg["final_vertices"] == 4 and sg["final_edges"] == 8
    pairs = [(0, 1), (1, 2), (2, 3), (3, 0), (4, 5), (5, 6), (6, 3)]
    off, col = pmtest.symmetric_csr(pairs, 7)
    sg = _check(off, col, tmp_path / "b", np.array([3, 4, 5, 6, 3, 4, 5], np.uint64))
    assert sg["final_vertices"] == 0


@pytest.mark.parametrize("scale,p_gen,alphabet,nranks,shards", [
    (10, 1, 8, 1, 0), (12, 4, 8, 2, 0), (14, 4, None, 1, 0), (13, 2, 16, 1, 0), (12, 4, 8, 1, 3)])
def test_selected_vertices_rmat(scale, p_gen, alphabet, nranks, shards, tmp_path):
    g = pm.rmat_graph(scale, p_gen)
    labels = None if alphabet is None else pmtest.hash_labels(g.n, alphabet, salt=3)
    _check(g.off, g.col, tmp_path, labels, nranks, shards)
