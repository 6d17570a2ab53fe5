"""GPU R-MAT generator (pm_rmat.hip): bit-identical to the host restatement of
generate_rmat (host/rmat.hpp, itself checked against the oracle and the
reference's hash_nbits vectors) for every scale / P_gen / substream split."""
import numpy as np
import pytest

import fuzzypatternmatching_amd as pm
import oracle

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("scale,p_gen", [(5, 1), (9, 1), (12, 3), (16, 4), (17, 2), (20, 4)])
def test_gpu_rmat_equals_host(scale, p_gen):
    h = pm.rmat_graph(scale, p_gen)
    g = pm.rmat_graph(scale, p_gen, device=0)
    assert g.n == h.n == 1 << scale
    assert np.array_equal(g.off, h.off)
    assert np.array_equal(g.col, h.col)


def test_gpu_rmat_equals_oracle_stream():
    # the oracle's own MT19937 / hash restatement (independent of the product's host code)
    off, col = oracle.rmat_csr(14, 4)
    g = pm.rmat_graph(14, 4, device=0)
    assert np.array_equal(g.off, off) and np.array_equal(g.col, col)


def test_device_resident_matcher_matches_host_graph(tree_pattern):
    # pm_create_rmat (adjacency generated in HBM) == pm_create over the host-built graph
    m, secs = pm.rmat_matcher(16, 4, tree_pattern)
    a = m.run_beta()
    m.close()
    g = pm.rmat_graph(16, 4)
    m2 = pm.PatternMatcher(g, tree_pattern)
    b = m2.run_beta()
    m2.close()
    for k in ("iterations", "lcc_edges", "nlcc_edges", "tds_edges", "walks", "final_vertices", "final_edges"):
        assert a[k] == b[k], k
