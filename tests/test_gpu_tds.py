"""Source-batched, frontier-capped TDS (tds_batch_1.hpp:1139-1253, batch loop at :1181): the exact path
enumerates the walk tree depth-first over chunks of at most PM_TDS_CAP walks per level (run_tds_line), and
the fused line kernel overflows into it when its walk storage would exceed the cap.  Results -- every result
file, the counters and the kept walks' order -- must not depend on the cap."""
import os

import pytest

import fuzzypatternmatching_amd as pm
import oracle
import pmtest

pytestmark = pytest.mark.gpu

CYCLE = os.path.join(pmtest.ROOT, "patterns", "rmat_log2_cycle4_pattern")


def test_tds_cap_invariance_matches_oracle(tmp_path, monkeypatch):
    # hash-label 4-cycle at S=13: 348 k kept walks, millions of partial walks per position -- many times
    # the small caps below
    g = pm.rmat_graph(13, 4)
    labels = pmtest.hash_labels(g.n, 8)
    so = oracle.run(g.off, g.col, CYCLE, str(tmp_path / "oracle"), labels=labels, threads=oracle.default_threads())
    assert so["paths"] > 100000
    digests = {}
    for cap in (None, 65536, 997):
        if cap is None:
            monkeypatch.delenv("PM_TDS_CAP", raising=False)
        else:
            monkeypatch.setenv("PM_TDS_CAP", str(cap))
        out = tmp_path / f"gpu_{cap}"
        m = pm.PatternMatcher(g, CYCLE, labels=labels)
        sg = m.run_beta(str(out), 100)
        m.close()
        assert pmtest.compare_result_dirs(str(tmp_path / "oracle"), str(out), 1) == []
        for k_g, k_o in (("tds_edges", "tds_edges"), ("walks", "paths"), ("nlcc_edges", "nlcc_edges"),
                         ("lcc_edges", "lcc_edges"), ("final_vertices", "final_vertices")):
            assert sg[k_g] == so[k_o], (cap, k_g)
        if cap is not None:  # the fused kernel overflowed into the chunked enumeration, in many chunks
            assert sg["tds_chunks"] > so["paths"] // cap, (cap, sg["tds_chunks"])
        digests[cap] = pmtest.result_digest(str(out), 1)
        print(f"cap {cap}: {sg['tds_chunks']} chunks, {sg['walks']} walks")
    assert digests[None] == digests[65536] == digests[997]


def test_tds_sink_order_is_cap_invariant(monkeypatch):
    # pm_tds streams kept walks chunk by chunk: the same walks in the same order for every cap
    g = pm.rmat_graph(12, 4)
    labels = pmtest.hash_labels(g.n, 8)
    runs = []
    for cap in (None, 4096, 61):
        if cap is None:
            monkeypatch.delenv("PM_TDS_CAP", raising=False)
        else:
            monkeypatch.setenv("PM_TDS_CAP", str(cap))
        m = pm.PatternMatcher(g, CYCLE, labels=labels)
        m.reset()
        m.lcc_bsp(True)
        for pl in range(4):
            m.token_passing(pl)
            m.post_token_passing(pl)
        got = []
        st = m.tds(4, lambda rank, v: got.append((rank, tuple(v))))
        m.close()
        assert st["walks"] == len(got) > 1000
        runs.append(got)
    assert runs[0] == runs[1] == runs[2]
