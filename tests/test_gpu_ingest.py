"""GPU text ingest (pm_ingest.hip) against the host ingest path and the
oracle: edge-list files -> CSR (ingest_edge_list.cpp:164-240, parallel_edge_list_reader.hpp:
242-266) and -v label files (vertex_data_db.hpp:137-257).  Bit-exact: the same offsets,
columns and symmetric flag as the host CLI, the same result files as the host label loader."""
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

# every line kind the reference's `iss >> src >> dst` meets: weights, tabs, CR, blank lines,
# comments, trailing junk after the second number (kept), junk after the first (skipped),
# a '+' sign, a lone number, duplicates and self-loops
EDGE_TEXT_A = ("0 1\n1 2 7\n\t2\t3\r\n\n# a comment\n3 4abc\n5abc 6\n+7 8\n8\n 9   10 w\n10 9\n4 3\n"
               "2 2\n2 2\n0 1\n")
EDGE_TEXT_B = "11 12\n12 11\n6 5"  # no final newline


def _write(tmp_path, name, text):
    p = tmp_path / name
    p.write_bytes(text.encode())
    return str(p)


def _host_cli(files, undirected, base, gpu=None):
    cmd = [os.path.join(BIN, "ingest_edge_list"), "-o", base, "-u", "1" if undirected else "0"]
    if gpu is not None:
        cmd += ["-g", str(gpu)]
    r = subprocess.run(cmd + files, capture_output=True, text=True)
    assert r.returncode == 0, r.stderr
    return pm.read_graph(base)


def _same_graph(a, b):
    assert a.n == b.n
    assert np.array_equal(a.off, b.off)
    assert np.array_equal(a.col, b.col)
    assert a.symmetric == b.symmetric


@pytest.mark.parametrize("undirected", [False, True])
@pytest.mark.parametrize("piece", [None, "64", "100"])
def test_ingest_edge_cases_match_host(undirected, piece, tmp_path, monkeypatch):
    if piece:
        monkeypatch.setenv("PM_INGEST_PIECE", piece)  # lines cross upload pieces
    files = [_write(tmp_path, "a.txt", EDGE_TEXT_A), str(tmp_path / "missing.txt"),
             _write(tmp_path, "empty.txt", ""), _write(tmp_path, "b.txt", EDGE_TEXT_B)]
    host = _host_cli(files, undirected, str(tmp_path / "h"))
    gpu = pm.ingest_edge_list_gpu(files, undirected)
    _same_graph(host, gpu)
    cli = _host_cli(files, undirected, str(tmp_path / "g"), gpu=0)
    _same_graph(host, cli)
    assert host.nnz == (2 if undirected else 1) * 14


def test_ingest_symmetric_detection(tmp_path):
    text = "0 1\n1 0\n1 2\n2 1\n2 2\n"
    g = pm.ingest_edge_list_gpu([_write(tmp_path, "s.txt", text)], False)
    assert g.symmetric
    g = pm.ingest_edge_list_gpu([_write(tmp_path, "t.txt", text + "1 2\n")], False)  # multiplicity differs
    assert not g.symmetric


def test_ingest_refuses_wide_ids(tmp_path):
    for bad in ("0 4294967295\n", "-1 2\n"):
        with pytest.raises(pm.PMError, match="32 bits"):
            pm.ingest_edge_list_gpu([_write(tmp_path, "w.txt", bad)], False)


def test_ingest_empty(tmp_path):
    g = pm.ingest_edge_list_gpu([_write(tmp_path, "e.txt", "\n# nothing\n")], True)
    assert g.n == 0 and g.nnz == 0


def _rmat_text(tmp_path, scale, p_gen, nfiles=3):
    """The generator's undirected pairs as text, split over nfiles files."""
    und = [oracle.rmat_rank_edges(scale, p_gen, r) for r in range(p_gen)]
    u = np.concatenate([x[0] for x in und]).astype(np.uint64)
    v = np.concatenate([x[1] for x in und]).astype(np.uint64)
    files = []
    for i, part in enumerate(np.array_split(np.arange(u.shape[0]), nfiles)):
        p = tmp_path / f"rmat_{i}.txt"
        np.savetxt(p, np.stack([u[part], v[part]], 1), fmt="%d")
        files.append(str(p))
    return files, u, v


def test_ingest_rmat_text_equals_generator(tmp_path):
    """-u 1 over the R-MAT stream written as text == generate_rmat's symmetrized graph."""
    files, _, _ = _rmat_text(tmp_path, 16, 4)
    g = pm.ingest_edge_list_gpu(files, True)
    ref = pm.rmat_graph(16, 4)
    # ids above the largest one that occurs are not rows of the ingested graph
    assert g.n <= ref.n
    assert np.array_equal(g.off, ref.off[: g.n + 1])
    assert np.array_equal(g.col, ref.col)
    assert g.symmetric


@pytest.mark.parametrize("undirected,pattern", [(True, TREE), (False, TREE), (False, CYCLE)])
def test_edge_list_matcher_matches_oracle(undirected, pattern, tmp_path):
    """pm_create_edge_list: text -> HBM CSR (and in-rows for a directed graph) -> search."""
    files, u, v = _rmat_text(tmp_path, 14, 2)
    m, secs = pm.edge_list_matcher(files, pattern, undirected=undirected)
    assert secs > 0
    assert m.graph.symmetric == undirected
    sg = m.run_beta(str(tmp_path / "gpu"))
    n = m.graph.n
    m.close()
    if undirected:
        off, col = pmtest.csr_from_edges(np.concatenate([u, v]), np.concatenate([v, u]), n)
    else:
        off, col = pmtest.csr_from_edges(u, v, n)
    so = oracle.run(off, col, pattern, str(tmp_path / "oracle"), threads=oracle.default_threads())
    assert pmtest.compare_result_dirs(str(tmp_path / "oracle"), str(tmp_path / "gpu"), 1) == []
    for k_g, k_o in (("final_vertices", "final_vertices"), ("final_edges", "final_edges"),
                     ("lcc_edges", "lcc_edges"), ("nlcc_edges", "nlcc_edges"), ("tds_edges", "tds_edges")):
        assert sg[k_g] == so[k_o], (k_g, sg[k_g], so[k_o])


def _label_files(tmp_path, n, alphabet):
    """Hash labels over two files plus overrides: a later file wins, a blank line and an
    unparsable line set label 0 on vertex 0, a vid >= n is ignored, '12abc' sets vertex 12 to 0."""
    lab = pmtest.hash_labels(n, alphabet)
    d = tmp_path / "labels"
    d.mkdir()
    half = n // 2
    with open(d / "vl.0", "w") as f:
        for v in range(half):
            f.write(f"{v} {lab[v]}\n")
        f.write(f"{n + 5} 3\n")
    with open(d / "vl.1", "w") as f:
        for v in range(half, n):
            f.write(f"{v}\t{lab[v]}\r\n")
        f.write("\n")            # -> vertex 0 label 0
        f.write("12abc\n")       # -> vertex 12 label 0
        f.write(f"7 {int(lab[7]) + 1}\n")  # later line wins
        f.write("x y")           # -> vertex 0 label 0, no final newline
    with open(d / "other_file", "w") as f:  # does not match the prefix
        f.write("1 99\n")
    want = lab.copy()
    want[0] = 0
    want[12] = 0
    want[7] = int(lab[7]) + 1
    return str(d / "vl"), want


@pytest.mark.parametrize("piece", [None, "64"])
def test_label_files_match_host_loader(piece, tmp_path, monkeypatch):
    if piece:
        monkeypatch.setenv("PM_INGEST_PIECE", piece)
    scale = 12
    g = pm.rmat_graph(scale, 2)
    prefix, want = _label_files(tmp_path, g.n, 8)
    m = pm.PatternMatcher(g, CYCLE)
    m.labels_from_files(prefix)
    sg = m.run_beta(str(tmp_path / "gpu"))
    m.close()
    so = oracle.run(g.off, g.col, CYCLE, str(tmp_path / "oracle"), labels=want)
    assert pmtest.compare_result_dirs(str(tmp_path / "oracle"), str(tmp_path / "gpu"), 1) == []
    assert sg["final_vertices"] == so["final_vertices"] and sg["final_edges"] == so["final_edges"]


def test_beta_cli_gpu_labels_equal_host_labels(tmp_path):
    """run_pattern_matching_beta -v: GPU label parse (default) == host loader (PM_HOST_LABELS=1)."""
    g = pm.rmat_graph(12, 2)
    base = str(tmp_path / "g")
    pm.write_graph(base, g, 2)
    prefix, _ = _label_files(tmp_path, g.n, 8)
    outs = []
    for host in (False, True):
        out = tmp_path / ("host" if host else "gpu")
        out.mkdir()
        env = dict(os.environ)
        if host:
            env["PM_HOST_LABELS"] = "1"
        r = subprocess.run([os.path.join(BIN, "run_pattern_matching_beta"), "-i", base, "-p", CYCLE, "-o", str(out),
                            "-v", prefix], capture_output=True, text=True, env=env)
        assert r.returncode == 0, r.stderr
        outs.append(str(out))
    assert pmtest.compare_result_dirs(outs[1], outs[0], 2) == []
