"""GPU parity at the BASELINE.json configurations (SURVEY.md 8(d) C2, C3, C4 on
one GPU, C5): every result file of the HIP path compared with the oracle (run on
all host threads) on the same R-MAT input, or with the oracle's committed S=28
result digest.

C2: S=24, P_gen=4, tree, degree labels, 1 and 4 ranks of output attribution.
C3: S=26, P_gen=4, 4-cycle pattern (NLCC token-passing stress).
C5: ingested text edge list (-u 1) + explicit -v label files (hash32(v) % 64)
    through the CLIs at S=18 (text size), hash labels through the library at
    S=22, and at size (S=27, alphabet 256, GPU ingest, chunked TDS, one context and
    8 in-process shards, against the oracle's S=27 digest).
C4': S=28, P_gen=8, tree on ONE GPU against tests/golden/rmat_s28_p8_tree.json
    (the oracle needs ~100 GB of host memory there, so its result was made once:
    tests/golden/make_rmat_fixture.py), and C4's sharded path at full size (2, 4 and
    8 in-process shards, delegates at -d 1048576) against the same fixture.
C5 at S=27 on the GPU-generated graph (hash-256 labels, 4-cycle), four and eight
    shards (every line split by owner), against tests/golden/rmat_s27_p8_cycle4_hash256.json.
"""
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

_graphs = {}


def _graph(scale, p_gen):
    # GPU generator (bit-identical to the host stream, tests/test_gpu_rmat.py), one copy per session
    key = (scale, p_gen)
    if key not in _graphs:
        _graphs.clear()
        _graphs[key] = pm.rmat_graph(scale, p_gen, device=0)
    return _graphs[key]


def _check(g, pattern, tmp_path, labels=None, nranks=1, tag=""):
    a, b = tmp_path / f"oracle{tag}", tmp_path / f"gpu{tag}"
    so = oracle.run(g.off, g.col, pattern, str(a), labels=labels, nranks=nranks, threads=oracle.default_threads())
    m = pm.PatternMatcher(pm.Graph(g.off, g.col, True, nranks), pattern, labels=labels)
    sg = m.run_beta(str(b))
    m.close()
    diffs = pmtest.compare_result_dirs(str(a), str(b), nranks)
    assert diffs == [], diffs[:5]
    for k_g, k_o in (("iterations", "iterations"), ("terminated", "terminated"), ("final_vertices", "final_vertices"),
                     ("final_edges", "final_edges"), ("lcc_edges", "lcc_edges"), ("nlcc_edges", "nlcc_edges"),
                     ("tds_edges", "tds_edges"), ("walks", "paths")):
        assert sg[k_g] == so[k_o], (k_g, sg[k_g], so[k_o])
    return sg


@pytest.mark.parametrize("nranks", [1, 4])
def test_c2_s24_tree(nranks, tmp_path):
    sg = _check(_graph(24, 4), TREE, tmp_path, nranks=nranks)
    assert sg["lcc_edges"] > 10 ** 8  # superstep 0 scans every label-matching row


def test_c3_s26_cycle4(tmp_path):
    sg = _check(_graph(26, 4), CYCLE, tmp_path)
    assert sg["nlcc_edges"] + sg["tds_edges"] > 0


def test_c5_s22_hash_labels(tmp_path):
    g = _graph(22, 4)
    # alphabet 64: with 8 labels the 4-cycle walks through R-MAT hubs explode
    # (S=14 already enumerates 1.2 M walks, S=16 runs for minutes on the oracle)
    labels = pmtest.hash_labels(g.n, 64)
    sg = _check(g, CYCLE, tmp_path, labels=labels, nranks=2)
    assert sg["walks"] > 0


def test_c5_ingested_edge_list_with_label_files(tmp_path):
    """generate -> text edge list -> ingest_edge_list -u 1 -> -v label files -> run_pattern_matching_beta."""
    scale, p_gen, nranks = 18, 4, 4
    und = [oracle.rmat_rank_edges(scale, p_gen, r) for r in range(p_gen)]
    u = np.concatenate([x[0] for x in und])
    v = np.concatenate([x[1] for x in und])
    txt = tmp_path / "edges.txt"
    np.savetxt(txt, np.stack([u, v], 1), fmt="%d")
    base = str(tmp_path / "ing")
    r = subprocess.run([os.path.join(BIN, "ingest_edge_list"), "-o", base, "-u", "1", "-n", str(nranks), str(txt)],
                       capture_output=True, text=True)
    assert r.returncode == 0, r.stderr
    g = pm.read_graph(base)
    assert g.symmetric
    # the ingested graph is the R-MAT graph (ids up to the max id seen)
    h = _graph(scale, p_gen)
    assert np.array_equal(g.col, h.col) and np.array_equal(g.off, h.off[: g.n + 1])
    labels = pmtest.hash_labels(g.n, 64, salt=5)
    for i, part in enumerate(np.array_split(np.arange(g.n), 3)):
        with open(tmp_path / f"lab.{i}", "w") as f:
            f.write("".join(f"{x} {labels[x]}\n" for x in part))
    out = tmp_path / "gpu"
    out.mkdir()
    r = subprocess.run([os.path.join(BIN, "run_pattern_matching_beta"), "-i", base, "-v", str(tmp_path / "lab"),
                        "-p", CYCLE, "-o", str(out)], capture_output=True, text=True)
    assert r.returncode == 0, r.stderr
    ora = tmp_path / "oracle"
    oracle.run(g.off, g.col, CYCLE, str(ora), labels=labels, nranks=nranks, threads=oracle.default_threads())
    assert pmtest.compare_result_dirs(str(ora), str(out), nranks) == []


C5_ALPHABET = 256


def test_c5_s27_ingested_label_files(tmp_path, monkeypatch):
    """BASELINE config C5 at size on one GPU: the S=27 R-MAT stream (P_gen=8) as 8 text edge-list files
    (~40 GB, written from the GPU generator's stream) ingested on the GPU with -u 1 (ingest_edge_list.cpp:164-240,
    parallel_edge_list_reader.hpp:242-266), explicit -v label files with hash32(v ^ 5) % 256 parsed on the GPU
    (vertex_data_db.hpp:137-257), and the 4-cycle pattern, whose template-driven enumeration runs in chunks
    (tds_batch_1.hpp:1139-1253).  Checks: the ingested graph's result equals the oracle's S=27 digest of the same
    graph and labels (tests/golden/rmat_s27_p8_cycle4_hash256.json: the oracle on the generated graph's host CSR,
    made by make_rmat_fixture.py -- ingest == generate is checked bit for bit at S=18 above); the result does not
    depend on the TDS chunk cap; and C5 as BASELINE runs it, an 8-way partition: the ingested CSR as 8 in-process
    shards (delegates split by target owner, NLC lines split by owner) with the -v files parsed once on the device
    (pm_run_beta_local_shards2, the drop-in executable's path for 8 partitions on one GPU) gives the same result.
    (An alphabet of 8 or 64 letters makes the 4-cycle enumeration ~10^13 edges at S=27 -- it grows ~6x per
    scale from the oracle's S=20-22 counts -- for the reference as for this path; 256 letters keep it
    tractable: tools/c5_at_size.py, DESIGN.md.)"""
    import ctypes
    import json
    import shutil
    import tempfile
    from fuzzypatternmatching_amd import _abi
    scale, p_gen, nranks = 27, 8, 8
    fx = json.load(open(os.path.join(pmtest.ROOT, "tests", "golden", "rmat_s27_p8_cycle4_hash256.json")))
    lib = _abi.load()
    n = 1 << scale
    shm = shutil.disk_usage("/dev/shm").free if os.path.isdir("/dev/shm") else 0
    work = tempfile.mkdtemp(prefix="c5_", dir="/dev/shm" if shm > 60e9 else str(tmp_path))
    _graphs.clear()
    try:
        nb = ctypes.c_uint64()
        assert lib.pm_write_rmat_text(scale, p_gen, 0, os.path.join(work, "edges").encode(), ctypes.byref(nb)) == 0
        files = [os.path.join(work, f"edges.{r}") for r in range(p_gen)]
        labels = pmtest.hash_labels(n, C5_ALPHABET, salt=5)
        assert lib.pm_write_label_text(labels.ctypes.data, n, os.path.join(work, "lab").encode(), 4, None) == 0
        del labels
        m, ingest_s = pm.edge_list_matcher(files, CYCLE, undirected=True, device=0, nranks=nranks)
        m.labels_from_files(os.path.join(work, "lab"))
        out_i = tmp_path / "ingested"
        si = m.run_beta(str(out_i), 64)
        # chunk-cap invariance: the same search with at most 2^20 walks per level chunk
        monkeypatch.setenv("PM_TDS_CAP", str(1 << 20))
        out_c = tmp_path / "ingested_cap"
        sc = m.run_beta(str(out_c), 64)
        monkeypatch.delenv("PM_TDS_CAP")
        m.close()
        print(f"C5 S={scale}: ingest {ingest_s:.2f}s ({nb.value / ingest_s / 1e9:.1f} GB/s of text), search {si}, "
              f"capped: {sc['tds_chunks']} chunks")
        assert si["walks"] > 0 and si["tds_edges"] > 0
        dig_i = pmtest.result_digest(str(out_i), nranks)
        assert pmtest.digest_diffs(dig_i, pmtest.result_digest(str(out_c), nranks)) == []
        assert sc["tds_chunks"] > si["tds_chunks"]
        # the 8-way partition of the ingested graph (host CSR from the same GPU ingest)
        g = pm.ingest_edge_list_gpu(files, undirected=True, device=0, nranks=nranks)
        for f in files:
            os.remove(f)  # (host memory: the shards' rows are built next)
        out_s = tmp_path / "ingested_8_shards"
        each = pm.run_beta_local_shards_each(g, CYCLE, 8, str(out_s), max_iterations=64,
                                             label_prefix=os.path.join(work, "lab"))
        del g
        print(f"C5 S={scale} as 8 shards: split lines {[x['split_lines'] for x in each]}, entries "
              f"{[x['shard_entries'] for x in each]}, {each[0]}")
        assert all(x["split_lines"] > 0 for x in each)
        assert pmtest.digest_diffs(dig_i, pmtest.result_digest(str(out_s), nranks)) == []
    finally:
        shutil.rmtree(work, ignore_errors=True)
    diffs = pmtest.digest_diffs(fx["digest"], dig_i)
    keys = ("iterations", "terminated", "final_vertices", "final_edges", "lcc_edges", "nlcc_edges", "tds_edges",
            "walks")
    for k in keys:
        k_o = "paths" if k == "walks" else k
        if not (si[k] == sc[k] == each[0][k] == fx["stats"][k_o]):
            diffs.append(f"{k}: ingested {si[k]}, capped {sc[k]}, 8 shards {each[0][k]} vs oracle {fx['stats'][k_o]}")
    assert diffs == [], diffs[:5]


def check_against_fixture(m, fixture, tmp_path, max_iterations=64):
    """Runs the search of matcher m with result files and compares them with an oracle
    fixture made by tests/golden/make_rmat_fixture.py (digest + counters)."""
    import json
    fx = json.load(open(fixture))
    out = tmp_path / "gpu"
    sg = m.run_beta(str(out), max_iterations)
    dig = pmtest.result_digest(str(out), fx["nranks"])
    diffs = pmtest.digest_diffs(fx["digest"], dig)
    for k_g, k_o in (("iterations", "iterations"), ("terminated", "terminated"), ("final_vertices", "final_vertices"),
                     ("final_edges", "final_edges"), ("lcc_edges", "lcc_edges"), ("nlcc_edges", "nlcc_edges"),
                     ("tds_edges", "tds_edges"), ("walks", "paths")):
        if sg[k_g] != fx["stats"][k_o]:
            diffs.append(f"{k_g}: gpu {sg[k_g]} != oracle {fx['stats'][k_o]}")
    return sg, diffs


def test_c4_s28_tree_one_gpu(tmp_path):
    """The north_star headline (S=28, P_gen=8, tree) on one GPU, on the bench's path (graph generated
    and laid out in HBM), against the oracle's S=28 result digest (tests/golden/rmat_s28_p8_tree.json,
    made once on the GPU box's host by tests/golden/make_rmat_fixture.py: the oracle needs ~100 GB there)."""
    fixture = os.path.join(pmtest.ROOT, "tests", "golden", "rmat_s28_p8_tree.json")
    _graphs.clear()
    m, _ = pm.rmat_matcher(28, 8, TREE, device=0)
    try:
        sg, diffs = check_against_fixture(m, fixture, tmp_path)
    finally:
        m.close()
    assert diffs == [], diffs[:5]
    print(f"S=28 parity vs the oracle fixture: {sg}")


@pytest.mark.parametrize("nshards", [2, 4, 8])
def test_c4_s28_sharded_delegates_one_gpu(nshards, tmp_path):
    """C4's sharded path at full size on one GPU: pm_run_rmat_local_shards(S=28, P_gen=8, tree, -d 1048576)
    with `nshards` shards as threads of this process (the RCCL exchanges replaced by the in-process Comm):
    every shard generates its generator ranks' streams, the entries reach their owners in one all-to-all,
    the delegates' rows (degree >= 1048576) are split by target owner and meet at their controllers, the
    survivors' codes are all-gathered and the state is replicated.  The result must equal the oracle's S=28
    digest (LCC and TDS results are partition-independent; the fixture's result files are
    written with one rank, so no rank attribution differs).  nshards = 8 is BASELINE C4's partition: every
    shard holds delegate shares and the controllers spread over the shards.  The per-shard balance (entries,
    rows, delegate shares, superstep-0 work, device time of the sharded part, exchanged bytes) goes to
    $PM_STATS_DIR/c4_s28_shards<N>.json when that is set."""
    fixture = os.path.join(pmtest.ROOT, "tests", "golden", "rmat_s28_p8_tree.json")
    import json
    fx = json.load(open(fixture))
    _graphs.clear()
    out = tmp_path / "shards"
    each = pm.run_rmat_local_shards_each(28, 8, TREE, nshards, str(out), max_iterations=64, nranks=1,
                                         hub_threshold=pm.DEFAULT_HUB_THRESHOLD, repeats=1)
    sg = each[0]
    print(f"S=28 sharded x{nshards}: {sg['hubs']} delegates at -d {pm.DEFAULT_HUB_THRESHOLD}, {sg}")
    keys = ("shard_entries", "shard_rows", "shard_hub_entries", "shard_hubs_controlled", "shard_ss0_entries",
            "shard_ss0_survivors", "lcc_first_kernel_ms", "shard_sharded_ms", "comm_calls", "comm_bytes",
            "replica_rows", "replica_entries", "nlcc_seconds", "device_seconds")
    table = {k: [s[k] for s in each] for k in keys}
    for k in keys[:6] + ("lcc_first_kernel_ms", "shard_sharded_ms"):
        v = table[k]
        print(f"  {k}: max/mean {max(v) / max(sum(v) / len(v), 1e-12):.3f}  {v}")
    if os.environ.get("PM_STATS_DIR"):
        os.makedirs(os.environ["PM_STATS_DIR"], exist_ok=True)
        with open(os.path.join(os.environ["PM_STATS_DIR"], f"c4_s28_shards{nshards}.json"), "w") as f:
            json.dump({"nshards": nshards, "per_shard": table, "stats": sg}, f, indent=1)
    assert sg["hubs"] > 0  # hubs exist at C4's threshold: the delegate split runs
    assert sum(table["shard_entries"]) == 32 << 28  # every directed entry held by exactly one shard
    assert all(x > 0 for x in table["shard_hub_entries"])  # every shard holds delegate shares
    assert sum(x > 0 for x in table["shard_hubs_controlled"]) >= min(2, nshards)  # controllers spread
    assert sum(table["shard_hubs_controlled"]) == sg["hubs"]
    diffs = pmtest.digest_diffs(fx["digest"], pmtest.result_digest(str(out), 1))
    for k_g, k_o in (("iterations", "iterations"), ("terminated", "terminated"), ("final_vertices", "final_vertices"),
                     ("final_edges", "final_edges"), ("lcc_edges", "lcc_edges"), ("nlcc_edges", "nlcc_edges"),
                     ("tds_edges", "tds_edges"), ("walks", "paths")):
        if sg[k_g] != fx["stats"][k_o]:
            diffs.append(f"{k_g}: gpu {sg[k_g]} != oracle {fx['stats'][k_o]}")
    assert diffs == [], diffs[:5]


@pytest.mark.parametrize("nshards", [4, 8])
def test_c5_s27_generated_split_lines_fixture(nshards, tmp_path):
    """Config C5's search (S=27, P_gen=8, labels hash32(v ^ 5) % 256, 4-cycle: 4 cycle-check lines + the TDS
    line) on the GPU-generated graph, four and eight (BASELINE C5's partition) in-process shards, against the
    oracle's S=27 digest
    (tests/golden/rmat_s27_p8_cycle4_hash256.json, made on the GPU box's host by make_rmat_fixture.py; the
    bench's nlcc_config checks the one-context path against it).  With several shards every NLC line runs split by
    source owner (the split is decided on the lines' first-position token census) and its
    effects are exchanged; the result must not change."""
    import json
    fixture = os.path.join(pmtest.ROOT, "tests", "golden", "rmat_s27_p8_cycle4_hash256.json")
    fx = json.load(open(fixture))
    _graphs.clear()
    out = tmp_path / "shards"
    labels = pmtest.hash_labels(1 << 27, 256, salt=5)
    each = pm.run_rmat_local_shards_each(27, 8, CYCLE, nshards, str(out), max_iterations=64, nranks=1,
                                         hub_threshold=pm.DEFAULT_HUB_THRESHOLD, labels=labels)
    sg = each[0]
    print(f"C5 S=27 x{nshards}: split lines {[s['split_lines'] for s in each]}, {sg}")
    if nshards > 1:
        assert all(s["split_lines"] > 0 for s in each)  # the lines ran split by owner
    diffs = pmtest.digest_diffs(fx["digest"], pmtest.result_digest(str(out), 1))
    for k_g, k_o in (("iterations", "iterations"), ("terminated", "terminated"), ("final_vertices", "final_vertices"),
                     ("final_edges", "final_edges"), ("lcc_edges", "lcc_edges"), ("nlcc_edges", "nlcc_edges"),
                     ("tds_edges", "tds_edges"), ("walks", "paths")):
        if sg[k_g] != fx["stats"][k_o]:
            diffs.append(f"{k_g}: gpu {sg[k_g]} != oracle {fx['stats'][k_o]}")
    assert diffs == [], diffs[:5]
