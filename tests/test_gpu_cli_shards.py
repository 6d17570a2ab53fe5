"""The drop-in executable on a P-partition graph (verdict r5 item 2): run_pattern_matching_beta reads P from the
graph files and runs the search as P shards -- in-process on the one GPU of the box (fewer GPUs than P), one
thread and GPU per shard with RCCL (here: one shard, PM_SHARDS=1, the one-rank communicator), or as P
processes launched like the reference under srun (README.md:30; PM_RANK / PM_WORLD_SIZE here), each reading its
own shard from the files and exchanging through the group's host collectives (the processes share the one GPU,
so not RCCL).  Every per-rank result file must equal the P-rank oracle's (compare_result_dirs, rank attribution
included), the same as the one-context run's.

Also the overflow agreement of replicated NLC lines: one shard alone reporting an overflow makes
every shard fail with the same message instead of leaving the others in a collective."""
import os
import socket
import subprocess

import numpy as np
import pytest

import fuzzypatternmatching_amd as pm
import oracle
import pmtest

pytestmark = pytest.mark.gpu

TREE = os.path.join(pmtest.ROOT, "patterns", "rmat_log2_tree_pattern")
CYCLE = os.path.join(pmtest.ROOT, "patterns", "rmat_log2_cycle4_pattern")
TRI = os.path.join(pmtest.ROOT, "patterns", "triangle_tail_pattern")
BIN = os.path.join(pmtest.ROOT, "fuzzypatternmatching_amd", "csrc", "tools", "bin")
CLI = os.path.join(BIN, "run_pattern_matching_beta")


def _port():
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _oracle_dir(base, pattern, out, labels=None):
    g = pm.read_graph(base)
    so = oracle.run(g.off, g.col, pattern, str(out), labels=labels, nranks=g.nranks, hub_threshold=g.hub_threshold,
                    threads=oracle.default_threads())
    return g, so


def _cli(base, pattern, out, env=None, labels_prefix=None, timeout=300):
    os.makedirs(out, exist_ok=True)
    cmd = [CLI, "-i", str(base), "-p", pattern, "-o", str(out)]
    if labels_prefix:
        cmd[3:3] = ["-v", str(labels_prefix)]
    return subprocess.run(cmd, capture_output=True, text=True, env=dict(os.environ, **(env or {})), timeout=timeout)


@pytest.mark.parametrize("pattern,hub", [(TREE, 1 << 20), (CYCLE, 1 << 20), (TREE, 96)])
def test_cli_partitioned_graph_in_process(tmp_path, pattern, hub):
    """generate_rmat -n 2 -> run_pattern_matching_beta: 2 shards in-process on the one GPU; hub 96: delegates."""
    base = tmp_path / "g"
    r = subprocess.run([os.path.join(BIN, "generate_rmat"), "-s", "15", "-n", "2", "-d", str(hub), "-o", str(base)],
                       capture_output=True, text=True)
    assert r.returncode == 0, r.stderr
    r = _cli(base, pattern, tmp_path / "gpu")
    assert r.returncode == 0, r.stderr
    assert "Shards 2 (in-process on one GPU)" in r.stdout, r.stdout
    g, so = _oracle_dir(str(base), pattern, tmp_path / "oracle")
    if hub < 1 << 20:
        assert (np.diff(g.off) >= hub).any()
    assert pmtest.compare_result_dirs(str(tmp_path / "oracle"), str(tmp_path / "gpu"), 2) == []


def test_cli_ingested_four_partitions_label_files(tmp_path):
    """ingest_edge_list -u 1 -n 4 of a text edge list, -v label files (hash labels, 64 letters), 4-cycle pattern:
    the CLI runs 4 in-process shards with the labels parsed on the device (pm_run_beta_local_shards2)."""
    scale, p_gen, nranks = 16, 4, 4
    und = [oracle.rmat_rank_edges(scale, p_gen, r) for r in range(p_gen)]
    u = np.concatenate([x[0] for x in und])
    v = np.concatenate([x[1] for x in und])
    txt = tmp_path / "edges.txt"
    np.savetxt(txt, np.stack([u, v], 1), fmt="%d")
    base = tmp_path / "ing"
    r = subprocess.run([os.path.join(BIN, "ingest_edge_list"), "-o", str(base), "-u", "1", "-n", str(nranks),
                        "-d", "200", str(txt)], capture_output=True, text=True)
    assert r.returncode == 0, r.stderr
    g = pm.read_graph(str(base))
    labels = pmtest.hash_labels(g.n, 64, salt=5)
    for i, part in enumerate(np.array_split(np.arange(g.n), 3)):
        with open(tmp_path / f"lab.{i}", "w") as f:
            f.write("".join(f"{x} {labels[x]}\n" for x in part))
    r = _cli(base, CYCLE, tmp_path / "gpu", labels_prefix=tmp_path / "lab")
    assert r.returncode == 0, r.stderr
    assert "Shards 4" in r.stdout
    oracle.run(g.off, g.col, CYCLE, str(tmp_path / "oracle"), labels=labels, nranks=nranks,
               hub_threshold=g.hub_threshold, threads=oracle.default_threads())
    assert pmtest.compare_result_dirs(str(tmp_path / "oracle"), str(tmp_path / "gpu"), nranks) == []


@pytest.mark.parametrize("nproc,pattern,hub", [(2, TREE, 96), (3, TRI, 1 << 20)])
def test_cli_launched_processes(tmp_path, nproc, pattern, hub):
    """The reference's launch shape: P processes of one run_pattern_matching_beta (PM_RANK / PM_WORLD_SIZE, as
    srun's SLURM_PROCID / SLURM_NTASKS would set them), each reading only its own shard of the P files; they
    share the box's one GPU, so the group carries the exchanges over TCP (pm_host_comm)."""
    base = tmp_path / "g"
    r = subprocess.run([os.path.join(BIN, "generate_rmat"), "-s", "14", "-n", str(nproc), "-d", str(hub), "-o",
                        str(base)], capture_output=True, text=True)
    assert r.returncode == 0, r.stderr
    port = _port()
    out = tmp_path / "gpu"
    out.mkdir()
    procs = []
    for q in range(nproc):
        env = dict(os.environ, PM_RANK=str(q), PM_WORLD_SIZE=str(nproc), PM_MASTER_ADDR="127.0.0.1",
                   PM_MASTER_PORT=str(port), PM_BOOTSTRAP_TIMEOUT="90")
        procs.append(subprocess.Popen([CLI, "-i", str(base), "-p", pattern, "-o", str(out)], env=env,
                                      stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True))
    outs = []
    try:
        outs = [p.communicate(timeout=240) for p in procs]
    finally:
        for p in procs:
            if p.poll() is None:
                p.kill()
    for p, (so, se) in zip(procs, outs):
        assert p.returncode == 0, (so, se)
    assert f"{nproc} ranks launched by PM, host collectives over TCP" in outs[0][0], outs[0][0]
    assert f"Shards {nproc} ({nproc} processes, host collectives of {nproc} ranks)" in outs[0][0], outs[0][0]
    _oracle_dir(str(base), pattern, tmp_path / "oracle")
    assert pmtest.compare_result_dirs(str(tmp_path / "oracle"), str(out), nproc) == []


def test_cli_gpu_threads_rccl_one_shard(tmp_path):
    """PM_SHARDS=1 on a 2-partition graph: one shard on one GPU through the one-thread-per-GPU mode and its RCCL
    communicator (the multi-GPU node's code path with the one GPU this box has); result files for P = 2."""
    base = tmp_path / "g"
    r = subprocess.run([os.path.join(BIN, "generate_rmat"), "-s", "14", "-n", "2", "-o", str(base)],
                       capture_output=True, text=True)
    assert r.returncode == 0, r.stderr
    r = _cli(base, TREE, tmp_path / "gpu", env={"PM_SHARDS": "1"})
    assert r.returncode == 0, r.stderr
    assert "one GPU each" in r.stdout
    _oracle_dir(str(base), TREE, tmp_path / "oracle")
    assert pmtest.compare_result_dirs(str(tmp_path / "oracle"), str(tmp_path / "gpu"), 2) == []


def test_replicated_line_overflow_on_one_shard_fails_every_shard(tmp_path, monkeypatch):
    """PM_DEBUG_OVERFLOW_SHARD=1: shard 1 alone reports its first replicated path line as overflowed.  The shards
    gather the first overflowed line before acting (one collective per line launch), see that they disagree, and
    every one of them fails with the same message -- none waits in regrow_hash's agreement for the others."""
    g = pm.rmat_graph(12, 4)
    labels = pmtest.hash_labels(g.n, 8)
    monkeypatch.setenv("PM_DEBUG_OVERFLOW_SHARD", "1")
    monkeypatch.setenv("PM_SPLIT_LINES", "0")  # (every line replicated)
    with pytest.raises(pm.PMError, match="overflowed its table on some shards only"):
        pm.run_beta_local_shards(g, CYCLE, 2, labels=labels)
    monkeypatch.setenv("PM_DEBUG_OVERFLOW_SHARD", "-1")
    so = oracle.run(g.off, g.col, CYCLE, None, labels=labels)
    st = pm.run_beta_local_shards(g, CYCLE, 2, labels=labels)
    assert (st["final_vertices"], st["nlcc_edges"], st["tds_edges"]) == (so["final_vertices"], so["nlcc_edges"],
                                                                         so["tds_edges"])
