"""CPU tests of the multi-GPU launch paths (no device needed):

* the launched CLI's process group (csrc/host/tcp_group.hpp): a host program compiled from
  tests/native/tcp_group_check.cpp runs every collective of pm_host_comm over TCP with known answers;
* pm_read_graph_shard: the shards read from the graph files partition the graph exactly as the sharded search
  expects (owner id % nshards, delegate rows split by target owner, delegate_partitioned_graph.ipp:1402-1648);
* run_pattern_matching_beta on a P-partition graph, in-process and launched as P processes, fails cleanly
  without a GPU (no hang, no partial result);
* bench.py --gpus N: the launcher's command / environment and its refusals.
"""
import os
import shutil
import socket
import subprocess
import sys

import numpy as np
import pytest

import fuzzypatternmatching_amd as pm
import pmtest

ROOT = pmtest.ROOT
CSRC = os.path.join(ROOT, "fuzzypatternmatching_amd", "csrc")
BIN = os.path.join(CSRC, "tools", "bin")
TREE = os.path.join(ROOT, "patterns", "rmat_log2_tree_pattern")


def _port():
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


@pytest.mark.parametrize("size", [2, 3, 5])
def test_tcp_group_collectives(tmp_path, size):
    cxx = shutil.which("g++")
    if cxx is None:
        pytest.skip("g++ not available")
    exe = tmp_path / "tcp_group_check"
    subprocess.check_call([cxx, "-O1", "-std=c++17", "-pthread", "-I", CSRC, "-o", str(exe),
                           os.path.join(ROOT, "tests", "native", "tcp_group_check.cpp")])
    r = subprocess.run([str(exe), str(_port()), str(size)], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr
    assert f"tcp group OK ({size} processes)" in r.stdout


def _partition(g, nshards, q):
    """The shard rows pm_create_shard takes, restated: owned rows whole, a delegate's entries by target owner."""
    deg = np.diff(g.off)
    off = np.zeros(g.n + 1, np.uint64)
    cols = []
    for v in range(g.n):
        row = g.col[g.off[v]:g.off[v + 1]]
        if nshards > 1 and deg[v] >= g.hub_threshold:
            row = row[row % nshards == q]
        elif v % nshards != q:
            row = row[:0]
        cols.append(row)
        off[v + 1] = off[v] + len(row)
    return off, np.concatenate(cols) if cols else np.zeros(0, np.uint32)


@pytest.mark.parametrize("P,nshards,hub", [(1, 1, 1 << 20), (2, 2, 1 << 20), (4, 3, 40), (3, 4, 25)])
def test_read_graph_shard_partitions_the_files(tmp_path, P, nshards, hub):
    g = pm.rmat_graph(10, 4, nranks=P, hub_threshold=hub)
    base = str(tmp_path / "g")
    pm.write_graph(base, g, P)
    assert pm.graph_partitions(base) == P
    held = 0
    for q in range(nshards):
        off, col, deg, info = pm.read_graph_shard(base, nshards, q)
        assert info == {"symmetric": True, "nranks": P, "hub_threshold": hub, "n": g.n}
        np.testing.assert_array_equal(deg, np.diff(g.off).astype(np.uint32))
        ro, rc = _partition(g, nshards, q)
        np.testing.assert_array_equal(off, ro)
        np.testing.assert_array_equal(col, rc)
        held += int(off[-1])
    assert held == g.nnz  # every directed entry on exactly one shard
    if hub < 100:
        assert (np.diff(g.off) >= hub).any()  # (the delegate rule was exercised)


def test_read_graph_shard_errors(tmp_path):
    with pytest.raises(pm.PMError, match="no graph files"):
        pm.read_graph_shard(str(tmp_path / "none"), 2, 0)
    g = pm.rmat_graph(8, 1)
    base = str(tmp_path / "g")
    pm.write_graph(base, g, 2)
    with pytest.raises(pm.PMError, match="bad shard index"):
        pm.read_graph_shard(base, 2, 2)


def _gen(base, scale, n):
    r = subprocess.run([os.path.join(BIN, "generate_rmat"), "-s", str(scale), "-n", str(n), "-o", base],
                       capture_output=True, text=True)
    assert r.returncode == 0, r.stderr


def test_beta_cli_partitioned_without_gpu(tmp_path):
    import torch
    if torch.cuda.is_available():
        pytest.skip("GPU present")
    base = str(tmp_path / "g")
    _gen(base, 10, 2)
    out = tmp_path / "out"
    out.mkdir()
    r = subprocess.run([os.path.join(BIN, "run_pattern_matching_beta"), "-i", base, "-p", TREE, "-o", str(out)],
                       capture_output=True, text=True, timeout=120)
    assert r.returncode == 1 and "no HIP device" in r.stderr, r.stderr
    assert not os.listdir(out)


def test_beta_cli_launched_ranks_without_gpu(tmp_path):
    """Two processes of one launch (PM_RANK / PM_WORLD_SIZE): they meet over TCP, read their own shards and fail
    alike at the device -- neither waits for the other forever."""
    import torch
    if torch.cuda.is_available():
        pytest.skip("GPU present")
    base = str(tmp_path / "g")
    _gen(base, 10, 2)
    out = tmp_path / "out"
    out.mkdir()
    port = _port()
    procs = []
    for r in range(2):
        env = dict(os.environ, PM_RANK=str(r), PM_WORLD_SIZE="2", PM_MASTER_ADDR="127.0.0.1",
                   PM_MASTER_PORT=str(port), PM_BOOTSTRAP_TIMEOUT="60")
        procs.append(subprocess.Popen([os.path.join(BIN, "run_pattern_matching_beta"), "-i", base, "-p", TREE,
                                       "-o", str(out)], env=env, stdout=subprocess.PIPE, stderr=subprocess.PIPE,
                                      text=True))
    outs = [p.communicate(timeout=120) for p in procs]
    for p, (so, se) in zip(procs, outs):
        assert p.returncode == 1, (so, se)
        assert "no HIP device" in se, se
    assert "2 ranks launched by PM" in outs[0][0]


def test_bench_launcher_command():
    sys.path.insert(0, ROOT)
    import bench
    cmd = bench.rank_launch_cmd(4, ["--gpus", "4", "--steps", "3"], 29999)
    assert cmd[:3] == [sys.executable, "-m", "torch.distributed.run"]
    assert "--nproc-per-node=4" in cmd and "--nnodes=1" in cmd
    assert "--master-addr=127.0.0.1" in cmd and "--master-port=29999" in cmd
    assert cmd[-4:] == ["--gpus", "4", "--steps", "3"] and cmd[-5].endswith("bench.py")
    assert bench.rank_launch_env()["HSA_ENABLE_IPC_MODE_LEGACY"] == "0"
    sp = bench.spread([1, 2, 3, 6])
    assert sp["max"] == 6 and sp["mean"] == 3 and sp["max_over_mean"] == 2


def test_bench_refuses_more_gpus_than_visible():
    import torch
    if torch.cuda.device_count() >= 2:
        pytest.skip("two GPUs visible")
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2"], capture_output=True,
                       text=True, env=env, timeout=300)
    assert r.returncode == 2
    assert "cannot be measured" in r.stderr and r.stdout.strip() == ""


def test_bench_refuses_world_size_mismatch():
    env = dict(os.environ, WORLD_SIZE="2", RANK="0", LOCAL_RANK="0")
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "4"], capture_output=True,
                       text=True, env=env, timeout=300)
    assert r.returncode == 2 and "WORLD_SIZE=2 but --gpus 4" in r.stderr and r.stdout.strip() == ""
