"""CPU (gloo, world_size 2 and 3) tests of the sharded path's host side: the distributed
R-MAT share of each process and the owner partitioning exchange that feeds pm_create_shard."""
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp

import fuzzypatternmatching_amd as pm


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, scale, p_gen, out_dir, thr=pm.DEFAULT_HUB_THRESHOLD):
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        src, dst = pm.rmat_edges(scale, p_gen, rank, world)
        off, col, deg = pm.partition_edges(src, dst, 1 << scale, hub_threshold=thr)
        np.savez(os.path.join(out_dir, f"r{rank}.npz"), off=off, col=col, deg=deg)
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_partition_edges_matches_full_csr(tmp_path, world):
    scale, p_gen = 10, 6
    mp.start_processes(_worker, args=(world, _free_port(), scale, p_gen, str(tmp_path)), nprocs=world,
                       join=True, start_method="spawn")
    g = pm.rmat_graph(scale, p_gen)
    deg = np.diff(g.off)
    n = g.n
    seen = np.zeros(n, bool)
    for r in range(world):
        z = np.load(tmp_path / f"r{r}.npz")
        off, col = z["off"], z["col"]
        assert np.array_equal(z["deg"].astype(np.uint64), deg)
        ldeg = np.diff(off)
        own = (np.arange(n) % world) == r
        assert np.array_equal(ldeg[own], deg[own])
        assert not ldeg[~own].any()
        for v in np.flatnonzero(own)[:: max(1, n // 97)]:
            assert np.array_equal(col[off[v]:off[v + 1]], g.col[g.off[v]:g.off[v + 1]])
        seen |= own
        assert int(off[-1]) == int(deg[own].sum())
    assert seen.all()


@pytest.mark.parametrize("world", [2, 3])
def test_partition_edges_splits_delegates_by_target(tmp_path, world):
    # delegates (degree >= thr): every process holds the entries whose target it owns
    scale, p_gen, thr = 10, 4, 40
    mp.start_processes(_worker, args=(world, _free_port(), scale, p_gen, str(tmp_path), thr), nprocs=world,
                       join=True, start_method="spawn")
    g = pm.rmat_graph(scale, p_gen)
    deg = np.diff(g.off)
    hubs = np.flatnonzero(deg >= thr)
    assert len(hubs) > 0
    parts = [np.load(tmp_path / f"r{r}.npz") for r in range(world)]
    total = 0
    for r, z in enumerate(parts):
        off, col = z["off"], z["col"]
        total += int(off[-1])
        for v in range(g.n):
            row = col[off[v]:off[v + 1]]
            full = g.col[g.off[v]:g.off[v + 1]]
            if deg[v] >= thr:
                assert np.array_equal(row, full[full % world == r])
            elif v % world == r:
                assert np.array_equal(row, full)
            else:
                assert len(row) == 0
    assert total == g.nnz


def test_rmat_edges_shares_cover_the_stream():
    scale, p_gen = 9, 4
    full_s, full_d = pm.rmat_edges(scale, p_gen)
    parts = [pm.rmat_edges(scale, p_gen, r, 2) for r in range(2)]
    per = len(full_s) // p_gen
    # rank r of 2 holds generator ranks r, r + 2 in order
    for r in range(2):
        s, d = parts[r]
        want_s = np.concatenate([full_s[q * per:(q + 1) * per] for q in range(r, p_gen, 2)])
        want_d = np.concatenate([full_d[q * per:(q + 1) * per] for q in range(r, p_gen, 2)])
        assert np.array_equal(s, want_s) and np.array_equal(d, want_d)
    g = pm.rmat_graph(scale, p_gen)
    assert len(full_s) == g.nnz
