"""CPU (gloo, world_size 2 and 3) tests of TorchHostComm, the pm_host_comm the sharded search calls from C++
when its processes exchange through the host (pm_create_shard_host_comm): each collective is called through
the struct's C function pointers, exactly as HostComm (pm_shard.hip) calls it, on ctypes host buffers."""
import ctypes
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


def _worker(rank, world, port, out_dir):
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    res = {}
    try:
        hc = pm.TorchHostComm()
        st = hc.struct
        assert (st.nshards, st.shard) == (world, rank)
        # all-gather of 5 bytes per shard
        send = (ctypes.c_uint8 * 5)(*[(rank * 10 + i) % 256 for i in range(5)])
        recv = (ctypes.c_uint8 * (5 * world))()
        assert st.allgather(None, ctypes.addressof(send), ctypes.addressof(recv), 5) == 0
        res["ag"] = np.frombuffer(recv, np.uint8).copy()
        # u64 sum with wrap-around, u32 sum with wrap-around
        a64 = (ctypes.c_uint64 * 3)((1 << 63) + rank, 7, 0xFFFFFFFFFFFFFFFF)
        assert st.allreduce_sum_u64(None, ctypes.addressof(a64), 3) == 0
        res["u64"] = np.frombuffer(a64, np.uint64).copy()
        a32 = (ctypes.c_uint32 * 3)(0xFFFFFFF0 + rank, 3, 1 << 31)
        assert st.allreduce_sum_u32(None, ctypes.addressof(a32), 3) == 0
        res["u32"] = np.frombuffer(a32, np.uint32).copy()
        # all-to-all of variable blocks (some empty): shard r sends r + g bytes of value 16 r + g to shard g
        sb = (ctypes.c_uint64 * world)(*[(rank + g) % 3 for g in range(world)])
        rb = (ctypes.c_uint64 * world)(*[(g + rank) % 3 for g in range(world)])
        sdata = bytes(b for g in range(world) for b in [16 * rank + g] * sb[g])
        sbuf = (ctypes.c_uint8 * max(len(sdata), 1)).from_buffer_copy(sdata.ljust(max(len(sdata), 1), b"\0"))
        rbuf = (ctypes.c_uint8 * max(sum(rb), 1))()
        assert st.alltoallv(None, ctypes.addressof(sbuf), ctypes.addressof(sb), ctypes.addressof(rbuf),
                            ctypes.addressof(rb)) == 0
        res["a2a"] = np.frombuffer(rbuf, np.uint8)[: sum(rb)].copy()
        # a failing collective returns nonzero and keeps the exception (the C++ side turns it into an error)
        assert st.allgather(None, None, None, 3) != 0 and hc.error is not None
        np.savez(os.path.join(out_dir, f"r{rank}.npz"), **res)
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_torch_host_comm_collectives(tmp_path, world):
    mp.start_processes(_worker, args=(world, _free_port(), str(tmp_path)), nprocs=world, join=True,
                       start_method="spawn")
    m64 = (1 << 64) - 1
    for r in range(world):
        z = np.load(tmp_path / f"r{r}.npz")
        assert z["ag"].tolist() == [(q * 10 + i) % 256 for q in range(world) for i in range(5)]
        assert z["u64"].tolist() == [(sum((1 << 63) + q for q in range(world))) & m64, 7 * world,
                                     (world * m64) & m64]
        assert z["u32"].tolist() == [sum(0xFFFFFFF0 + q for q in range(world)) & 0xFFFFFFFF, 3 * world,
                                     (world << 31) & 0xFFFFFFFF]
        want = [16 * g + r for g in range(world) for _ in range((g + r) % 3)]
        assert z["a2a"].tolist() == want
