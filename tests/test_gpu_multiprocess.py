"""The sharded search across a process boundary: `world` processes, each holding its own
shard context (pm_create_shard_host_comm) on device 0 of the test box, their exchanges carried by
torch.distributed gloo through host staging (TorchHostComm; the same all-gather / all-reduce / all-to-all
calls RcclComm makes).  Each process builds its share of the input the way a multi-GPU run does: its
generator ranks' edge stream (pm_rmat_edges) routed to the owners by pm.partition_edges over gloo (owner
id % world, delegates split by target owner, delegate_partitioned_graph.ipp:818-969, 1402-1648).  Every
result file (written by shard 0) and the counters must equal the oracle's: delegates, split NLC lines
(PM_SPLIT_LINES=1) with cycle flags exchanged, and three processes."""
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp

import fuzzypatternmatching_amd as pm
import oracle
import pmtest

pytestmark = pytest.mark.gpu

PATTERNS = {
    "tree": os.path.join(pmtest.ROOT, "patterns", "rmat_log2_tree_pattern"),
    "cycle": os.path.join(pmtest.ROOT, "patterns", "rmat_log2_cycle4_pattern"),
    "triangle": os.path.join(pmtest.ROOT, "patterns", "triangle_tail_pattern"),
}


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, scale, p_gen, pat, alphabet, thr, nranks, out_dir, env):
    import json
    import torch.distributed as dist
    os.environ.update(env)
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        n = 1 << scale
        src, dst = pm.rmat_edges(scale, p_gen, rank, world)
        off, col, deg = pm.partition_edges(src, dst, n, hub_threshold=thr)
        comm = pm.TorchHostComm()
        m = pm.ShardedPatternMatcher(n, off, col, deg, PATTERNS[pat], world, rank, device=0, nranks=nranks,
                                     hub_threshold=thr, host_comm=comm)
        if alphabet:
            m.set_labels(pmtest.hash_labels(n, alphabet))
        st = m.run_beta(os.path.join(out_dir, "shards"), max_iterations=100)  # collective; shard 0 writes
        st2 = m.run_beta("", max_iterations=100)  # a second search on the same contexts
        m.close()
        with open(os.path.join(out_dir, f"stats{rank}.json"), "w") as f:
            json.dump({"first": st, "second": st2}, f)
    finally:
        dist.destroy_process_group()


# (pattern, scale, P_gen, label alphabet, hub threshold, result ranks, processes, env)
CASES = [
    ("tree", 14, 4, None, 64, 2, 2, {}),
    ("cycle", 12, 4, 8, pm.DEFAULT_HUB_THRESHOLD, 1, 2, {"PM_SPLIT_LINES": "1"}),
    ("cycle", 13, 4, 16, 16, 2, 3, {"PM_SPLIT_LINES": "1"}),
    ("triangle", 12, 4, 6, pm.DEFAULT_HUB_THRESHOLD, 1, 2, {"PM_SPLIT_LINES": "1"}),
]


@pytest.mark.parametrize("pat,scale,p_gen,alphabet,thr,nranks,world,env", CASES)
def test_sharded_processes_match_oracle(pat, scale, p_gen, alphabet, thr, nranks, world, env, tmp_path):
    import json
    mp.start_processes(_worker, args=(world, _free_port(), scale, p_gen, pat, alphabet, thr, nranks, str(tmp_path),
                                      env), nprocs=world, join=True, start_method="spawn")
    g = pm.rmat_graph(scale, p_gen)
    labels = None if alphabet is None else pmtest.hash_labels(g.n, alphabet)
    so = oracle.run(g.off, g.col, PATTERNS[pat], str(tmp_path / "oracle"), labels=labels, nranks=nranks,
                    hub_threshold=thr, max_iterations=100)
    assert pmtest.compare_result_dirs(str(tmp_path / "oracle"), str(tmp_path / "shards"), nranks) == []
    stats = [json.load(open(tmp_path / f"stats{r}.json")) for r in range(world)]
    for s in stats:
        for run in ("first", "second"):
            sg = s[run]
            assert (sg["iterations"], sg["terminated"]) == (so["iterations"], so["terminated"])
            assert (sg["final_vertices"], sg["final_edges"]) == (so["final_vertices"], so["final_edges"])
            assert (sg["lcc_edges"], sg["nlcc_edges"], sg["tds_edges"]) == (so["lcc_edges"], so["nlcc_edges"],
                                                                           so["tds_edges"])
            assert sg["walks"] == so["paths"]
            assert sg["comm_calls"] > 0
    assert sum(s["first"]["shard_entries"] for s in stats) == g.nnz
    if thr < pm.DEFAULT_HUB_THRESHOLD:
        assert stats[0]["first"]["hubs"] > 0
    if env.get("PM_SPLIT_LINES"):
        assert stats[0]["first"]["split_lines"] > 0
