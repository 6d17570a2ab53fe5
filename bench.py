#!/usr/bin/env python3
"""Benchmark: edges-traversed/s of the LCC+NLCC driver loop (BASELINE.json metric).

One "step" = one complete run_pattern_matching_beta pattern search
(run_pattern_matching_beta.cpp:539-1356: every LCC superstep, every NLC line,
post-processing and interleaved LCC calls until the loop terminates) over the
graph already resident in HBM.  Workload at every N: the north_star headline,
R-MAT scale 28 from P_gen = 8 generator ranks (BASELINE.json configs[3]; 8.6 G
directed entries), degree-log2 labels, examples/rmat_log2_tree_pattern.  The
graph is generated on the GPU (pm_rmat.hip, bit-identical to the generate_rmat
stream).

Edges traversed: adjacency entries scanned by LCC senders
(full CSR degree in superstep 0 of the first call, |M[v]| later) plus those
scanned by NLCC/TDS initiators and relays; counted identically by the oracle.

N = 1: one context holds the whole graph (pm_create_rmat).  N > 1 GPUs
(torch.distributed.run, one process per GPU): ONE search over the same S=28
graph sharded across the ranks (owner = id % N, delegate rows split by target
owner; pm_create_rmat_shard: every rank generates the streams of generator
ranks r = rank (mod N) on its GPU and the entries reach their owners in one
RCCL all-to-all, untimed setup).  Strong scaling: the total work is the same
at every N.  `value` = edges traversed by the whole search / max-over-ranks
time.  `--sharded` takes the sharded path at N = 1 (rehearsal).

Parity: after the timed steps the same search is run once more with result
files and compared with the oracle's S=28 digest (tests/golden/
rmat_s28_p8_tree.json, made by tests/golden/make_rmat_fixture.py); the CPU
baseline leg runs the oracle on a bounded S=24 sample and the GPU on the same
sample, and compares their counters.  A mismatch prints "invalid" and exits 3.
"""
import argparse
import json
import os
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "edges-traversed/sec (LCC+NLCC) on R-MAT + tree pattern, 1/2/4/8 GPU"
HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md chip table: HBM3E 8.0 TB/s


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def edges_of(s):
    return s["lcc_edges"] + s["nlcc_edges"] + s["tds_edges"]


def host_cpu_share():
    """Host CPUs this process may use: the affinity mask, bounded by the cgroup CPU quota and by the pool's
    OMP_NUM_THREADS (a one-GPU lease is given 16 of the host's CPUs); every bound is reported."""
    info = {"affinity": len(os.sched_getaffinity(0)), "os_cpu_count": os.cpu_count()}
    share = info["affinity"]
    try:
        q, per = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if q != "max":
            info["cgroup_quota_cpus"] = round(int(q) / int(per), 2)
            share = min(share, max(1, int(int(q) / int(per))))
    except (OSError, ValueError):
        pass
    omp = os.environ.get("OMP_NUM_THREADS")
    if omp and omp.isdigit() and int(omp) > 0:
        info["omp_num_threads"] = int(omp)
        share = min(share, int(omp))
    info["threads_used"] = share
    return share, info


def free_port():
    import socket
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as sk:
        sk.bind(("127.0.0.1", 0))
        return sk.getsockname()[1]


def rank_launch_cmd(n, argv, port):
    """The N-rank launch of this script (one process per GPU), as the driver itself runs it for N > 1."""
    return [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
            "--master-addr=127.0.0.1", f"--master-port={port}", os.path.abspath(__file__)] + list(argv)


def rank_launch_env():
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")  # (dmabuf IPC only: RCCL needs it)
    return env


def launch_ranks(n, argv):
    """`bench.py --gpus N` started without a launcher: start N ranks as a child torch.distributed.run (this process
    never touches the GPU -- torch.cuda.device_count() does not initialise it -- and never execs), wait for them and
    return their exit status; rank 0 prints the JSON line to the shared stdout."""
    import subprocess
    import torch
    have = torch.cuda.device_count()
    if have < n:
        log(f"bench.py --gpus {n}: only {have} GPU(s) visible to this process; a {n}-GPU line cannot be measured "
            f"here (no line printed)")
        return 2
    cmd = rank_launch_cmd(n, argv, free_port())
    log("launching: " + " ".join(cmd))
    return subprocess.run(cmd, env=rank_launch_env()).returncode


def line_stream():
    """The stream the JSON line goes to: this process's original stdout.  File descriptor 1 itself is pointed at
    stderr, so whatever the libraries write there (RCCL's version banner at communicator creation, on every rank)
    cannot come before or between the JSON lines of a run."""
    sys.stdout.flush()
    fd = os.dup(1)
    os.dup2(2, 1)
    return os.fdopen(fd, "w")


def spread(vals):
    vals = [float(v) for v in vals]
    mean = sum(vals) / len(vals) if vals else 0.0
    return {"max": max(vals), "mean": round(mean, 6), "min": min(vals),
            "max_over_mean": round(max(vals) / mean, 4) if mean else None}


def main():
    import faulthandler
    faulthandler.enable()  # a fatal signal prints the Python stack
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--scale", type=int, default=28)
    ap.add_argument("--p-gen", type=int, default=8)
    ap.add_argument("--pattern", default="rmat_log2_tree_pattern")
    ap.add_argument("--max-iterations", type=int, default=64)
    ap.add_argument("--hub-threshold", type=int, default=1048576, help="-d of generate_rmat (delegates)")
    ap.add_argument("--cpu-baseline", choices=["auto", "off"], default="auto")
    ap.add_argument("--cpu-scale", type=int, default=24,
                    help="the CPU baseline runs the same search at min(scale, cpu-scale) (bounded sample)")
    ap.add_argument("--fixture-check", choices=["auto", "off"], default="auto")
    ap.add_argument("--graph-cache", default=os.environ.get("PM_GRAPH_CACHE"),
                    help="directory: reuse / store the generated one-GPU graph (repeated profiling runs)")
    ap.add_argument("--gen", choices=["gpu", "host"], default="gpu",
                    help="R-MAT generator: gpu (pm_rmat.hip, adjacency built in HBM) or host (host/rmat.hpp)")
    ap.add_argument("--sharded", action="store_true",
                    help="take the sharded (RCCL) path even at N=1 (rehearsal of the multi-GPU code on one GPU)")
    ap.add_argument("--pmc", default=None, help="PMC summary of k_lcc_first (default: the newest profiles/r*_pmc_lcc_first.json)")
    ap.add_argument("--c3", choices=["auto", "off"], default="auto",
                    help="also time BASELINE config C3 (S=26, P_gen=4, 4-cycle: the token-passing stress) at N=1")
    ap.add_argument("--sharded-n1", choices=["auto", "off"], default="auto",
                    help="at N=1 also time the sharded path with one shard (one-rank RCCL communicator, the code every "
                         "rank of an N-GPU run executes) on the same search")
    ap.add_argument("--nlcc", choices=["auto", "off"], default="auto",
                    help="also time the token-passing path with real work at N=1: config C5's search (S=27, "
                         "hash32(v ^ 5) % 256 labels, 4-cycle) on the GPU-generated graph, checked against "
                         "tests/golden/rmat_s27_p8_cycle4_hash256.json")
    args = ap.parse_args()

    env_world = os.environ.get("WORLD_SIZE")
    if env_world is None and args.gpus > 1:
        return launch_ranks(args.gpus, sys.argv[1:])
    if env_world is not None and int(env_world) != args.gpus:
        log(f"bench.py: launched with WORLD_SIZE={env_world} but --gpus {args.gpus}; the line would mislabel the run")
        return 2
    out_stream = line_stream()  # (after the launcher branch: its ranks inherit the real stdout)
    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    dist = None
    sharded = world > 1 or args.sharded
    if sharded:
        import torch
        import torch.distributed as dist
        if world > 1 and local_rank >= torch.cuda.device_count():
            log(f"bench.py rank {rank}: local rank {local_rank} but only {torch.cuda.device_count()} GPU(s) visible")
            return 2
        torch.cuda.set_device(local_rank)
        dist.init_process_group(backend="nccl")

    import numpy as np
    import fuzzypatternmatching_amd as pm

    pattern_dir = os.path.join(ROOT, "patterns", args.pattern)
    t_setup = time.time()
    g = None
    setup = {}
    if not sharded and args.gen == "gpu" and not args.graph_cache:
        m, gen_s = pm.rmat_matcher(args.scale, args.p_gen, pattern_dir, device=0, hub_threshold=args.hub_threshold)
        setup["generate_rmat_gpu"] = round(gen_s, 3)
    elif not sharded:
        cache = (os.path.join(args.graph_cache, f"rmat_s{args.scale}_p{args.p_gen}") if args.graph_cache else None)
        if cache and os.path.exists(cache + "_0_of_1"):
            g = pm.read_graph(cache)
        else:
            g = pm.rmat_graph(args.scale, args.p_gen)
            if cache:
                os.makedirs(args.graph_cache, exist_ok=True)
                pm.write_graph(cache, g, 1)
        setup["generate_rmat_host"] = round(time.time() - t_setup, 3)
        g.hub_threshold = args.hub_threshold
        m = pm.PatternMatcher(g, pattern_dir, device=0)
    else:
        uid = [pm.comm_unique_id() if rank == 0 else None]
        dist.broadcast_object_list(uid, src=0)
        m, gen_s = pm.rmat_shard_matcher(args.scale, args.p_gen, pattern_dir, world, rank, uid[0], device=local_rank,
                                         hub_threshold=args.hub_threshold)
        setup["generate_rmat_gpu_and_route_to_owners"] = round(gen_s, 3)
    n, nnz = 1 << args.scale, (1 << args.scale) * 32
    setup["context_total"] = round(time.time() - t_setup, 3)
    log(f"[rank {rank}] R-MAT S={args.scale} P_gen={args.p_gen} ({'sharded over ' + str(world) if sharded else 'one GPU'})"
        f": context ready after {setup['context_total']:.1f}s")

    def barrier_sync():
        if dist is not None:
            import torch
            torch.cuda.synchronize()
            dist.barrier()

    # the first search of the context: what a single run_pattern_matching_beta invocation pays on top of
    # the setup (graph generation / load + layout)
    t0 = time.time()
    first = m.run_beta("", args.max_iterations)
    setup["first_search_s"] = round(time.time() - t0, 4)
    setup["first_search_including_setup_s"] = round(time.time() - t_setup, 3)
    for _ in range(max(args.warmup - 1, 0)):
        m.run_beta("", args.max_iterations)
    barrier_sync()
    from fuzzypatternmatching_amd import _abi
    raw = [_abi.RunStats() for _ in range(args.steps)]  # (filled in the timed loop, read after it)
    t_start = time.perf_counter()
    for st in raw:
        m.run_beta_into(st, args.max_iterations)
    barrier_sync()
    elapsed = time.perf_counter() - t_start
    stats = [st.as_dict() for st in raw]
    # the stats of a sharded search already cover the whole graph (every rank reports the same)
    edges = sum(edges_of(s) for s in stats)
    kern_ms = float(np.mean([s["lcc_first_kernel_ms"] for s in stats]))
    kern_bytes = stats[-1]["lcc_first_bytes"]
    if dist is not None:
        import torch
        t = torch.tensor([elapsed], dtype=torch.float64, device="cuda")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    s0 = stats[-1]
    log(f"[rank {rank}] per step: {s0['iterations']} iterations (terminated={s0['terminated']}), "
        f"lcc {s0['lcc_edges']} nlcc {s0['nlcc_edges']} tds {s0['tds_edges']} edges, walks {s0['walks']}, "
        f"final |S|={s0['final_vertices']} |M|={s0['final_edges']}, host {s0['seconds'] * 1e3:.3f} ms, "
        f"device {s0['device_seconds'] * 1e3:.3f} ms, lcc_first kernel {kern_ms:.4f} ms")

    # parity of this very context at the headline size: the oracle's S=28 digest
    invalid = []
    fixture = None
    fx_path = os.path.join(ROOT, "tests", "golden", f"rmat_s{args.scale}_p{args.p_gen}_"
                           f"{args.pattern.replace('rmat_log2_', '').replace('_pattern', '')}.json")
    if args.fixture_check == "auto" and os.path.exists(fx_path) and args.hub_threshold == 1048576:
        sys.path.insert(0, os.path.join(ROOT, "tests"))
        import pmtest
        fx = json.load(open(fx_path))
        td = tempfile.mkdtemp(prefix="pmbench") if rank == 0 else ""
        sf = m.run_beta(td, args.max_iterations)  # collective; shard 0 writes the files
        if rank == 0:
            diffs = pmtest.digest_diffs(fx["digest"], pmtest.result_digest(td, fx["nranks"]))
            for k_g, k_o in (("final_vertices", "final_vertices"), ("final_edges", "final_edges"),
                             ("lcc_edges", "lcc_edges"), ("nlcc_edges", "nlcc_edges"), ("tds_edges", "tds_edges"),
                             ("walks", "paths"), ("iterations", "iterations")):
                if sf[k_g] != fx["stats"][k_o] or s0[k_g] != fx["stats"][k_o]:
                    diffs.append(f"{k_g}: gpu {s0[k_g]}/{sf[k_g]} != oracle {fx['stats'][k_o]}")
            import shutil
            shutil.rmtree(td, ignore_errors=True)
            fixture = {"file": os.path.relpath(fx_path, ROOT), "match": not diffs,
                       "what": "every result file of the timed search (digest: count files, sorted-line-set sha256 "
                               "of vertices / edges / subgraphs) and its counters against the oracle's"}
            if diffs:
                invalid.append("GPU search differs from the oracle's S=28 fixture: " + "; ".join(diffs[:4]))

    # N GPUs: the communicator as the library sees it, and every shard's share of the search
    shards = None
    if sharded:
        info = m.comm_info()
        mine = {k: s0[k] for k in ("shard_entries", "shard_rows", "shard_hub_entries", "shard_hubs_controlled",
                                   "shard_ss0_entries", "shard_ss0_survivors", "shard_sharded_ms", "comm_calls",
                                   "comm_bytes", "comm_seconds", "lcc_first_kernel_ms")}
        mine.update(info)
        every = [None] * world
        dist.all_gather_object(every, mine)
        shards = {"transport": info["transport"], "comm_ranks": info["comm_ranks"], "nshards": info["nshards"],
                  "per_shard": {k: spread([e[k] for e in every])
                                for k in ("shard_entries", "shard_rows", "shard_ss0_entries", "shard_sharded_ms",
                                          "lcc_first_kernel_ms", "comm_bytes", "comm_seconds")},
                  "comm_calls_per_search": s0["comm_calls"], "replica_rows": s0["replica_rows"],
                  "replica_entries": s0["replica_entries"]}
        if any(e["comm_ranks"] != world or e["nshards"] != world for e in every):
            invalid.append(f"communicator ranks {[e['comm_ranks'] for e in every]} / shards "
                           f"{[e['nshards'] for e in every]} differ from the {world} launched ranks")

    lay = None
    if not sharded:
        import ctypes
        from fuzzypatternmatching_amd import _abi
        st = (ctypes.c_uint64 * 7)()
        if _abi.load().pm_debug_layout_stats(m._ctx, st, 7) == 0:
            lay = list(st)
    m.close()  # release device memory before the runtime (and any profiler) tears down
    if rank != 0:
        if dist is not None:
            dist.barrier()
            dist.destroy_process_group()
        return 0

    achieved = kern_bytes / (kern_ms * 1e-3) / 1e9 if kern_ms > 0 else 0.0
    traffic = None
    if args.pmc is None:
        import glob
        cands = sorted(glob.glob(os.path.join(ROOT, "profiles", "r[0-9][0-9]_pmc_lcc_first.json")))
        args.pmc = cands[-1] if cands else ""
    if args.pmc and os.path.exists(args.pmc):
        try:
            pmc = json.load(open(args.pmc))
            if (pmc.get("scale") == args.scale and pmc.get("p_gen") == args.p_gen and pmc.get("pattern") == args.pattern
                    and not sharded):
                traffic = pmc.get("hbm_bytes_per_launch")
        except Exception as ex:  # noqa: BLE001
            log(f"pmc file unreadable: {ex}")
    import ctypes
    from fuzzypatternmatching_amd import _abi
    copy = ctypes.c_double()
    copy_gbs = None
    if _abi.load().pm_debug_copy_gbs(local_rank, 4 << 30, 20, ctypes.byref(copy)) == 0:
        copy_gbs = round(copy.value, 1)
    roofline = {"bound": "hbm", "kernel": "k_lcc_first", "achieved": round(achieved, 2), "peak": HBM_PEAK_GBS,
                "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": traffic,
                "algorithmic_bytes_per_launch": kern_bytes, "avg_launch_ms": round(kern_ms, 5),
                "measured_copy_gbs": copy_gbs,
                # the whole search step against the same bytes (every later superstep / NLC line moves
                # little): effective bandwidth of the step
                "step_achieved": round(kern_bytes / (elapsed / args.steps) / 1e9, 2),
                "step_frac": round(kern_bytes / (elapsed / args.steps) / 1e9 / HBM_PEAK_GBS, 4)}
    if sharded:
        roofline["scope"] = "rank 0's shard (its superstep-0 launch and bytes)"
    if lay is not None:
        real, slots, rows, tiles = lay[0], lay[1], lay[2], lay[3]
        setup["label_major_layout_and_tiling"] = round(lay[6] * 1e-6, 3)
        roofline.update({"scanned_entries": real, "loaded_slots": slots,
                         "padded_slot_ratio": round(slots / max(real, 1), 4), "scanned_rows": rows, "tiles": tiles})

    # a single run_pattern_matching_beta invocation: the layout (labels -> label-major CSR + tiling) and the
    # first search, with and without the graph's generation
    if "label_major_layout_and_tiling" in setup and setup.get("first_search_s"):
        fe = edges_of(first)
        setup["single_invocation_edges_per_s"] = round(
            fe / (setup["label_major_layout_and_tiling"] + setup["first_search_s"]), 1)
        setup["single_invocation_edges_per_s_incl_generation"] = round(fe / setup["first_search_including_setup_s"], 1)

    # BASELINE.json configs[2] (C3): S=26, P_gen=4, the 4-cycle pattern -- the NLCC token-passing stress
    c3 = None
    if args.c3 == "auto" and world == 1 and not sharded:
        cyc = os.path.join(ROOT, "patterns", "rmat_log2_cycle4_pattern")
        m3, g3 = pm.rmat_matcher(26, 4, cyc, device=0)
        f3 = m3.run_beta("", args.max_iterations)
        for _ in range(2):
            m3.run_beta("", args.max_iterations)
        t3 = time.perf_counter()
        r3 = [m3.run_beta("", args.max_iterations) for _ in range(5)]
        e3 = (time.perf_counter() - t3) / 5
        m3.close()
        c3 = {"workload": "R-MAT scale-26 (P_gen=4) + rmat_log2_cycle4_pattern (4 cycle-check lines + TDS line), one GPU",
              "value": round(edges_of(r3[-1]) / e3, 1), "unit": "edges/s", "ms_per_step": round(e3 * 1e3, 3),
              "steps": 5, "edges_per_step": edges_of(r3[-1]), "lcc_edges": r3[-1]["lcc_edges"],
              "nlcc_edges": r3[-1]["nlcc_edges"], "tds_edges": r3[-1]["tds_edges"], "walks": r3[-1]["walks"],
              "iterations": r3[-1]["iterations"],
              "nlcc_ms_per_step": round(sum(r["nlcc_seconds"] for r in r3) / 5 * 1e3, 3),
              "nlcc_share": round(sum(r["nlcc_seconds"] for r in r3) / 5 / e3, 4),
              "nlcc_edges_per_s": round((r3[-1]["nlcc_edges"] + r3[-1]["tds_edges"]) /
                                        max(sum(r["nlcc_seconds"] for r in r3) / 5, 1e-9), 1),
              "first_search_s": round(f3["seconds"], 4), "generate_rmat_gpu_s": round(g3, 3),
              "parity": "tests/test_gpu_configs.py::test_c3_s26_cycle4 (every result file vs the oracle)"}
        log(f"C3 S=26 4-cycle: {c3['ms_per_step']} ms/step, {c3['value'] / 1e9:.2f} G edges/s, "
            f"NLC lines {c3['nlcc_ms_per_step']} ms ({c3['nlcc_share']:.0%})")

    # the token-passing path with real work: config C5's search (S=27, explicit hash labels, 4-cycle) on the
    # GPU-generated graph, checked against the oracle's digest of the same search
    nlcc = None
    if args.nlcc == "auto" and world == 1 and not sharded:
        sys.path.insert(0, os.path.join(ROOT, "tests"))
        import pmtest
        cyc = os.path.join(ROOT, "patterns", "rmat_log2_cycle4_pattern")
        s5, p5, alphabet, salt = 27, 8, 256, 5
        m5, g5 = pm.rmat_matcher(s5, p5, cyc, device=0)
        t5 = time.perf_counter()
        m5.set_labels(pmtest.hash_labels(1 << s5, alphabet, salt=salt))
        lay5 = time.perf_counter() - t5
        f5 = m5.run_beta("", args.max_iterations)
        m5.run_beta("", args.max_iterations)
        raw5 = [_abi.RunStats() for _ in range(5)]
        t5 = time.perf_counter()
        for st5 in raw5:
            m5.run_beta_into(st5, args.max_iterations)
        e5 = (time.perf_counter() - t5) / len(raw5)
        r5 = [x.as_dict() for x in raw5]
        last = r5[-1]
        nl_s = sum(r["nlcc_seconds"] for r in r5) / len(r5)
        nlcc = {"workload": f"R-MAT scale-{s5} (P_gen={p5}), labels hash32(v ^ {salt}) % {alphabet} (config C5's "
                            f"explicit labels, generated instead of ingested), rmat_log2_cycle4_pattern (4 cycle-check "
                            f"lines + TDS line), one GPU",
                "value": round(edges_of(last) / e5, 1), "unit": "edges/s", "ms_per_step": round(e5 * 1e3, 3),
                "steps": len(r5), "edges_per_step": edges_of(last), "lcc_edges": last["lcc_edges"],
                "path_cycle_edges": last["nlcc_edges"], "tds_edges": last["tds_edges"], "walks": last["walks"],
                "iterations": last["iterations"], "split_lines": last["split_lines"],
                "line_overflows": last["line_overflows"], "exact_lines": last["exact_lines"],
                "nlc_lines_ms_per_step": round(nl_s * 1e3, 3), "nlc_lines_share": round(nl_s / e5, 4),
                "path_cycle_and_tds_edges_per_s_in_lines": round((last["nlcc_edges"] + last["tds_edges"]) /
                                                                 max(nl_s, 1e-9), 1),
                "first_search_s": round(f5["seconds"], 4), "generate_rmat_gpu_s": round(g5, 3),
                "labels_and_layout_s": round(lay5, 3)}
        fx5 = os.path.join(ROOT, "tests", "golden", f"rmat_s{s5}_p{p5}_cycle4_hash{alphabet}.json")
        if os.path.exists(fx5):
            fx = json.load(open(fx5))
            td = tempfile.mkdtemp(prefix="pmbench5")
            sf = m5.run_beta(td, args.max_iterations)
            diffs = pmtest.digest_diffs(fx["digest"], pmtest.result_digest(td, fx["nranks"]))
            for k_g, k_o in (("final_vertices", "final_vertices"), ("final_edges", "final_edges"),
                             ("lcc_edges", "lcc_edges"), ("nlcc_edges", "nlcc_edges"), ("tds_edges", "tds_edges"),
                             ("walks", "paths"), ("iterations", "iterations")):
                if sf[k_g] != fx["stats"][k_o] or last[k_g] != fx["stats"][k_o]:
                    diffs.append(f"{k_g}: gpu {last[k_g]}/{sf[k_g]} != oracle {fx['stats'][k_o]}")
            import shutil
            shutil.rmtree(td, ignore_errors=True)
            nlcc["fixture"] = {"file": os.path.relpath(fx5, ROOT), "match": not diffs}
            if diffs:
                invalid.append("C5-like search differs from the oracle's fixture: " + "; ".join(diffs[:4]))
        m5.close()
        log(f"NLCC config (S=27 hash-256 4-cycle): {nlcc['ms_per_step']} ms/step, {nlcc['value'] / 1e9:.2f} G edges/s, "
            f"lines {nlcc['nlc_lines_ms_per_step']} ms ({nlcc['nlc_lines_share']:.0%}), fixture "
            f"{nlcc.get('fixture', {}).get('match')}")

    # the sharded path at N=1: the same S=28 search through the code every rank of an N-GPU run executes (shard
    # generation + owner routing, delegates' combine, code exchange, T_pub exchange, replica hand-off) with a
    # one-rank RCCL communicator -- its fixed cost over the one-context step
    sharded1 = None
    if args.sharded_n1 == "auto" and world == 1 and not sharded:
        uid1 = pm.comm_unique_id()
        ms1, g1s = pm.rmat_shard_matcher(args.scale, args.p_gen, pattern_dir, 1, 0, uid1, device=0,
                                         hub_threshold=args.hub_threshold)
        for _ in range(max(args.warmup, 1)):
            ms1.run_beta("", args.max_iterations)
        raw1 = [_abi.RunStats() for _ in range(args.steps)]
        t1 = time.perf_counter()
        for st1 in raw1:
            ms1.run_beta_into(st1, args.max_iterations)
        e1 = (time.perf_counter() - t1) / args.steps
        l1 = raw1[-1].as_dict()
        info1 = ms1.comm_info()
        ms1.close()
        same = all(l1[k] == s0[k] for k in ("lcc_edges", "nlcc_edges", "tds_edges", "walks", "final_vertices",
                                            "final_edges", "iterations"))
        if not same:
            invalid.append("the sharded path at N=1 differs from the one-context search")
        sharded1 = {"ms_per_step": round(e1 * 1e3, 4), "value": round(edges_of(l1) / e1, 1), "unit": "edges/s",
                    "over_one_context": round(e1 / (elapsed / args.steps), 4), "steps": args.steps,
                    "transport": info1["transport"], "comm_ranks": info1["comm_ranks"],
                    "comm_calls_per_search": l1["comm_calls"], "comm_bytes": l1["comm_bytes"],
                    "replica_rows": l1["replica_rows"], "shard_sharded_ms": round(l1["shard_sharded_ms"], 4),
                    "same_counters_as_one_context": same, "generate_and_route_s": round(g1s, 3)}
        log(f"sharded path at N=1: {sharded1['ms_per_step']} ms/step ({sharded1['over_one_context']}x the one-context "
            f"step), {l1['comm_calls']} collectives")

    cpu = None
    if args.cpu_baseline == "auto" and world == 1:
        sys.path.insert(0, os.path.join(ROOT, "oracle"))
        import oracle
        cscale = min(args.scale, args.cpu_scale)
        threads, cpu_info = host_cpu_share()
        t0 = time.time()
        gc = pm.rmat_graph(cscale, args.p_gen, device=0)
        runs = [oracle.run(gc.off, gc.col, pattern_dir, None, max_iterations=args.max_iterations, threads=threads)
                for _ in range(3)]
        secs = sorted(r["seconds"] for r in runs)
        so = runs[0]
        oe = edges_of(so)
        # the GPU on the same sample: value beside the CPU's, and the counters compared
        mc = pm.PatternMatcher(gc, pattern_dir, device=0)
        for _ in range(2):
            mc.run_beta("", args.max_iterations)
        tg = time.perf_counter()
        gs = [mc.run_beta("", args.max_iterations) for _ in range(10)]
        gsec = (time.perf_counter() - tg) / 10
        mc.close()
        ge = edges_of(gs[-1])
        if (oe, so["final_vertices"], so["final_edges"], so["paths"]) != (
                ge, gs[-1]["final_vertices"], gs[-1]["final_edges"], gs[-1]["walks"]):
            invalid.append(f"S={cscale} sample: oracle edges {oe} |S| {so['final_vertices']} |M| {so['final_edges']} "
                           f"walks {so['paths']} != GPU {ge} {gs[-1]['final_vertices']} {gs[-1]['final_edges']} "
                           f"{gs[-1]['walks']}")
        cpu = {"value": round(oe / secs[1], 1), "unit": "edges/s", "cores": threads, "kind": "port",
               "sample": f"one full pattern search of R-MAT S={cscale}, P_gen={args.p_gen}, {args.pattern} (a bounded "
                         f"sample of the headline search) by oracle/pm_oracle.cpp on {threads} host threads "
                         f"(rank-partitioned BSP), median of 3 runs ({', '.join(f'{x:.2f}' for x in secs)} s; "
                         f"{time.time() - t0:.1f}s incl. setup)",
               "edges": oe, "host_cpus": cpu_info,
               "gpu_value_same_sample": round(ge / gsec, 1),
               "gpu_over_cpu_same_sample": round(ge / gsec / (oe / secs[1]), 1)}
        # BASELINE.json configs[0] (C1): R-MAT S=21, P_gen=4, the reference's CPU-runnable case with 4 MPI
        # ranks: the oracle as 4 emulated ranks on 4 threads, the GPU search on the same input beside it
        g1 = pm.rmat_graph(21, 4, device=0)
        r1 = [oracle.run(g1.off, g1.col, pattern_dir, None, nranks=4, max_iterations=args.max_iterations, threads=4)
              for _ in range(3)]
        s1 = sorted(r["seconds"] for r in r1)
        m1 = pm.PatternMatcher(g1, pattern_dir, device=0)
        for _ in range(2):
            m1.run_beta("", args.max_iterations)
        t1 = time.perf_counter()
        q1 = [m1.run_beta("", args.max_iterations) for _ in range(10)]
        gs1 = (time.perf_counter() - t1) / 10
        m1.close()
        e1 = edges_of(r1[0])
        if (e1, r1[0]["final_vertices"], r1[0]["final_edges"]) != (edges_of(q1[-1]), q1[-1]["final_vertices"],
                                                                   q1[-1]["final_edges"]):
            invalid.append(f"C1 S=21: oracle edges {e1} |S| {r1[0]['final_vertices']} != GPU {edges_of(q1[-1])} "
                           f"{q1[-1]['final_vertices']}")
        cpu["c1_config"] = {"value": round(e1 / s1[1], 1), "unit": "edges/s", "cores": 4, "ranks": 4,
                            "seconds": [round(x, 4) for x in s1], "edges": e1,
                            "what": "BASELINE configs[0]: R-MAT S=21, P_gen=4, rmat_log2_tree_pattern, the oracle as 4 "
                                    "ranks on 4 host threads (median of 3)",
                            "gpu_value_same_input": round(edges_of(q1[-1]) / gs1, 1)}
        if os.path.exists(fx_path):
            ot = json.load(open(fx_path)).get("oracle_timing")
            if ot:
                cpu["same_workload_recorded"] = {
                    "value": ot["edges_per_s"], "cores": ot["threads"], "seconds": ot["seconds"],
                    "what": f"the oracle on the headline S={args.scale} search itself, timed once on a GPU box's host "
                            f"by tests/golden/make_rmat_fixture.py (median of {len(ot['seconds'])}; too slow and "
                            f"~100 GB for every bench run)"}

    out = {
        "metric": METRIC,
        "value": round(edges / elapsed, 1),
        "unit": "edges/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(elapsed / args.steps * 1e3, 4),
        "higher_is_better": True,
        "scaling": "strong",
        "vs_baseline": None,
        "dtype": "u16",
        "data": "synthetic R-MAT (generate_rmat.cpp stream, a,b,c,d=.57/.19/.19/.05, scrambled, symmetrized), "
                "degree-log2 labels",
        "config": {"workload": (f"R-MAT scale-{args.scale} (P_gen={args.p_gen}) + {args.pattern}, "
                                + (f"one search sharded over {world} GPU(s) (owner = id % {world}, delegates of degree "
                                   f">= {args.hub_threshold} split by target owner)" if sharded else "one GPU")
                                + ", full LCC+NLCC driver loop per step"),
                   "scale": args.scale, "p_gen": args.p_gen, "pattern": args.pattern,
                   "vertices": n, "directed_entries": nnz,
                   "parallelism": f"shard{world}" if sharded else "single"},
        "roofline": roofline,
        "cpu_baseline": cpu,
        "fixture": fixture,
        "c3_config": c3,
        "nlcc_config": nlcc,
        "shards": shards,
        "sharded_n1": sharded1,
        # one-time work outside the timed region (the reference's graph load + label init analogue)
        "setup_s": setup,
    }
    if invalid:
        for x in invalid:
            log("PARITY FAILURE: " + x)
        out["invalid"] = " | ".join(invalid)
    print(json.dumps(out), file=out_stream, flush=True)
    if dist is not None:
        dist.barrier()
        dist.destroy_process_group()
    return 3 if invalid else 0


if __name__ == "__main__":
    rc = main()
    sys.stdout.flush()
    sys.stderr.flush()
    sys.exit(rc or 0)
