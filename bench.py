#!/usr/bin/env python3
"""Benchmark: edges-traversed/s of the LCC+NLCC driver loop (BASELINE.json metric).

One "step" = one complete run_pattern_matching_beta pattern search
(run_pattern_matching_beta.cpp:539-1356: every LCC superstep, every NLC line,
post-processing and interleaved LCC calls until the loop terminates) over the
graph already resident in HBM.  Default workload at N = 1: the north_star
headline, R-MAT scale 28 from P_gen = 8 generator ranks (BASELINE.json
configs[3] on one GPU; 8.6 G directed entries in 288 GB of HBM), degree-log2
labels, examples/rmat_log2_tree_pattern.  The graph is generated on the GPU
(pm_rmat.hip, bit-identical to the generate_rmat stream).

Edges traversed: adjacency entries scanned by LCC senders
(full CSR degree in superstep 0 of the first call, |M[v]| later) plus those
scanned by NLCC/TDS initiators and relays; counted identically by the oracle.

N > 1 GPUs (torch.distributed.run, one process per GPU): ONE search over one
graph sharded across the ranks (owner = id % N rows per GPU, RCCL exchanges
between supersteps).  Weak scaling: the default graph
grows with N -- scale 24 + log2(N) from 4N generator ranks, so every GPU holds
the edge count of the one-GPU config; each process generates the stream of
its own generator ranks and the edges reach their owners in one all-to-all
(untimed setup).  `value` = edges traversed by the whole search / max-over-
ranks time.
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "edges-traversed/sec (LCC+NLCC) on R-MAT + tree pattern, 1/2/4/8 GPU"
HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md chip table: HBM3E 8.0 TB/s


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def main():
    import faulthandler
    faulthandler.enable()  # a fatal signal prints the Python stack
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--scale", type=int, default=None, help="default 24 + log2(N)")
    ap.add_argument("--p-gen", type=int, default=None, help="default 4 N")
    ap.add_argument("--pattern", default="rmat_log2_tree_pattern")
    ap.add_argument("--max-iterations", type=int, default=64)
    ap.add_argument("--cpu-baseline", choices=["auto", "off"], default="auto")
    ap.add_argument("--cpu-scale", type=int, default=24,
                    help="the CPU baseline runs the same search at min(scale, cpu-scale) (bounded sample)")
    ap.add_argument("--graph-cache", default=os.environ.get("PM_GRAPH_CACHE"),
                    help="directory: reuse / store the generated one-GPU graph (repeated profiling runs)")
    ap.add_argument("--gen", choices=["gpu", "host"], default="gpu",
                    help="R-MAT generator: gpu (pm_rmat.hip, adjacency built in HBM) or host (host/rmat.hpp)")
    ap.add_argument("--sharded", action="store_true",
                    help="take the sharded (RCCL) path even at N=1 (rehearsal of the multi-GPU code on one GPU)")
    ap.add_argument("--pmc", default=os.path.join(ROOT, "profiles", "r02_pmc_lcc_first.json"))
    args = ap.parse_args()

    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    dist = None
    sharded = world > 1 or args.sharded
    if sharded:
        import torch
        import torch.distributed as dist
        torch.cuda.set_device(local_rank)
        dist.init_process_group(backend="nccl")

    import numpy as np
    import fuzzypatternmatching_amd as pm

    if args.scale is None:
        args.scale = 28 if not sharded else 24 + max(0, (world - 1).bit_length())
    if args.p_gen is None:
        args.p_gen = 8 if not sharded else 4 * world
    pattern_dir = os.path.join(ROOT, "patterns", args.pattern)
    t0 = time.time()
    g = None
    setup = None
    if not sharded and args.gen == "gpu" and not args.graph_cache:
        m, gen_s = pm.rmat_matcher(args.scale, args.p_gen, pattern_dir, device=0)
        n, nnz = 1 << args.scale, (1 << args.scale) * 32
        ctx_s = time.time() - t0
        log(f"[rank {rank}] generated R-MAT S={args.scale} P_gen={args.p_gen} on the GPU: V={n} E={nnz} "
            f"in {gen_s:.1f}s; context (layout, tiling) ready after {ctx_s:.1f}s")
        setup = {"generate_rmat_gpu": round(gen_s, 3), "context_total": round(ctx_s, 3)}
        t0 = time.time()
    elif not sharded:
        cache = (os.path.join(args.graph_cache, f"rmat_s{args.scale}_p{args.p_gen}") if args.graph_cache else None)
        if cache and os.path.exists(cache + "_0_of_1"):
            g = pm.read_graph(cache)
        else:
            g = pm.rmat_graph(args.scale, args.p_gen)
            if cache:
                os.makedirs(args.graph_cache, exist_ok=True)
                pm.write_graph(cache, g, 1)
        n, nnz = g.n, g.nnz
        log(f"[rank {rank}] generated R-MAT S={args.scale} P_gen={args.p_gen}: V={g.n} E={g.nnz} "
            f"in {time.time() - t0:.1f}s")
        t0 = time.time()
        m = pm.PatternMatcher(g, pattern_dir, device=0)
    else:
        import torch
        n = 1 << args.scale
        src, dst = pm.rmat_edges(args.scale, args.p_gen, rank, world)
        log(f"[rank {rank}] generated {src.shape[0]} directed edges of R-MAT S={args.scale} P_gen={args.p_gen} "
            f"(generator ranks {rank}::{world}) in {time.time() - t0:.1f}s")
        t0 = time.time()
        off, col, deg = pm.partition_edges(src, dst, n, device=f"cuda:{local_rank}")
        del src, dst
        t = torch.tensor([int(off[-1])], dtype=torch.int64, device="cuda")
        if world > 1:
            dist.all_reduce(t)
        nnz = int(t.item())
        uid = [pm.comm_unique_id() if rank == 0 else None]
        dist.broadcast_object_list(uid, src=0)
        log(f"[rank {rank}] owner partitioning: {int(off[-1])} of {nnz} entries in {time.time() - t0:.1f}s")
        t0 = time.time()
        m = pm.ShardedPatternMatcher(n, off, col, deg, pattern_dir, world, rank, uid[0], device=local_rank)
        del off, col, deg
    log(f"[rank {rank}] uploaded graph in {time.time() - t0:.1f}s")

    def barrier_sync():
        if dist is not None:
            import torch
            torch.cuda.synchronize()
            dist.barrier()

    for _ in range(args.warmup):
        m.run_beta("", args.max_iterations)
    barrier_sync()
    t_start = time.perf_counter()
    stats = []
    for _ in range(args.steps):
        stats.append(m.run_beta("", args.max_iterations))
    barrier_sync()
    elapsed = time.perf_counter() - t_start
    # the stats of a sharded search already cover the whole graph (every rank reports the same)
    edges = sum(s["lcc_edges"] + s["nlcc_edges"] + s["tds_edges"] for s in stats)
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
        return

    achieved = kern_bytes / (kern_ms * 1e-3) / 1e9 if kern_ms > 0 else 0.0
    traffic = None
    if os.path.exists(args.pmc):
        try:
            pmc = json.load(open(args.pmc))
            if pmc.get("scale") == args.scale and pmc.get("p_gen") == args.p_gen and pmc.get("pattern") == args.pattern:
                traffic = pmc.get("hbm_bytes_per_launch")
        except Exception as ex:  # noqa: BLE001
            log(f"pmc file unreadable: {ex}")
    roofline = {"bound": "hbm", "kernel": "k_lcc_first", "achieved": round(achieved, 2), "peak": HBM_PEAK_GBS,
                "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": traffic,
                "algorithmic_bytes_per_launch": kern_bytes, "avg_launch_ms": round(kern_ms, 5),
                # the whole search step against the same bytes (every later superstep / NLC line moves
                # little): effective bandwidth of the step
                "step_achieved": round(kern_bytes / (elapsed / args.steps) / 1e9, 2),
                "step_frac": round(kern_bytes / (elapsed / args.steps) / 1e9 / HBM_PEAK_GBS, 4)}
    if lay is not None:
        real, slots, rows, tiles = lay[0], lay[1], lay[2], lay[3]
        setup = dict(setup or {}, label_major_layout_and_tiling=round(lay[6] * 1e-6, 3))
        roofline.update({"scanned_entries": real, "loaded_slots": slots,
                         "padded_slot_ratio": round(slots / max(real, 1), 4), "scanned_rows": rows, "tiles": tiles})

    cpu = None
    parity_fail = None
    if args.cpu_baseline == "auto" and not sharded:
        sys.path.insert(0, os.path.join(ROOT, "oracle"))
        import oracle
        cscale = min(args.scale, args.cpu_scale)
        threads = oracle.default_threads()
        t0 = time.time()
        if g is None or cscale != args.scale:
            g = pm.rmat_graph(cscale, args.p_gen, device=0)
        runs = [oracle.run(g.off, g.col, pattern_dir, None, max_iterations=args.max_iterations, threads=threads)
                for _ in range(3)]
        secs = sorted(r["seconds"] for r in runs)
        so = runs[0]
        oe = so["lcc_edges"] + so["nlcc_edges"] + so["tds_edges"]
        same = "the same workload" if cscale == args.scale else f"the same search at scale {cscale} (bounded sample)"
        cpu = {"value": round(oe / secs[1], 1), "unit": "edges/s", "cores": threads, "kind": "port",
               "sample": f"one full pattern search of {same} (S={cscale}, P_gen={args.p_gen}, {args.pattern}) by "
                         f"oracle/pm_oracle.cpp on {threads} host threads (rank-partitioned BSP), median of 3 runs "
                         f"({', '.join(f'{x:.2f}' for x in secs)} s; {time.time() - t0:.1f}s incl. setup)",
               "edges": oe}
        if cscale == args.scale:
            ge = s0["lcc_edges"] + s0["nlcc_edges"] + s0["tds_edges"]
            if oe != ge or so["final_vertices"] != s0["final_vertices"] or so["final_edges"] != s0["final_edges"]:
                parity_fail = (f"oracle edges {oe} |S| {so['final_vertices']} |M| {so['final_edges']} != GPU edges {ge} "
                               f"|S| {s0['final_vertices']} |M| {s0['final_edges']}")

    out = {
        "metric": METRIC,
        "value": round(edges / elapsed, 1),
        "unit": "edges/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(elapsed / args.steps * 1e3, 4),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "u16",
        "data": "synthetic R-MAT (generate_rmat.cpp stream, a,b,c,d=.57/.19/.19/.05, scrambled, symmetrized), "
                "degree-log2 labels",
        "config": {"workload": (f"R-MAT scale-{args.scale} (P_gen={args.p_gen}) + {args.pattern} on one GPU, "
                                f"full LCC+NLCC driver loop per step" if not sharded else
                                f"R-MAT scale-{args.scale} (P_gen={args.p_gen}) + {args.pattern}, one search "
                                f"sharded over {world} GPUs (owner = id % {world}), full LCC+NLCC driver loop "
                                f"per step"),
                   "scale": args.scale, "p_gen": args.p_gen, "pattern": args.pattern,
                   "vertices": n, "directed_entries": nnz,
                   "parallelism": "single" if not sharded else f"shard{world}"},
        "roofline": roofline,
        "cpu_baseline": cpu,
        # one-time work outside the timed region (the reference's graph load + label init analogue)
        "setup_s": setup,
    }
    if parity_fail:
        log("PARITY FAILURE: " + parity_fail)
        out["invalid"] = "GPU search differs from the oracle: " + parity_fail
    print(json.dumps(out), flush=True)
    if dist is not None:
        dist.barrier()
        dist.destroy_process_group()
    return 3 if parity_fail else 0


if __name__ == "__main__":
    rc = main()
    if os.environ.get("PM_DUMP_MAPS"):  # diagnostics: shared-object map for symbolising a crash at exit
        sys.stderr.write(open("/proc/self/maps").read())
    sys.stdout.flush()
    sys.stderr.flush()
    sys.exit(rc or 0)
