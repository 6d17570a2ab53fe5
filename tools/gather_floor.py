"""Floor of the first later superstep's neighbour-T_pub gathers at S=28 (pm_debug_gather_floor).

usage: gather_floor.py [SCALE] [P_GEN] [variants]   (default 28 8 0,1,2,3,4,5,6,7)
Superstep 0 runs (product kernel); its light survivors' alive M entries are collected as code indices in record
order and gather-only kernels are timed over them: 0 record order (index stream + code gather, 4 in flight per
lane), 1 index stream only, 2 XCD-sliced buckets, 3 the buckets spread over every XCD, 4 uniformly random, 5 sorted,
6 one 4-B load per distinct 128-B line of a 4 GiB buffer (FETCH_SIZE calibration), 7 the bucketing pass.
Prints one JSON object (median of 5 interleaved rounds of 5 launches each).
"""
import ctypes
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import fuzzypatternmatching_amd as pm  # noqa: E402
from fuzzypatternmatching_amd import _abi  # noqa: E402

scale = int(sys.argv[1]) if len(sys.argv) > 1 else 28
p_gen = int(sys.argv[2]) if len(sys.argv) > 2 else 8
variants = [int(x) for x in sys.argv[3].split(",")] if len(sys.argv) > 3 else list(range(8))
m, _ = pm.rmat_matcher(scale, p_gen, os.path.join(ROOT, "patterns", "rmat_log2_tree_pattern"))
lib = _abi.load()
res = {v: [] for v in variants}
info = {}
for rnd in range(int(os.environ.get("GF_ROUNDS", "5"))):
    for v in variants:
        ms = ctypes.c_float()
        inf = (ctypes.c_uint64 * 3)()
        if lib.pm_debug_gather_floor(m._ctx, v, 5, ctypes.byref(ms), inf) != 0:
            raise RuntimeError(lib.pm_last_error(m._ctx))
        res[v].append(ms.value)
        info[v] = list(inf)
        print(f"round {rnd} variant {v}: {ms.value * 1e3:.1f} us", file=sys.stderr, flush=True)
names = {0: "record order", 1: "index stream only", 2: "XCD-sliced", 3: "buckets on every XCD", 4: "uniform random",
         5: "sorted", 6: "distinct-line misses, 4 GiB", 7: "bucketing pass"}
n = next(iter(info.values()))[0]
out = {"scale": scale, "p_gen": p_gen, "entries": n, "code_bytes": next(iter(info.values()))[2], "variants": {}}
for v in variants:
    t = sorted(res[v])[len(res[v]) // 2]
    out["variants"][str(v)] = {"name": names[v], "us": round(t * 1e3, 2), "gathers_per_ns": round(n / (t * 1e6), 3),
                              "checksum": info[v][1]}
print(json.dumps(out))
