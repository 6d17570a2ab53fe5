"""Ablation timing of the superstep-0 kernel variants (one process, interleaved rounds)."""
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import fuzzypatternmatching_amd as pm  # noqa: E402
from fuzzypatternmatching_amd import _abi  # noqa: E402

scale = int(sys.argv[1]) if len(sys.argv) > 1 else 22
variants = [int(x) for x in sys.argv[2].split(",")] if len(sys.argv) > 2 else [0, 8, 9, 2, 7]
g = pm.rmat_graph(scale, 4)
m = pm.PatternMatcher(g, os.path.join(ROOT, "patterns", "rmat_log2_tree_pattern"))
lib = _abi.load()
res = {v: [] for v in variants}
for rnd in range(5):
    for v in variants:
        ms = ctypes.c_float()
        if lib.pm_debug_time_lcc_first(m._ctx, v, 5, ctypes.byref(ms)) != 0:
            raise RuntimeError(lib.pm_last_error(m._ctx))
        res[v].append(ms.value)
for v in variants:
    xs = sorted(res[v])
    print(f"S={scale} variant {v:2d}: median {xs[len(xs)//2]*1e3:8.1f} us  min {xs[0]*1e3:8.1f} us")
