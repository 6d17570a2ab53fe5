"""Superstep-0 kernel timing at several grid sizes (one process, interleaved rounds).

usage: ubench.py SCALE [grid,grid,...]   (grid 0 = the library default)
"""
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import fuzzypatternmatching_amd as pm  # noqa: E402
from fuzzypatternmatching_amd import _abi  # noqa: E402

scale = int(sys.argv[1]) if len(sys.argv) > 1 else 22
variants = [int(x) for x in sys.argv[2].split(",")] if len(sys.argv) > 2 else [0, 1, 8, 2, 4, 10, 12]
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
st = m.run_beta("", 64)
nbytes = st["lcc_first_bytes"]
print(f"S={scale}: superstep-0 algorithmic bytes {nbytes}, run_beta kernel {st['lcc_first_kernel_ms']:.4f} ms, "
      f"step {st['seconds'] * 1e3:.3f} ms")
for v in variants:
    xs = sorted(res[v])
    med = xs[len(xs) // 2]
    print(f"S={scale} variant {v:5d}: median {med*1e3:8.1f} us  min {xs[0]*1e3:8.1f} us  "
          f"{nbytes / (med * 1e-3) / 1e9:8.1f} GB/s")
