"""Superstep-0 kernel timing: diagnostic variants / grid sizes (one process, interleaved rounds).

usage: ubench.py SCALE [P_GEN] [variant,variant,...]
  variant & 0xFFFF: diagnostic MODE (pm_kernels.hip k_lcc_first: 0 product, 1 no M stores,
  8 loads + label test only, 2 skip light tiles, 4 skip heavy tiles, 16 phase A only,
  32 phases A + B1, 512 no T_pub code atomics; 5 / 13: 5 / 6 waves per SIMD; 17 / 21 / 25: two tiles per wait at
  8 / 6 / 7 waves per SIMD; 29 / 33: three tiles per wait at 5 / 4; 37: four at 4), plus grid << 16 (grid blocks;
  0: the product grid -- only the product grid is valid in records mode, whose per-wave record slices follow it).
  The graph is generated on the GPU.
"""
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
# the ablation variants live in the diagnostics build (make -C fuzzypatternmatching_amd/csrc diag)
os.environ.setdefault("PM_LIB", os.path.join(ROOT, "fuzzypatternmatching_amd", "lib", "libpm_diag.so"))
sys.path.insert(0, ROOT)
import fuzzypatternmatching_amd as pm  # noqa: E402
from fuzzypatternmatching_amd import _abi  # noqa: E402

scale = int(sys.argv[1]) if len(sys.argv) > 1 else 22
p_gen = int(sys.argv[2]) if len(sys.argv) > 2 else 4
variants = [int(x, 0) for x in sys.argv[3].split(",")] if len(sys.argv) > 3 else [0, 1, 8, 2, 4]
m, _ = pm.rmat_matcher(scale, p_gen, os.path.join(ROOT, "patterns", "rmat_log2_tree_pattern"))
lib = _abi.load()
st = (ctypes.c_uint64 * 6)()
if lib.pm_debug_layout_stats(m._ctx, st, 6) != 0:
    raise RuntimeError(lib.pm_last_error(m._ctx))
real, slots, rows, tiles, ranges, heavy = list(st)
print(f"S={scale} P_gen={p_gen}: scanned rows {rows}, real entries {real}, loaded slots {slots} "
      f"(padding ratio {slots / max(real, 1):.3f}), tiles {tiles}, ranges {ranges}, heavy rows {heavy}", flush=True)
res = {v: [] for v in variants}
for rnd in range(5):
    for v in variants:
        ms = ctypes.c_float()
        if lib.pm_debug_time_lcc_first(m._ctx, v, 5, ctypes.byref(ms)) != 0:
            raise RuntimeError(lib.pm_last_error(m._ctx))
        res[v].append(ms.value)
s = m.run_beta("", 64)
nbytes = s["lcc_first_bytes"]
print(f"S={scale}: superstep-0 algorithmic bytes {nbytes}, run_beta kernel {s['lcc_first_kernel_ms']:.4f} ms, "
      f"step {s['seconds'] * 1e3:.3f} ms, lcc edges {s['lcc_edges']}")
for v in variants:
    xs = sorted(res[v])
    med = xs[len(xs) // 2]
    print(f"S={scale} variant {v:5d}: median {med*1e3:8.1f} us  min {xs[0]*1e3:8.1f} us  "
          f"{nbytes / (med * 1e-3) / 1e9:8.1f} GB/s  real-entry read {real * 4 / (med * 1e-3) / 1e9:8.1f} GB/s  "
          f"slot read {slots * 4 / (med * 1e-3) / 1e9:8.1f} GB/s", flush=True)
m.close()
