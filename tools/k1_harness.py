"""Launches only the superstep-0 kernel (k_lcc_first) a few times on an R-MAT
graph generated on the GPU: the target of the rocprofv3 --pmc passes.

usage: k1_harness.py SCALE P_GEN [REPS] [VARIANT]
"""
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import fuzzypatternmatching_amd as pm  # noqa: E402
from fuzzypatternmatching_amd import _abi  # noqa: E402

scale, p_gen = int(sys.argv[1]), int(sys.argv[2])
reps = int(sys.argv[3]) if len(sys.argv) > 3 else 3
variant = int(sys.argv[4]) if len(sys.argv) > 4 else 0
m, _ = pm.rmat_matcher(scale, p_gen, os.path.join(ROOT, "patterns", "rmat_log2_tree_pattern"))
lib = _abi.load()
ms = ctypes.c_float()
if lib.pm_debug_time_lcc_first(m._ctx, variant, reps, ctypes.byref(ms)) != 0:
    raise RuntimeError(lib.pm_last_error(m._ctx))
print(f"k_lcc_first variant {variant}: {ms.value:.4f} ms per launch ({reps} + 1 warm launches)", flush=True)
m.close()
