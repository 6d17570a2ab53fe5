"""Times the diagnostic variants of the superstep-0 kernel on one generated
R-MAT graph (phase breakdown: MODE bits in pm_kernels.hip, k_lcc_first).

usage: k1_variants.py SCALE P_GEN [VARIANTS...]
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

scale, p_gen = int(sys.argv[1]), int(sys.argv[2])
variants = [int(v) for v in sys.argv[3:]] or [0, 1, 2, 4, 8, 16, 32]
m, _ = pm.rmat_matcher(scale, p_gen, os.path.join(ROOT, "patterns", "rmat_log2_tree_pattern"))
lib = _abi.load()
for v in variants:
    ms = ctypes.c_float()
    if lib.pm_debug_time_lcc_first(m._ctx, v, 5, ctypes.byref(ms)) != 0:
        raise RuntimeError(lib.pm_last_error(m._ctx))
    print(f"variant {v}: {ms.value:.4f} ms per launch", flush=True)
m.close()
