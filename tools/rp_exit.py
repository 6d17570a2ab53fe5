"""Diagnostics for the crash at the end of a rocprofv3-profiled search: runs one
search through the library in MODE and exits normally, with a native backtrace
printed on a fatal signal (tools/diag/libsegv_trace.so).

usage: rp_exit.py MODE   (lcc: superstep-0 kernel only; beta: run_beta + close;
                          beta_noclose: run_beta, context left to the exit;
                          beta_nocoop: run_beta with PM_FUSED_LINES=0)
"""
import ctypes
import faulthandler
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
faulthandler.enable()
ctypes.CDLL(os.path.join(ROOT, "tools", "diag", "libsegv_trace.so")).segv_trace_install()
import fuzzypatternmatching_amd as pm  # noqa: E402
from fuzzypatternmatching_amd import _abi  # noqa: E402

mode = sys.argv[1]
if mode == "beta_nocoop":  # the NLC lines without the cooperative (grid-barrier) kernel
    os.environ["PM_FUSED_LINES"] = "0"
m, _ = pm.rmat_matcher(16, 2, os.path.join(ROOT, "patterns", "rmat_log2_tree_pattern"))
if mode == "lcc":
    ms = ctypes.c_float()
    _abi.load().pm_debug_time_lcc_first(m._ctx, 0, 2, ctypes.byref(ms))
else:
    print(m.run_beta("", 100)["final_vertices"], flush=True)
if mode != "beta_noclose":
    m.close()
print("main done", flush=True)
with open("/proc/self/maps") as f:
    sys.stderr.write("".join(l for l in f if ".so" in l and "r-xp" in l))
