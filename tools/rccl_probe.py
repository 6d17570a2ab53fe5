"""One-rank RCCL collectives through the product library (librccl of /opt/rocm), one
subprocess per (size, op, env) so that a fatal signal is recorded, not fatal here.

usage: rccl_probe.py            (driver)   |   rccl_probe.py BYTES OP   (one case)
"""
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

if len(sys.argv) == 3:
    sys.path.insert(0, ROOT)
    from fuzzypatternmatching_amd import _abi
    lib = _abi.load()
    rc = lib.pm_debug_rccl_selftest(0, int(sys.argv[1]), int(sys.argv[2]))
    if rc < 0:
        print("error:", lib.pm_last_error(None).decode(), flush=True)
    sys.exit(rc & 0xFF)

envs = [("default", {}), ("NCCL_ALGO=Ring", {"NCCL_ALGO": "Ring"}), ("NCCL_PROTO=Simple", {"NCCL_PROTO": "Simple"})]
for name, extra in envs:
    for op in (0, 1):
        for bytes_ in (0, 8, 1 << 10, 1 << 16, 1 << 20, 1 << 24, 1 << 26, 1 << 28):
            env = dict(os.environ, **extra)
            r = subprocess.run([sys.executable, __file__, str(bytes_), str(op)], env=env, capture_output=True,
                               text=True, timeout=120)
            tail = (r.stdout + r.stderr).strip().splitlines()[-1:] if r.returncode else []
            print(f"{name:18s} op={'allgather' if op == 0 else 'allreduce'} bytes={bytes_:>10d} rc={r.returncode} {tail}",
                  flush=True)
