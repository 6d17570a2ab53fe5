"""Superstep-0 layout rules (degree classes, slot -> row divisor, tile row-start
masks per alignment shift, 2-bit T_pub code): a host program compiled from
tests/native/layout_check.cpp against the product header pm_internal.hpp."""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "fuzzypatternmatching_amd", "csrc")


@pytest.mark.skipif(shutil.which("hipcc") is None and not os.path.exists("/opt/rocm/bin/hipcc"),
                    reason="hipcc not available")
def test_layout_rules(tmp_path):
    hipcc = shutil.which("hipcc") or "/opt/rocm/bin/hipcc"
    exe = tmp_path / "layout_check"
    subprocess.check_call([hipcc, "-O1", "-std=c++17", "-I", CSRC, "-o", str(exe),
                           os.path.join(ROOT, "tests", "native", "layout_check.cpp")])
    out = subprocess.run([str(exe)], capture_output=True, text=True, timeout=120)
    assert out.returncode == 0, out.stderr
    assert "layout checks passed" in out.stdout
