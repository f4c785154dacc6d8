"""CPU unit tests of the host planner (VERDICT r2 housekeeping: plan_wave,
band_rows and the band schedule get tests of their own): builds
tests/cpp/planner_unit.cpp against capi_internal.h and the in-tree
libmxd_amd.so (hipcc, host code only) and runs it; no device is touched."""
import os
import subprocess

import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
PKG = os.path.join(os.path.dirname(HERE), "mlx-data_amd")
HIPCC = "/opt/rocm/bin/hipcc"


@pytest.mark.skipif(not os.path.exists(HIPCC), reason="hipcc not available")
def test_planner_unit(tmp_path):
    exe = str(tmp_path / "planner_unit")
    subprocess.run([HIPCC, "-O1", "-std=c++17", "-I", os.path.join(os.path.dirname(HERE), "include"), "-I",
                    os.path.join(PKG, "csrc"), os.path.join(HERE, "cpp", "planner_unit.cpp"), "-L", PKG,
                    "-lmxd_amd", "-Wl,-rpath," + PKG, "-o", exe], check=True, capture_output=True, timeout=300)
    r = subprocess.run([exe], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0 and r.stdout.startswith("ok"), r.stdout + r.stderr
