"""The JPEG decoder's vectorised inner kernels (32-bit guarded IDCT, integer
YCbCr->RGB, column-sum h2v2 upsampling) against their scalar statements on
random and extreme inputs -- tests/native/jpeg_kernels_check.cpp, built with
g++ here (both target clones exist; the running CPU picks one)."""
import os
import subprocess

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_vectorised_kernels_match_scalar(tmp_path):
    exe = tmp_path / "jpeg_kernels_check"
    src = os.path.join(REPO, "tests", "native", "jpeg_kernels_check.cpp")
    b = subprocess.run(["g++", "-O2", "-std=c++17", "-I", os.path.join(REPO, "mlx-data_amd", "csrc"), src, "-o",
                        str(exe)], capture_output=True, text=True, timeout=300)
    assert b.returncode == 0, b.stderr[-3000:]
    r = subprocess.run([str(exe)], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "0 failures" in r.stdout
    fast = int(r.stdout.split(",")[1].split()[0])
    assert fast > 50000  # the guarded int32 path is the common one
