"""Timing breakdown of jpeg_prog by scan kind (diagnostic): 128 C4-shape
progressive files (bench_pipeline's c4p) decoded at identity geometry by
mxd_jpeg_resize_crop_host, median of 8 calls, with MXD_PROG_SKIP masking
DC-first (1), AC-first (2) or AC-refinement (4) scans -- each setting in its
own process (the switch is read once)."""
import json
import os
import subprocess
import sys
import tempfile
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "mlx-data_amd"), os.path.join(REPO, "tools"), os.path.join(REPO, "tests")]


def run(root):
    import numpy as np
    from mlx_data_amd import capi
    from test_gpu_jpeg_entropy import _decode_gpu

    files = sorted(os.path.join(dp, f) for dp, _, fs in os.walk(root) for f in fs if f.endswith(".jpg"))
    datas = [open(f, "rb").read() for f in files]
    _decode_gpu(datas)
    ts = []
    for _ in range(8):
        t = time.perf_counter()
        _decode_gpu(datas)
        ts.append(time.perf_counter() - t)
    print(json.dumps({"skip": int(os.environ.get("MXD_PROG_SKIP", "0")), "ms_per_call": round(1e3 * float(np.median(ts)), 2)}),
          flush=True)


if __name__ == "__main__":
    if len(sys.argv) > 1:
        run(sys.argv[1])
        sys.exit(0)
    import bench_pipeline as bp

    with tempfile.TemporaryDirectory() as root:
        bp.make_files(root, "c4p", 128)
        for skip in (0, 1, 2, 4, 6, 7):
            env = dict(os.environ, MXD_PROG_SKIP=str(skip), MXD_DEVICE_PROGRESSIVE="1")
            subprocess.run([sys.executable, __file__, root], env=env, check=True, timeout=240)
