"""Round 6: the host-ending C4 pipeline (bench.py e2e_jpeg host_out: 128
ImageNet-shape JPEGs -> load_image -> resize 256 -> crop 224 -> image_to_float
-> batch(128) into host memory, prefetch(16, 16)) by the share of images
whose f32 results cross the link as u8 and are expanded on the host
(MXD_TUNE_F32_LINK: 0 = all, 1 = none, 2..99 = that percentage), alternating
the settings, two repetitions; one JSON line per run."""
import json
import os
import sys
import tempfile
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "mlx-data_amd"))
sys.path.insert(0, os.path.join(REPO, "tools"))

import bench_pipeline as bp  # noqa: E402
from mlx_data_amd import capi  # noqa: E402


def main():
    settings = [int(v) for v in (sys.argv[1] if len(sys.argv) > 1 else "0,1,80,65,50").split(",")]
    workers, batch, min_s = 16, 128, 3.0
    root = tempfile.mkdtemp()
    files = bp.make_files(root, "c4", batch)
    bp.run_surface(files, batch, workers, "fused", 2 * workers)
    for rep in range(2):
        for v in settings:
            capi.set_tuning(capi.MXD_TUNE_F32_LINK, v)
            bp.run_surface(files, batch, workers, "fused", workers)
            capi.narrow_returns(reset=True)
            repeat = 8 * workers
            while True:
                n, dt = bp.run_surface(files, batch, workers, "fused", repeat)
                if dt >= min_s:
                    break
                repeat = int(repeat * 1.2 * min_s / max(dt, 1e-3)) + 1
            nar = capi.narrow_returns(reset=True)
            print(json.dumps({"f32_link": v, "rep": rep, "value": round(n / dt, 1), "images": n,
                              "seconds": round(dt, 3), "narrowed_share": round(nar / max(n, 1), 3)}), flush=True)
    capi.set_tuning(capi.MXD_TUNE_F32_LINK, 0)


if __name__ == "__main__":
    main()
