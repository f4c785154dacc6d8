"""Probe (torch imported FIRST): does libmxd_amd.so bind torch's HIP runtime
(same SONAME libamdhip64.so.7 already loaded), and can its kernels then read
and write torch device tensors?  Prints one JSON line."""
import ctypes
import json
import os
import sys

import numpy as np
import torch

res = {"torch_cuda": torch.cuda.is_available()}
x0 = torch.zeros(16, device="cuda")  # torch's runtime opens the GPU first
torch.cuda.synchronize()

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "mlx-data_amd"))
from mlx_data_amd import capi  # noqa: E402

L = capi.lib()
maps = open("/proc/self/maps").read()
res["hip_runtimes"] = sorted({ln.split()[-1] for ln in maps.splitlines() if "libamdhip64" in ln})
n = ctypes.c_int(0)
res["mxd_device_count_rc"] = L.mxd_device_count(ctypes.byref(n))
res["mxd_device_count"] = n.value
try:
    img = torch.from_numpy(np.random.default_rng(0).integers(0, 256, (96, 128, 3), dtype=np.uint8)).cuda()
    out = torch.zeros((48, 64, 3), dtype=torch.uint8, device="cuda")
    torch.cuda.synchronize()
    arr, k = capi.make_images([dict(src=img.data_ptr(), src_stride=128 * 3, src_w=128, src_h=96, channels=3,
                                    resize_w=64, resize_h=48, crop_x=0, crop_y=0, crop_w=64, crop_h=48, flip=0,
                                    dst=out.data_ptr(), dst_stride=64 * 3)])
    capi.resize_crop_batch(arr, k, capi.MXD_U8, 0, None)
    L.mxd_device_synchronize(0) if hasattr(L, "mxd_device_synchronize") else None
    torch.cuda.synchronize()
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "oracle"))
    import oracle as O  # noqa: E402

    ref = O.resize(img.cpu().numpy(), 64, 48)
    res["resize_into_torch_maxdiff"] = int(np.abs(out.cpu().numpy().astype(int) - ref).max())
except Exception as e:  # noqa: BLE001
    res["error"] = repr(e)
print(json.dumps(res))
