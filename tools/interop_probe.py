"""Probe: can the C ABI (/opt/rocm HIP runtime) write into torch-allocated
device memory (torch bundles its own HIP runtime)?  Prints one JSON line."""
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "mlx-data_amd"))
from mlx_data_amd import capi  # noqa: E402

capi.lib()
s = capi.Stream()  # the C ABI's runtime initialises the GPU first
import torch  # noqa: E402

res = {}
x = torch.zeros(1 << 20, dtype=torch.uint8, device="cuda")
torch.cuda.synchronize()
src = np.arange(1 << 20, dtype=np.uint8)
capi.check(capi.lib().mxd_memcpy_h2d_async(__import__("ctypes").c_void_p(x.data_ptr()),
                                            src.ctypes.data_as(__import__("ctypes").c_void_p),
                                            __import__("ctypes").c_size_t(src.nbytes),
                                            __import__("ctypes").c_void_p(s.handle)))
s.synchronize()
res["h2d_into_torch"] = bool(np.array_equal(x.cpu().numpy(), src))
# kernel writing into a torch tensor, reading a torch tensor
img = torch.from_numpy(np.random.default_rng(0).integers(0, 256, (64, 96, 3), dtype=np.uint8)).cuda()
out = torch.zeros((64, 96, 1), dtype=torch.uint8, device="cuda")
torch.cuda.synchronize()
arr, n = capi.make_pixmaps([dict(src=img.data_ptr(), src_stride=96 * 3, src_w=96, src_h=64, channels=3, dst_w=96,
                                 dst_h=64, dst=out.data_ptr(), dst_stride=96, params=capi.channel_reduction_preset("green"))])
capi.pixmap_batch(arr, n, capi.MXD_CHANNEL_REDUCTION, 0, s.handle)
s.synchronize()
res["kernel_on_torch_memory"] = bool(torch.equal(out[..., 0], img[..., 1]))
print(json.dumps(res))
