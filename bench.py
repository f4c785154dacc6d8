"""Benchmark: device-resident fused resize 256 + center crop 224 + f32 /255.

Workload (BASELINE.json configs[1]): a batch of 256 synthetic 1280x960 RGB uint8
images already resident in HBM -> image_resize_smallest_side(256) ->
image_center_crop(224, 224) -> float32 / 255, i.e. one fused kernel launch per
step over the whole batch (one "step" = one pass of the hot path over one
batch).  One process per GPU (torch.distributed.run for N > 1); every rank
processes its own batch (weak scaling, no collective on the data path);
`value` = images processed by all ranks / max-over-ranks wall time.

Extra fields:
  roofline      HBM roofline of the fused kernel: algorithmic bytes per launch
                (source footprint the 224x224 window depends on + f32 output, per
                image, x 256) / average launch time from HIP events recorded on
                the kernel's own stream; `traffic` from the committed rocprofv3
                PMC summary (profiles/*pmc*.json) when present.
  cpu_baseline  the oracle's C restatement of the reference CPU path
                (stbir-semantics resize -> crop -> batch -> numpy /255) on a
                bounded sample, on this host's cores (rank 0, N = 1 only).
  e2e           the same batch including pinned H2D of the sources and D2H of
                the f32 outputs (PCIe-inclusive rate; never `value`).
"""
import argparse
import ctypes
import glob
import json
import os
import sys
import threading
import time

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(REPO, "mlx-data_amd"))

import numpy as np  # noqa: E402

from mlx_data_amd import capi  # noqa: E402

BATCH = 256
SRC_W, SRC_H, C = 1280, 960, 3
SIZE, CROP = 256, 224
HBM_PEAK_GBS = 8000.0  # MI355X spec (MI355X_MICROARCH.md)


def footprint_bytes(src_w, src_h, c, rw, rh, cx, cy, cw, ch):
    """Source bytes the kept window depends on (rows x cols of the tap footprint)."""
    fx, nx, _ = capi.axis_taps(src_w, rw, cx, cw)
    fy, ny, _ = capi.axis_taps(src_h, rh, cy, ch)
    cols = int((fx + nx - 1).max() - fx.min() + 1)
    rows = int((fy + ny - 1).max() - fy.min() + 1)
    return rows * cols * c


def load_traffic():
    files = sorted(glob.glob(os.path.join(REPO, "profiles", "*pmc*.json")))
    if not files:
        return None
    try:
        with open(files[-1]) as f:
            return json.load(f).get("hbm_bytes_per_launch")
    except Exception:
        return None


def cpu_baseline(threads, sample):
    """Reference-algorithm CPU restatement (oracle) on `threads` host threads."""
    sys.path.insert(0, os.path.join(REPO, "oracle"))
    import oracle as O

    lib = O.lib()
    u8p = ctypes.POINTER(ctypes.c_uint8)
    rng = np.random.default_rng(123)
    srcs = [rng.integers(0, 256, (SRC_H, SRC_W, C), dtype=np.uint8) for _ in range(min(16, sample))]
    per_batch = 32
    nb = sample // per_batch

    def work(bidx, out):
        crops = np.empty((per_batch, CROP, CROP, C), np.uint8)
        for i in range(per_batch):
            s = srcs[(bidx * per_batch + i) % len(srcs)]
            rc = lib.orc_resize_smallest_side_center_crop(s.ctypes.data_as(u8p), SRC_W, SRC_H, C, SIZE, CROP, CROP,
                                                          crops[i].ctypes.data_as(u8p))
            assert rc == 0
        batch = O.batch(list(crops), 0)
        out[bidx] = batch.astype("float32") / 255

    outs = [None] * nb
    t0 = time.perf_counter()
    next_b = [0]
    lock = threading.Lock()

    def worker():
        while True:
            with lock:
                b = next_b[0]
                next_b[0] += 1
            if b >= nb:
                return
            work(b, outs)

    ts = [threading.Thread(target=worker) for _ in range(threads)]
    for t in ts:
        t.start()
    for t in ts:
        t.join()
    dt = time.perf_counter() - t0
    return {"value": round(nb * per_batch / dt, 2), "unit": "images/s", "cores": threads, "kind": "port",
            "sample": f"{nb * per_batch} images 1280x960 -> resize 256 -> crop 224 -> batch {per_batch} -> f32/255 "
                      f"(oracle C restatement of stbir + numpy normalize, {threads} threads, GIL released in C)"}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--batch", type=int, default=BATCH)
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--no-e2e", action="store_true")
    ap.add_argument("--cpu-sample", type=int, default=512)
    ap.add_argument("--no-copy", action="store_true")
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    capi.lib()  # bind /opt/rocm HIP runtime before torch (which bundles its own) loads
    dist = None
    if world > 1:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        import torch.distributed as dist  # noqa: F811

        dist.init_process_group("gloo", rank=rank, world_size=world)

    def barrier():
        if dist is not None:
            dist.barrier()

    def max_over_ranks(x):
        if dist is None:
            return x
        import torch

        t = torch.tensor([x], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        return float(t.item())

    dev = local
    capi.check(capi.lib().mxd_set_device(dev))
    B = args.batch
    rw, rh = capi.resize_smallest_side_dims(SRC_W, SRC_H, SIZE)
    cx, cy = capi.center_crop_origin(rw, rh, CROP, CROP)
    pitch = SRC_W * C
    img_bytes = pitch * SRC_H
    out_bytes = CROP * CROP * C * 4

    rng = np.random.default_rng(1000 + rank)
    host_src = rng.integers(0, 256, (B, SRC_H, SRC_W, C), dtype=np.uint8)
    stream = capi.Stream(dev)
    src = capi.DeviceBuffer(B * img_bytes, dev)
    dst = capi.DeviceBuffer(B * out_bytes, dev)
    src.upload(host_src, stream=stream)
    entries = [dict(src=src.ptr + i * img_bytes, src_stride=pitch, src_w=SRC_W, src_h=SRC_H, channels=C,
                    resize_w=rw, resize_h=rh, crop_x=cx, crop_y=cy, crop_w=CROP, crop_h=CROP, flip=0,
                    dst=dst.ptr + i * out_bytes, dst_stride=CROP * C * 4) for i in range(B)]
    imgs, n = capi.make_images(entries)
    L = capi.lib()
    sh = ctypes.c_void_p(stream.handle)

    def step():
        capi.check(L.mxd_resize_crop_batch(imgs, n, capi.MXD_F32_DIV255, dev, sh))

    for _ in range(args.warmup):
        step()
    stream.synchronize()
    e0, e1 = capi.Event(), capi.Event()
    barrier()
    stream.synchronize()
    t0 = time.perf_counter()
    e0.record(stream)
    for _ in range(args.steps):
        step()
    e1.record(stream)
    stream.synchronize()
    t1 = time.perf_counter()
    barrier()
    wall = max_over_ranks(t1 - t0)
    kernel_ms = e0.elapsed_ms(e1) / args.steps

    fp = footprint_bytes(SRC_W, SRC_H, C, rw, rh, cx, cy, CROP, CROP)
    alg_bytes = B * (fp + out_bytes)
    achieved = alg_bytes / (kernel_ms * 1e-3) / 1e9
    traffic = load_traffic()
    copy_gbs = capi.copy_bandwidth(1 << 30, dev, 20) if not args.no_copy else None

    e2e = None
    if not args.no_e2e and world == 1:
        pin_src = ctypes.c_void_p()
        pin_dst = ctypes.c_void_p()
        capi.check(L.mxd_malloc_pinned(ctypes.byref(pin_src), ctypes.c_size_t(B * img_bytes)))
        capi.check(L.mxd_malloc_pinned(ctypes.byref(pin_dst), ctypes.c_size_t(B * out_bytes)))
        ctypes.memmove(pin_src, host_src.ctypes.data, B * img_bytes)
        k = max(3, args.steps // 10)

        def e2e_step():
            capi.check(L.mxd_memcpy_h2d_async(ctypes.c_void_p(src.ptr), pin_src, ctypes.c_size_t(B * img_bytes), sh))
            step()
            capi.check(L.mxd_memcpy_d2h_async(pin_dst, ctypes.c_void_p(dst.ptr), ctypes.c_size_t(B * out_bytes), sh))

        e2e_step()
        stream.synchronize()
        ta = time.perf_counter()
        for _ in range(k):
            e2e_step()
        stream.synchronize()
        tb = time.perf_counter()
        e2e = {"value": round(B * k / (tb - ta), 1), "unit": "images/s", "steps": k,
               "note": "pinned H2D of 256 sources (943.7 MB) + fused kernel + D2H of f32 outputs (154 MB), "
                       "serialized on one stream"}
        capi.check(L.mxd_free_pinned(pin_src))
        capi.check(L.mxd_free_pinned(pin_dst))

    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu:
        cpu = cpu_baseline(min(16, os.cpu_count() or 1), args.cpu_sample)

    if rank == 0:
        value = world * B * args.steps / wall
        line = {
            "metric": "images/sec device-resident resize+crop→224×224 at 1/2/4/8 MI355X",
            "value": round(value, 1),
            "unit": "images/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(wall / args.steps * 1e3, 4),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "u8->f32",
            "data": "synthetic (seeded uniform random uint8 RGB, resident in HBM)",
            "config": {"workload": "C2: 256 x 1280x960 RGB u8 in HBM -> resize_smallest_side 256 -> "
                                   "center_crop 224 -> f32/255, one fused launch per batch",
                       "global_batch": world * B, "per_gpu_batch": B, "parallelism": f"replicas x{world} (no collective)"},
            "roofline": {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": traffic,
                         "alg_bytes_per_launch": alg_bytes, "alg_bytes_per_image": fp + out_bytes,
                         "kernel_ms_per_launch": round(kernel_ms, 5),
                         "copy_ceiling_gbs": round(copy_gbs, 1) if copy_gbs else None},
            "cpu_baseline": cpu,
            "e2e": e2e,
        }
        print(json.dumps(line), flush=True)
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
