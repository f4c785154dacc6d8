"""Benchmark: device-resident fused resize + crop (+ f32 /255) of image batches.

Default workload (BASELINE.json configs[1], the metric's configuration): a batch
of 256 synthetic 1280x960 RGB uint8 images already resident in HBM ->
image_resize_smallest_side(256) -> image_center_crop(224, 224) -> float32 / 255,
one fused kernel launch per step over the whole batch (one "step" = one pass
of the hot path over one batch).  One process per GPU (torch.distributed.run
for N > 1); every rank processes its own batch (weak scaling, no collective on
the data path; gloo only for the barrier and the max-over-ranks time);
`value` = images processed by all ranks / max-over-ranks wall time.

`--workload c3` (configs[2]: 512 mixed 480p-4K images -> 256 -> 224 u8),
`--workload c4` (configs[3], device part: 128 ImageNet-shape images per GPU ->
256 -> 224 f32; e2e adds the pinned copies) and `--workload c5` (configs[4]:
128 4K frames -> 512 -> random_crop 448 + hflip, u8) are the other
device-resident configurations; DESIGN.md quotes them.

Extra fields:
  roofline      HBM roofline of the fused kernel: algorithmic bytes per launch
                (source footprint the kept window depends on + output bytes, per
                image, summed over the batch) / average launch time from HIP
                events recorded on the kernel's own stream; `traffic` = HBM bytes
                per launch from the committed rocprofv3 PMC summary
                (profiles/**/*<workload>*pmc*.json, tools/pmc_traffic.py).
  cpu_baseline  the oracle's C restatement of the reference CPU path
                (stbir-semantics resize -> crop -> batch -> numpy /255) on a
                bounded sample, on this host's cores (rank 0, N = 1, c2 only).
  e2e           the same batch including pinned H2D of the sources and D2H of
                the outputs (PCIe-inclusive rate; never `value`).
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

HBM_PEAK_GBS = 8000.0  # MI355X spec (MI355X_MICROARCH.md)
C = 3
METRIC = "images/sec device-resident resize+crop→224×224 at 1/2/4/8 MI355X"

WORKLOADS = {
    "c2": dict(batch=256, f32=True,
               desc="C2: 256 x 1280x960 RGB u8 in HBM -> resize_smallest_side 256 -> center_crop 224 -> f32/255, "
                    "one fused launch per batch"),
    "c3": dict(batch=512, f32=False,
               desc="C3: 512 RGB u8 in HBM, sizes uniform over {640x480, 1280x720, 1280x960, 1920x1080, 2560x1440, "
                    "3840x2160} (seed 1) -> resize_smallest_side 256 -> center_crop 224, u8"),
    "c4": dict(batch=128, f32=True,
               desc="C4 (device part): 128 ImageNet-shape RGB u8 per GPU in HBM, sizes uniform over {500x375, "
                    "375x500, 500x333} (seed 2) -> resize_smallest_side 256 -> center_crop 224 -> f32/255 "
                    "(host JPEG decode not included; e2e adds pinned H2D/D2H)"),
    "c5": dict(batch=128, f32=False,
               desc="C5: 128 x 3840x2160 RGB u8 in HBM -> resize_smallest_side 512 -> random_crop 448 -> "
                    "random_h_flip 0.5 (seeded), u8"),
}
C3_SIZES = [(640, 480), (1280, 720), (1280, 960), (1920, 1080), (2560, 1440), (3840, 2160)]
C4_SIZES = [(500, 375), (375, 500), (500, 333)]


def footprint_bytes(src_w, src_h, c, rw, rh, cx, cy, cw, ch):
    """Source bytes the kept window depends on (rows x cols of the tap footprint)."""
    fx, nx, _ = capi.axis_taps(src_w, rw, cx, cw)
    fy, ny, _ = capi.axis_taps(src_h, rh, cy, ch)
    cols = int((fx + nx - 1).max() - fx.min() + 1)
    rows = int((fy + ny - 1).max() - fy.min() + 1)
    return rows * cols * c


def make_workload(name, batch, rank):
    """(sizes [(w, h)], geoms [(rw, rh, cx, cy, cw, ch, flip)], f32) for one rank."""
    if name == "c2":
        sizes = [(1280, 960)] * batch
    elif name == "c3":
        rng = np.random.default_rng(1)
        sizes = [C3_SIZES[i] for i in rng.integers(0, len(C3_SIZES), batch)]
    elif name == "c4":
        rng = np.random.default_rng(2)
        sizes = [C4_SIZES[i] for i in rng.integers(0, len(C4_SIZES), batch)]
    else:
        sizes = [(3840, 2160)] * batch
    rng = np.random.default_rng(3 + rank)
    geoms = []
    for (sw, sh) in sizes:
        if name == "c5":
            rw, rh = capi.resize_smallest_side_dims(sw, sh, 512)
            cx, cy = int(rng.integers(0, rw - 448 + 1)), int(rng.integers(0, rh - 448 + 1))
            geoms.append((rw, rh, cx, cy, 448, 448, int(rng.random() <= 0.5)))
        else:
            rw, rh = capi.resize_smallest_side_dims(sw, sh, 256)
            cx, cy = capi.center_crop_origin(rw, rh, 224, 224)
            geoms.append((rw, rh, cx, cy, 224, 224, 0))
    return sizes, geoms, WORKLOADS[name]["f32"]


def load_traffic(workload):
    """HBM bytes per launch measured for this workload's kernel (committed PMC summary)."""
    files = sorted(glob.glob(os.path.join(REPO, "profiles", "**", f"*{workload}*pmc*.json"), recursive=True))
    if not files:
        return None
    try:
        with open(files[-1]) as f:
            return json.load(f).get("hbm_bytes_per_launch")
    except Exception:
        return None


def cpu_baseline(threads, sample):
    """Reference-algorithm CPU restatement (oracle) on `threads` host threads, C2 shapes."""
    sys.path.insert(0, os.path.join(REPO, "oracle"))
    import oracle as O

    lib = O.lib()
    u8p = ctypes.POINTER(ctypes.c_uint8)
    rng = np.random.default_rng(123)
    srcs = [rng.integers(0, 256, (960, 1280, C), dtype=np.uint8) for _ in range(min(16, sample))]
    per_batch = 32
    nb = sample // per_batch

    def work(bidx, out):
        crops = np.empty((per_batch, 224, 224, C), np.uint8)
        for i in range(per_batch):
            s = srcs[(bidx * per_batch + i) % len(srcs)]
            rc = lib.orc_resize_smallest_side_center_crop(s.ctypes.data_as(u8p), 1280, 960, C, 256, 224, 224,
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


class Ranks:
    """Rank bookkeeping: one process per GPU, gloo for the barrier and the
    max-over-ranks time only (no collective on the data path)."""

    def __init__(self):
        self.world = int(os.environ.get("WORLD_SIZE", "1"))
        self.rank = int(os.environ.get("RANK", "0"))
        self.local = int(os.environ.get("LOCAL_RANK", "0"))
        self.dist = None
        if self.world > 1:
            os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
            import torch.distributed as dist

            if not dist.is_initialized():
                dist.init_process_group("gloo", rank=self.rank, world_size=self.world)
            self.dist = dist

    def barrier(self):
        if self.dist is not None:
            self.dist.barrier()

    def max(self, x):
        if self.dist is None:
            return x
        import torch

        t = torch.tensor([x], dtype=torch.float64)
        self.dist.all_reduce(t, op=self.dist.ReduceOp.MAX)
        return float(t.item())

    def close(self):
        if self.dist is not None:
            self.dist.destroy_process_group()


def timed_steps(ranks, step, sync, steps):
    """Exactly `steps` steps bracketed by a barrier and a device sync on both
    sides.  Returns (max-over-ranks wall seconds, this rank's seconds)."""
    sync()
    ranks.barrier()
    sync()
    t0 = time.perf_counter()
    for _ in range(steps):
        step()
    sync()
    t1 = time.perf_counter()
    ranks.barrier()
    return ranks.max(t1 - t0), t1 - t0


def bench_line(workload, world, batch, steps, warmup, wall, roofline, cpu, e2e):
    w = WORKLOADS[workload]
    return {
        "metric": METRIC,
        "value": round(world * batch * steps / wall, 1),
        "unit": "images/s",
        "n_gpus": world,
        "steps": steps,
        "warmup": warmup,
        "ms_per_step": round(wall / steps * 1e3, 4),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "u8->f32" if w["f32"] else "u8",
        "data": "synthetic (seeded uniform random uint8 RGB, resident in HBM)",
        "config": {"workload": w["desc"], "global_batch": world * batch, "per_gpu_batch": batch,
                   "parallelism": f"replicas x{world} (no collective)"},
        "roofline": roofline,
        "cpu_baseline": cpu,
        "e2e": e2e,
    }


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--workload", choices=sorted(WORKLOADS), default="c2")
    ap.add_argument("--batch", type=int, default=0, help="images per GPU (default: the workload's)")
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--no-e2e", action="store_true")
    ap.add_argument("--cpu-sample", type=int, default=512)
    ap.add_argument("--no-copy", action="store_true")
    args = ap.parse_args()

    capi.lib()  # bind /opt/rocm's HIP runtime before torch (which bundles its own) loads
    ranks = Ranks()
    dev = ranks.local
    capi.check(capi.lib().mxd_set_device(dev))
    B = args.batch or WORKLOADS[args.workload]["batch"]
    sizes, geoms, f32 = make_workload(args.workload, B, ranks.rank)
    elem = 4 if f32 else 1

    # Sources packed in one device buffer (256-B aligned slots, rows padded to
    # 16 B as mxd_resize_crop_host stages them), outputs NHWC.
    offs, pitches, total = [], [], 0
    for (sw, sh) in sizes:
        offs.append(total)
        pitches.append((sw * C + 15) // 16 * 16)
        total += (pitches[-1] * sh + 255) // 256 * 256 + int(os.environ.get("MXD_BENCH_SLOT_PAD", "0"))
    out_bytes = [g[4] * g[5] * C * elem for g in geoms]
    out_offs = np.concatenate([[0], np.cumsum(out_bytes)[:-1]]).astype(np.int64)
    rng = np.random.default_rng(1000 + ranks.rank)
    host = np.empty(total, np.uint8)
    if args.workload == "c2":
        host[:] = rng.integers(0, 256, total, dtype=np.uint8)
    else:  # one random 4K frame; every image is a slice of it (timing is data-independent)
        base = rng.integers(0, 256, 2160 * 3840 * C, dtype=np.uint8)
        for (sw, sh), o, pt in zip(sizes, offs, pitches):
            host[o:o + pt * sh] = base[:pt * sh]
    stream = capi.Stream(dev)
    src = capi.DeviceBuffer(total, dev)
    dst = capi.DeviceBuffer(int(sum(out_bytes)), dev)
    src.upload(host, stream=stream)
    entries = [dict(src=src.ptr + o, src_stride=pt, src_w=sw, src_h=sh, channels=C,
                    resize_w=g[0], resize_h=g[1], crop_x=g[2], crop_y=g[3], crop_w=g[4], crop_h=g[5], flip=g[6],
                    dst=dst.ptr + int(oo), dst_stride=g[4] * C * elem)
               for (sw, sh), o, pt, g, oo in zip(sizes, offs, pitches, geoms, out_offs)]
    imgs, n = capi.make_images(entries)
    L = capi.lib()
    hs = ctypes.c_void_p(stream.handle)
    mode = capi.MXD_F32_DIV255 if f32 else capi.MXD_U8

    def step():
        capi.check(L.mxd_resize_crop_batch(imgs, n, mode, dev, hs))

    for _ in range(args.warmup):
        step()
    e0, e1 = capi.Event(), capi.Event()
    stream.synchronize()
    e0.record(stream)
    wall, _ = timed_steps(ranks, step, stream.synchronize, args.steps)
    e1.record(stream)
    stream.synchronize()
    # The events bracket exactly the timed launches on the kernel's stream (the
    # barrier and host syncs between them add no device work).
    kernel_ms = e0.elapsed_ms(e1) / args.steps

    alg_bytes = sum(footprint_bytes(sw, sh, C, *g[:6]) for (sw, sh), g in zip(sizes, geoms)) + sum(out_bytes)
    achieved = alg_bytes / (kernel_ms * 1e-3) / 1e9
    copy_gbs = capi.copy_bandwidth(1 << 30, dev, 20) if not args.no_copy else None
    roofline = {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": load_traffic(args.workload),
                "alg_bytes_per_launch": int(alg_bytes), "alg_bytes_per_image": round(alg_bytes / B, 1),
                "kernel_ms_per_launch": round(kernel_ms, 5),
                "copy_ceiling_gbs": round(copy_gbs, 1) if copy_gbs else None}

    e2e = None
    if not args.no_e2e and ranks.world == 1:
        in_b, out_b = total, int(sum(out_bytes))
        pin_src, pin_dst = ctypes.c_void_p(), ctypes.c_void_p()
        capi.check(L.mxd_malloc_pinned(ctypes.byref(pin_src), ctypes.c_size_t(in_b)))
        capi.check(L.mxd_malloc_pinned(ctypes.byref(pin_dst), ctypes.c_size_t(out_b)))
        ctypes.memmove(pin_src, host.ctypes.data, in_b)
        k = max(3, args.steps // 10)

        def e2e_step():
            capi.check(L.mxd_memcpy_h2d_async(ctypes.c_void_p(src.ptr), pin_src, ctypes.c_size_t(in_b), hs))
            step()
            capi.check(L.mxd_memcpy_d2h_async(pin_dst, ctypes.c_void_p(dst.ptr), ctypes.c_size_t(out_b), hs))

        e2e_step()
        stream.synchronize()
        ta = time.perf_counter()
        for _ in range(k):
            e2e_step()
        stream.synchronize()
        tb = time.perf_counter()
        e2e = {"value": round(B * k / (tb - ta), 1), "unit": "images/s", "steps": k,
               "note": f"pinned H2D of the {B} sources ({in_b / 1e6:.1f} MB) + fused kernel + D2H of the outputs "
                       f"({out_b / 1e6:.1f} MB), serialized on one stream"}
        # Double-buffered: two streams, each with its own device batch, so the
        # H2D of one batch overlaps the kernel and D2H of the other (PCIe is
        # full duplex).
        stream2 = capi.Stream(dev)
        hs2 = ctypes.c_void_p(stream2.handle)
        src2 = capi.DeviceBuffer(total, dev)
        dst2 = capi.DeviceBuffer(out_b, dev)
        pin_dst2 = ctypes.c_void_p()
        capi.check(L.mxd_malloc_pinned(ctypes.byref(pin_dst2), ctypes.c_size_t(out_b)))
        imgs2, _ = capi.make_images([dict(e, src=e["src"] - src.ptr + src2.ptr, dst=e["dst"] - dst.ptr + dst2.ptr)
                                     for e in entries])
        sets = ((src, dst, imgs, hs, pin_dst), (src2, dst2, imgs2, hs2, pin_dst2))

        def overlap_step():
            for s_buf, d_buf, im, h, pd in sets:
                capi.check(L.mxd_memcpy_h2d_async(ctypes.c_void_p(s_buf.ptr), pin_src, ctypes.c_size_t(in_b), h))
                capi.check(L.mxd_resize_crop_batch(im, n, mode, dev, h))
                capi.check(L.mxd_memcpy_d2h_async(pd, ctypes.c_void_p(d_buf.ptr), ctypes.c_size_t(out_b), h))

        overlap_step()
        stream.synchronize()
        stream2.synchronize()
        ta = time.perf_counter()
        for _ in range(k):
            overlap_step()
        stream.synchronize()
        stream2.synchronize()
        tb = time.perf_counter()
        e2e["overlapped"] = {"value": round(2 * B * k / (tb - ta), 1), "unit": "images/s", "steps": k,
                             "note": "two streams, two device batches: H2D of one overlaps kernel + D2H of the other"}
        capi.check(L.mxd_free_pinned(pin_src))
        capi.check(L.mxd_free_pinned(pin_dst))
        capi.check(L.mxd_free_pinned(pin_dst2))
        src2.free()
        dst2.free()

    cpu = None
    if ranks.rank == 0 and ranks.world == 1 and not args.no_cpu and args.workload == "c2":
        cpu = cpu_baseline(min(16, os.cpu_count() or 1), args.cpu_sample)

    if ranks.rank == 0:
        print(json.dumps(bench_line(args.workload, ranks.world, B, args.steps, args.warmup, wall, roofline, cpu,
                                    e2e)), flush=True)
    ranks.close()


if __name__ == "__main__":
    main()
