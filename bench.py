"""Benchmark: device-resident fused resize + crop (+ f32 /255) of image batches.

Default workload (BASELINE.json configs[1], the metric's configuration): a batch
of 256 synthetic 1280x960 RGB uint8 images already resident in HBM ->
image_resize_smallest_side(256) -> image_center_crop(224, 224) -> float32 / 255,
one fused kernel launch per step over the whole batch (one "step" = one pass
of the hot path over one batch).  Two source sets and two output batches
alternate step by step (different HBM addresses), so no step re-reads bytes
the previous one left in the 256 MiB Infinity Cache.  Consecutive steps are
independent batches and alternate over two HIP streams (`--streams`, each
stream with its own sets), the way the pipeline's prefetch workers each launch
on their own stream: one batch's drain overlaps the next one's start.  `value`
is images / wall time of the K steps; the roofline's per-launch kernel time is
measured separately, the same launches back to back on ONE stream.

Multi-GPU: one process per GPU.  `--gpus N` without a launcher spawns N rank
processes itself (RANK / LOCAL_RANK / WORLD_SIZE / MASTER_* in their
environment, before any GPU call); under torch.distributed.run the ranks come
from the environment.  Every rank processes its own batch on its own device
(weak scaling, no collective on the data path; gloo only for the barrier and
the max-over-ranks time); `value` = images of all ranks / max-over-ranks wall.

`--workload c3` (configs[2]: 512 mixed 480p-4K images -> 256 -> 224 u8),
`--workload c4` (configs[3], device part: 128 ImageNet-shape images per GPU ->
256 -> 224 f32) and `--workload c5` (configs[4]: 128 4K frames -> 512 ->
random_crop 448 + hflip, u8) are the other device-resident configurations;
`--workload c6` / `c7` (32 x 12 MP 4032x3024 / 24 MP 6000x4000 photos -> 256 ->
224 f32: 11.8:1 and 15.6:1 downscales) measure large ratios.  DESIGN.md
quotes them.

Extra fields:
  roofline      HBM roofline of the fused kernel: algorithmic bytes per launch
                (source footprint the kept window depends on + output bytes, per
                image, summed over the batch) / average launch time from HIP
                events recorded on the kernel's own stream (launches back to
                back on one stream); `sustained_gbs` = the same bytes per step
                / the timed wall per step (streams overlapped); `traffic` = HBM bytes
                per launch from the PMC summary recorded for this workload in
                profiles/traffic.json; `copy_ceiling_gbs` = the measured
                streaming-copy rate of this box (default cache policy),
                `copy_ceiling_nt_gbs` / `copy_ceiling_nt_sc1_gbs` the same
                copy with nontemporal (+ sc1) loads and stores, and
                `frac_of_streaming_copy_ceiling` the kernel against the
                better of those; `load_policy` the planner's choice for the
                kernel's source loads (nt for >= 128 MiB of sources).
  workloads     (c2 runs) per-launch records of C3 / C4 / C5 on the same box
                and build: kernel ms per launch, frac of 8 TB/s, traffic.
  cpu_baseline  the oracle's C restatement of the reference CPU path
                (stbir-semantics resize -> crop -> batch -> numpy /255) on a
                bounded sample at 1, 8 and all of this rank's cores (rank 0,
                N = 1, c2 only), with Pillow BILINEAR and torch-CPU bilinear
                antialias on all cores as independent CPU points.
  e2e_jpeg      the end-to-end JPEG pipeline (configs[3]'s chain on one GPU's
                slice): 128 ImageNet-shape JPEG files (seed
                2, Pillow q=90) through the operator surface -- load_image ->
                image_resize_smallest_side(256) -> image_center_crop(224) ->
                image_to_float -> batch(128, device=0) -> prefetch(16, 16) --
                repeated for >= 3 s, at the box's GPU_MAX_HW_QUEUES;
                `device_busy` (isolated device time per image x the rate) and
                the `bound` it implies; `host_out` the host-ending form
                (batch(128) into host memory, D2H inside the timed run) with
                its D2H GB/s; `hwq16` the device leg in a child process with
                16 hardware queues; `progressive` the files saved progressive
                (host entropy decode, device finish); beside them the same
                chain with the Huffman decode on the host, and the
                reference-algorithm CPU restatement (Pillow's libjpeg-turbo
                decode -> the oracle's C stbir -> crop -> /255) on the same
                files and this rank's cores.
  e2e           the product's host-resident path (mxd_resize_crop_host: host
                images in, host batch out; the kernel reads each image's
                source footprint and writes results over PCIe, from / to
                page-locked memory -- in place when the caller's buffers are):
                the PCIe-inclusive rate, never `value`.
"""
import argparse
import ctypes
import json
import os
import socket
import subprocess
import sys
import threading
import time

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(REPO, "mlx-data_amd"))

import numpy as np  # noqa: E402

# The JPEG pipeline's prefetch workers each launch on a stream of their own;
# HIP maps a process's streams onto GPU_MAX_HW_QUEUES hardware queues (the
# boxes export 4).  The benchmark runs at the box's setting (VERDICT r5 weak
# 9); e2e_jpeg adds the device-batch rate at 16 queues from a child process
# (`hwq16`), since the setting is read once, when HIP initialises.  The C2
# line does not depend on it (profiles/r04/hwq_bench.jsonl).

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
                    "(host JPEG decode not included; e2e adds the host path)"),
    "c5": dict(batch=128, f32=False,
               desc="C5: 128 x 3840x2160 RGB u8 in HBM -> resize_smallest_side 512 -> random_crop 448 -> "
                    "random_h_flip 0.5 (seeded), u8"),
    "c6": dict(batch=32, f32=True,
               desc="C6: 32 x 4032x3024 RGB u8 (12 MP) in HBM -> resize_smallest_side 256 -> center_crop 224 -> "
                    "f32/255 (11.8:1 downscale)"),
    "c7": dict(batch=32, f32=True,
               desc="C7: 32 x 6000x4000 RGB u8 (24 MP) in HBM -> resize_smallest_side 256 -> center_crop 224 -> "
                    "f32/255 (15.6:1 downscale)"),
}
C3_SIZES = [(640, 480), (1280, 720), (1280, 960), (1920, 1080), (2560, 1440), (3840, 2160)]
C4_SIZES = [(500, 375), (375, 500), (500, 333)]


def footprint_bytes(capi, src_w, src_h, c, rw, rh, cx, cy, cw, ch):
    """Source bytes the kept window depends on (rows x cols of the tap footprint)."""
    fx, nx, _ = capi.axis_taps(src_w, rw, cx, cw)
    fy, ny, _ = capi.axis_taps(src_h, rh, cy, ch)
    cols = int((fx + nx - 1).max() - fx.min() + 1)
    rows = int((fy + ny - 1).max() - fy.min() + 1)
    return rows * cols * c


def make_workload(capi, name, batch, rank, c3_sizes=None):
    """(sizes [(w, h)], geoms [(rw, rh, cx, cy, cw, ch, flip)], f32) for one rank."""
    if name == "c2":
        sizes = [(1280, 960)] * batch
    elif name == "c3":
        rng = np.random.default_rng(1)
        pool = c3_sizes or C3_SIZES
        sizes = [pool[i] for i in rng.integers(0, len(pool), batch)]
    elif name == "c4":
        rng = np.random.default_rng(2)
        sizes = [C4_SIZES[i] for i in rng.integers(0, len(C4_SIZES), batch)]
    elif name == "c6":
        sizes = [(4032, 3024)] * batch
    elif name == "c7":
        sizes = [(6000, 4000)] * batch
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


def kernel_name(capi, size, g, f32, policy):
    """Which kernel family runs the workload's first image under `policy`."""
    sw, sh = size
    e = dict(src_w=sw, src_h=sh, src_stride=(sw * C + 15) // 16 * 16, channels=C, resize_w=g[0], resize_h=g[1],
             crop_x=g[2], crop_y=g[3], crop_w=g[4], crop_h=g[5], flip=g[6], dst_stride=g[4] * C * (4 if f32 else 1))
    dt = capi.MXD_F32_DIV255 if f32 else capi.MXD_U8
    prev = capi.set_kernel_policy(policy)
    try:
        b = capi.describe_band_plan(e, dt)
        band = "resample_band (taps {taps}, rows/group {db}, window {nq} KiB, strips {nstrips}, ahead {la})".format(**b)
        if b["band"] and policy & capi.MXD_POLICY_PREFER_BAND:
            return band
        if capi.describe_plan(e, dt)["wave"]:
            return "resample_wave"
        return band if b["band"] else "resample_tiles"
    finally:
        capi.set_kernel_policy(prev)


def load_traffic(workload):
    """HBM bytes per launch measured for this workload's kernel: the record
    profiles/traffic.json names for it (file, tag and corrected bytes)."""
    path = os.path.join(REPO, "profiles", "traffic.json")
    try:
        with open(path) as f:
            rec = json.load(f).get(workload)
    except (OSError, ValueError):
        return None
    return None if rec is None else rec.get("hbm_bytes_per_launch")


def host_cores():
    """Cores this rank may use: the box's per-GPU CPU share when OMP_NUM_THREADS
    states it, else the affinity mask."""
    env = os.environ.get("OMP_NUM_THREADS")
    if env and env.isdigit() and int(env) > 0:
        return min(int(env), len(os.sched_getaffinity(0)))
    return len(os.sched_getaffinity(0))


def _pool_rate(threads, total, work):
    """Images/s of `work(batch_index)` over `total` batches on `threads` threads
    (each task builds a whole batch, like stream/Prefetch.cpp:29-56)."""
    nxt = [0]
    lock = threading.Lock()

    def worker():
        while True:
            with lock:
                b = nxt[0]
                nxt[0] += 1
            if b >= total:
                return
            work(b)

    t0 = time.perf_counter()
    ts = [threading.Thread(target=worker) for _ in range(threads)]
    for t in ts:
        t.start()
    for t in ts:
        t.join()
    return time.perf_counter() - t0


def cpu_baseline(sample_per_thread=96):
    """Reference-algorithm CPU restatement (oracle C code, GIL released) on C2
    shapes, at 1, 8 and all of this rank's cores, plus Pillow BILINEAR."""
    sys.path.insert(0, os.path.join(REPO, "oracle"))
    import oracle as O

    lib = O.lib()
    u8p = ctypes.POINTER(ctypes.c_uint8)
    rng = np.random.default_rng(123)
    srcs = [rng.integers(0, 256, (960, 1280, C), dtype=np.uint8) for _ in range(8)]
    per_batch = 8

    def port_batch(b):
        crops = np.empty((per_batch, 224, 224, C), np.uint8)
        for i in range(per_batch):
            s = srcs[(b * per_batch + i) % len(srcs)]
            rc = lib.orc_resize_smallest_side_center_crop(s.ctypes.data_as(u8p), 1280, 960, C, 256, 224, 224,
                                                          crops[i].ctypes.data_as(u8p))
            assert rc == 0
        return O.batch(list(crops), 0).astype("float32") / 255

    cores = host_cores()
    points = {}
    for n in sorted({1, min(8, cores), cores}):
        nb = max(1, n * sample_per_thread // per_batch)
        dt = _pool_rate(n, nb, port_batch)
        points[str(n)] = round(nb * per_batch / dt, 2)
    pil = None
    try:
        from PIL import Image

        pims = [Image.fromarray(s) for s in srcs]

        def pil_batch(b):
            out = np.empty((per_batch, 224, 224, C), np.uint8)
            for i in range(per_batch):
                r = pims[(b * per_batch + i) % len(pims)].resize((341, 256), Image.BILINEAR)
                out[i] = np.asarray(r)[16:240, 58:282]
            return out.astype("float32") / 255

        nb = max(1, cores * sample_per_thread // per_batch)
        dt = _pool_rate(cores, nb, pil_batch)
        pil = round(nb * per_batch / dt, 2)
    except ImportError:
        pass
    tch = None
    try:
        # torch CPU: uint8 NCHW (channels-last) bilinear with antialias (the
        # tent filter stbir uses when downsampling), intra-op threads = cores
        import torch
        import torch.nn.functional as F

        prev = torch.get_num_threads()
        torch.set_num_threads(cores)
        tsrc = torch.from_numpy(np.stack(srcs)).permute(0, 3, 1, 2).contiguous(memory_format=torch.channels_last)
        nb = max(1, cores * sample_per_thread // per_batch)
        t0 = time.perf_counter()
        for b in range(nb):
            r = F.interpolate(tsrc, size=(256, 341), mode="bilinear", antialias=True, align_corners=False)
            _ = r[:, :, 16:240, 58:282].permute(0, 2, 3, 1).float() / 255
        tch = round(nb * per_batch / (time.perf_counter() - t0), 2)
        torch.set_num_threads(prev)
    except Exception:  # noqa: BLE001  (an extra CPU point never fails the bench)
        pass
    return {"value": points[str(cores)], "unit": "images/s", "cores": cores, "kind": "port",
            "points": points, "pillow_bilinear": pil, "torch_cpu_antialias": tch,
            "sample": f"C2 shapes (1280x960 -> resize 256 -> crop 224 -> batch {per_batch} -> f32/255), "
                      f"{sample_per_thread} images per thread per point; oracle C restatement of stbir + numpy "
                      f"normalize, threads = cores; pillow_bilinear = Pillow resize(BILINEAR) + crop + /255 "
                      f"on all cores, torch_cpu_antialias = torch interpolate(bilinear, antialias) on uint8 + crop + /255 "
                      f"with cores intra-op threads (independent CPU points)"}


class Ranks:
    """Rank bookkeeping: one process per GPU, gloo for the barrier and the
    max-over-ranks time only (no collective on the data path, no torch GPU use)."""

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
    for i in range(steps):
        step(i)
    sync()
    t1 = time.perf_counter()
    ranks.barrier()
    return ranks.max(t1 - t0), t1 - t0


HEADLINE_WINDOWS = 3
LAUNCH_WINDOWS = 3
MIN_WINDOW_LAUNCHES = 100
MIN_WINDOW_MS = 20.0


def launch_windows(capi, stream, launch, sync):
    """Average time per launch, back to back on `stream`, from HIP events
    recorded on that stream: LAUNCH_WINDOWS windows of >= MIN_WINDOW_LAUNCHES
    launches and >= MIN_WINDOW_MS each (sized from a 10-launch pilot).
    Returns (median ms per launch, median host ms per call, every window's ms
    per launch)."""
    e0, e1 = capi.Event(), capi.Event()

    def window(k):
        sync()
        e0.record(stream)
        t0 = time.perf_counter()
        for i in range(k):
            launch(i)
        host = (time.perf_counter() - t0) * 1e3 / k
        e1.record(stream)
        stream.synchronize()
        return e0.elapsed_ms(e1) / k, host

    pilot, _ = window(10)
    k = max(MIN_WINDOW_LAUNCHES, int(MIN_WINDOW_MS / max(pilot, 1e-4)) + 1)
    k += k % 2  # whole alternations of the input/output sets
    runs = [window(k) for _ in range(LAUNCH_WINDOWS)]
    ks = sorted(r[0] for r in runs)
    hs = sorted(r[1] for r in runs)
    return ks[len(ks) // 2], hs[len(hs) // 2], [round(v, 5) for v in (r[0] for r in runs)]


def marketing_name(arch):
    """The agent's "Marketing Name" from rocminfo (a child process), or None."""
    out = ""
    for exe in ("rocminfo", "/opt/rocm/bin/rocminfo"):
        try:
            out = subprocess.run([exe], capture_output=True, text=True, timeout=30).stdout
        except (OSError, subprocess.SubprocessError):
            continue
        if out:
            break
    want = arch.split(":")[0]
    name = None
    for line in out.splitlines():
        line = line.strip()
        if line.startswith("Name:"):
            name = line.split(":", 1)[1].strip()
        elif line.startswith("Marketing Name:") and name and want and name.startswith(want):
            return line.split(":", 1)[1].strip() or None
    return None


def manifest(capi, dev):
    """Run manifest: device, ROCm, host cores, decoder."""
    m = {"host_cores": host_cores(), "jpeg": "native (libjpeg-turbo ISLOW semantics, mxd_jpeg_decode)"}
    try:
        name, arch, cus = capi.device_properties(dev)
        m.update(gpu=name, arch=arch, compute_units=cus)
    except Exception:  # noqa: BLE001  (a manifest never fails the bench)
        pass
    m["gpu_marketing_name"] = marketing_name(m.get("arch", ""))
    try:
        with open("/opt/rocm/.info/version") as f:
            m["rocm"] = f.read().strip()
    except OSError:
        pass
    return m


def bench_line(workload, world, batch, steps, warmup, wall, roofline, cpu, e2e, man=None):
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
                   "parallelism": f"dp{world} (one process per GPU, batch per rank, no collective)"},
        "roofline": roofline,
        "cpu_baseline": cpu,
        "e2e": e2e,
        "manifest": man,
    }


def free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def launch_ranks(n):
    """--gpus N without a launcher: N rank processes of this script, one per
    GPU, started before this process touches any GPU.  Rank 0's stdout (the
    JSON line) passes through; the exit code is the first failing rank's."""
    port = free_port()
    procs = []
    for r in range(n):
        env = dict(os.environ, WORLD_SIZE=str(n), RANK=str(r), LOCAL_RANK=str(r), LOCAL_WORLD_SIZE=str(n),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + sys.argv[1:], env=env,
                                      stdout=None if r == 0 else subprocess.DEVNULL))
    rc = 0
    for p in procs:
        p.wait()
        rc = rc or p.returncode
    return rc


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--workload", choices=sorted(WORKLOADS), default="c2")
    ap.add_argument("--batch", type=int, default=0, help="images per GPU (default: the workload's)")
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--no-e2e", action="store_true")
    ap.add_argument("--no-e2e-jpeg", action="store_true")
    ap.add_argument("--no-copy", action="store_true")
    ap.add_argument("--no-others", action="store_true", help="skip the C3/C4/C5 kernel records of a C2 run")
    # kernel policy (include/mxd_amd.h mxd_policy; tuning measurements only)
    ap.add_argument("--policy", type=int, default=0, help=argparse.SUPPRESS)
    # tuning: C3 drawn from these sizes only ("WxH,WxH")
    ap.add_argument("--c3-sizes", default="", help=argparse.SUPPRESS)
    # input/output sets that alternate step by step (1 = every step re-reads the same batch)
    ap.add_argument("--sets", type=int, default=2, help=argparse.SUPPRESS)
    # streams the timed steps alternate over (independent batches, like prefetch workers)
    ap.add_argument("--streams", type=int, default=2)
    # tuning knobs (include/mxd_amd.h mxd_tune; measurements only): band rows, groups ahead
    ap.add_argument("--tune-rows", type=int, default=0, help=argparse.SUPPRESS)
    ap.add_argument("--tune-la", type=int, default=0, help=argparse.SUPPRESS)
    ap.add_argument("--tune-desc", type=int, default=0, help=argparse.SUPPRESS)
    # one process, D devices: every step launches one batch slice per device
    # (the pipeline's own split, pipeline.cpp run_host); devices from
    # MXD_BENCH_SPLIT_DEVICES ("0,0" rehearses on one card) or range(D)
    ap.add_argument("--split-devices", type=int, default=1)
    # timing plumbing without a GPU (tests/test_bench_dist.py): each step sleeps
    ap.add_argument("--simulate", type=float, default=0.0, help=argparse.SUPPRESS)
    # e2e_jpeg's 16-queue leg (a child process of the default run)
    ap.add_argument("--e2e-jpeg-child", action="store_true", help=argparse.SUPPRESS)
    args = ap.parse_args()
    if args.e2e_jpeg_child:
        from mlx_data_amd import capi

        capi.check(capi.lib().mxd_set_device(0))
        print(json.dumps(e2e_jpeg(0, device_only=True)), flush=True)
        return

    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        sys.exit(launch_ranks(args.gpus))

    B = args.batch or WORKLOADS[args.workload]["batch"]
    if args.simulate > 0:
        ranks = Ranks()
        wall, _ = timed_steps(ranks, lambda i: time.sleep(args.simulate * (1 + ranks.rank)), lambda: None,
                              args.steps)
        if ranks.rank == 0:
            print(json.dumps(bench_line(args.workload, ranks.world, B, args.steps, args.warmup, wall, None, None,
                                        None)), flush=True)
        ranks.close()
        return

    from mlx_data_amd import capi

    capi.lib()  # bind /opt/rocm's HIP runtime first (torch, for gloo, bundles its own)
    ranks = Ranks()
    dev = int(os.environ.get("MXD_BENCH_DEVICE", ranks.local))  # rehearsal: several ranks on one GPU
    capi.check(capi.lib().mxd_set_device(dev))
    if args.policy:
        capi.set_kernel_policy(args.policy)
    if args.tune_rows:
        capi.set_tuning(capi.MXD_TUNE_BAND_ROWS, args.tune_rows)
    if args.tune_la:
        capi.set_tuning(capi.MXD_TUNE_BAND_LA, args.tune_la)
    if args.tune_desc:
        capi.set_tuning(capi.MXD_TUNE_DESC, args.tune_desc)
    c3_sizes = [tuple(int(v) for v in t.split("x")) for t in args.c3_sizes.split(",") if t]
    sizes, geoms, f32 = make_workload(capi, args.workload, B, ranks.rank, c3_sizes)
    elem = 4 if f32 else 1
    if args.split_devices > 1:
        split_run(capi, args, ranks, sizes, geoms, f32, B)
        ranks.close()
        return

    # Sources packed in one device buffer per set (256-B aligned slots, rows
    # padded to 16 B), outputs NHWC; two sets alternate step by step.
    offs, pitches, total = [], [], 0
    for (sw, sh) in sizes:
        offs.append(total)
        pitches.append((sw * C + 15) // 16 * 16)
        total += (pitches[-1] * sh + 255) // 256 * 256
    out_bytes = [g[4] * g[5] * C * elem for g in geoms]
    out_offs = np.concatenate([[0], np.cumsum(out_bytes)[:-1]]).astype(np.int64)
    rng = np.random.default_rng(1000 + ranks.rank)
    host = np.empty(total, np.uint8)
    if args.workload == "c2":
        host[:] = rng.integers(0, 256, total, dtype=np.uint8)
    else:  # one random 4K frame, repeated through every image (timing is data-independent)
        base = rng.integers(0, 256, 2160 * 3840 * C, dtype=np.uint8)
        for (sw, sh), o, pt in zip(sizes, offs, pitches):
            n = pt * sh
            host[o:o + n] = np.resize(base, n)
    stream = capi.Stream(dev)
    streams = [stream] + [capi.Stream(dev) for _ in range(max(1, args.streams) - 1)]
    mode = capi.MXD_F32_DIV255 if f32 else capi.MXD_U8
    L = capi.lib()
    hs = ctypes.c_void_p(stream.handle)
    sets = []
    # a stream never shares its input/output set with another stream
    nsets = max(1, args.sets)
    if args.streams > 1:
        nsets = (nsets + args.streams - 1) // args.streams * args.streams
    for _ in range(nsets):
        src = capi.DeviceBuffer(total, dev)
        dst = capi.DeviceBuffer(int(sum(out_bytes)), dev)
        src.upload(host, stream=stream)
        entries = [dict(src=src.ptr + o, src_stride=pt, src_w=sw, src_h=sh, channels=C,
                        resize_w=g[0], resize_h=g[1], crop_x=g[2], crop_y=g[3], crop_w=g[4], crop_h=g[5], flip=g[6],
                        dst=dst.ptr + int(oo), dst_stride=g[4] * C * elem)
                   for (sw, sh), o, pt, g, oo in zip(sizes, offs, pitches, geoms, out_offs)]
        imgs, n = capi.make_images(entries)
        sets.append((src, dst, imgs, n))

    shs = [ctypes.c_void_p(s.handle) for s in streams]

    def step(i, ns=len(streams)):
        _, _, imgs, n = sets[i % len(sets)]
        capi.check(L.mxd_resize_crop_batch(imgs, n, mode, dev, shs[i % ns]))

    def sync_all():
        for s in streams:
            s.synchronize()

    for i in range(args.warmup + len(streams)):
        step(i)
    # The headline: the K requested steps, timed as three windows of exactly K
    # steps each (barrier + device sync on both sides of every window); the
    # median window is `value` / `ms_per_step` (a window of 20 C2 steps lasts
    # ~3 ms, so a single one scatters by a few per cent).
    walls = sorted(timed_steps(ranks, step, sync_all, args.steps)[0] for _ in range(HEADLINE_WINDOWS))
    wall = walls[len(walls) // 2]
    # Per-launch kernel time for the roofline: the same launches back to back
    # on ONE stream, bracketed by HIP events on that stream (the kernel's own),
    # over windows of >= 100 launches and >= 20 ms each, independent of
    # --steps; the median of three windows.  host_ms: the submitting thread's
    # time per call (planning, descriptor upload, launch); when it reaches the
    # per-launch time the loop is host-bound.
    kernel_ms, host_ms, kernel_windows = launch_windows(capi, stream, lambda i: step(i, 1), sync_all)

    # The same launches with descriptor caching off: every batch uploads its
    # descriptor array (what a batch of fresh pointers costs); reported, not
    # the headline.  Same windows.
    fresh_ms = fresh_host_ms = None
    if args.steps > 0:
        prev = capi.set_kernel_policy(args.policy | capi.MXD_POLICY_NO_DESC_CACHE)
        for i in range(40):  # untimed: every descriptor slot allocated and written (twice)
            step(i, 1)
        fresh_ms, fresh_host_ms, _ = launch_windows(capi, stream, lambda i: step(i, 1), sync_all)
        capi.set_kernel_policy(prev)

    alg_bytes = sum(footprint_bytes(capi, sw, sh, C, *g[:6]) for (sw, sh), g in zip(sizes, geoms)) + sum(out_bytes)
    achieved = alg_bytes / (kernel_ms * 1e-3) / 1e9
    copy_gbs = capi.copy_bandwidth(1 << 30, dev, 20) if not args.no_copy else None
    # the streaming forms (nontemporal loads and stores, + sc1): the ceiling
    # the nt-load kernels are held to
    copy_nt = ({p: capi.copy_bandwidth(1 << 30, dev, 20, policy=p) for p in (1, 2)}
               if not args.no_copy else None)
    best_copy = max(copy_nt.values()) if copy_nt else None
    roofline = {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": load_traffic(args.workload),
                "alg_bytes_per_launch": int(alg_bytes), "alg_bytes_per_image": round(alg_bytes / B, 1),
                "kernel_ms_per_launch": round(kernel_ms, 5),
                "kernel_ms_windows": kernel_windows,
                "sustained_gbs": round(alg_bytes / (wall / max(1, args.steps)) / 1e9, 1) if args.steps else None,
                "headline_window_ms": [round(w * 1e3, 4) for w in walls],
                "ms_per_launch_fresh_descriptors": round(fresh_ms, 5) if fresh_ms else None,
                "host_ms_per_call": round(host_ms, 5) if args.steps else None,
                "host_ms_per_call_fresh": round(fresh_host_ms, 5) if fresh_host_ms else None,
                "kernel": kernel_name(capi, sizes[0], geoms[0], f32, args.policy),
                "copy_ceiling_gbs": round(copy_gbs, 1) if copy_gbs else None,
                "frac_of_copy_ceiling": round(achieved / copy_gbs, 4) if copy_gbs else None,
                "copy_ceiling_nt_gbs": round(copy_nt[1], 1) if copy_nt else None,
                "copy_ceiling_nt_sc1_gbs": round(copy_nt[2], 1) if copy_nt else None,
                "frac_of_streaming_copy_ceiling": round(achieved / best_copy, 4) if best_copy else None,
                # the planner's choice (batch.cpp: nt when the call's sources total >= 128 MiB)
                "load_policy": "nt" if sum(sw * sh * C for sw, sh in sizes) >= (128 << 20) else "default"}

    # the other single-GPU BASELINE configs' kernels on this box and build
    # (rank 0 of a single-rank C2 run; each a few seconds)
    others = None
    if ranks.world == 1 and args.workload == "c2" and not args.no_others and args.steps > 0:
        others = {w: workload_record(capi, dev, w) for w in ("c3", "c4", "c5")}

    e2e = None
    if not args.no_e2e and ranks.world == 1:
        e2e = e2e_host(capi, args, sizes, geoms, f32, host, offs, pitches, dev)

    cpu = None
    if ranks.rank == 0 and ranks.world == 1 and not args.no_cpu and args.workload == "c2":
        cpu = cpu_baseline()

    jpeg = None
    if ranks.rank == 0 and ranks.world == 1 and not args.no_e2e_jpeg and args.workload == "c2":
        jpeg = e2e_jpeg(dev, no_cpu=args.no_cpu)

    for src, dst, _, _ in sets:
        src.free()
        dst.free()
    if ranks.rank == 0:
        line = bench_line(args.workload, ranks.world, B, args.steps, args.warmup, wall, roofline, cpu, e2e,
                          manifest(capi, dev))
        line["config"]["streams"] = len(streams)
        line["e2e_jpeg"] = jpeg
        line["workloads"] = others
        print(json.dumps(line), flush=True)
    ranks.close()


def device_sets(capi, dev, sizes, geoms, f32, nsets, seed):
    """nsets (src, dst, images, n) of the workload on `dev` (bench layout)."""
    elem = 4 if f32 else 1
    offs, pitches, total = [], [], 0
    for (sw, sh) in sizes:
        offs.append(total)
        pitches.append((sw * C + 15) // 16 * 16)
        total += (pitches[-1] * sh + 255) // 256 * 256
    out_bytes = [g[4] * g[5] * C * elem for g in geoms]
    out_offs = np.concatenate([[0], np.cumsum(out_bytes)[:-1]]).astype(np.int64)
    # random bytes, a 64 MiB block repeated past that (timing is data-independent)
    host = np.resize(np.random.default_rng(seed).integers(0, 256, min(total, 64 << 20), dtype=np.uint8), total)
    sets = []
    for _ in range(nsets):
        src = capi.DeviceBuffer(total, dev)
        dst = capi.DeviceBuffer(int(sum(out_bytes)), dev)
        src.upload(host)
        entries = [dict(src=src.ptr + o, src_stride=pt, src_w=sw, src_h=sh, channels=C, resize_w=g[0], resize_h=g[1],
                        crop_x=g[2], crop_y=g[3], crop_w=g[4], crop_h=g[5], flip=g[6], dst=dst.ptr + int(oo),
                        dst_stride=g[4] * C * elem)
                   for (sw, sh), o, pt, g, oo in zip(sizes, offs, pitches, geoms, out_offs)]
        imgs, n = capi.make_images(entries)
        sets.append((src, dst, imgs, n))
    return sets, sum(out_bytes)


def workload_record(capi, dev, name):
    """Kernel record of another BASELINE config on the same box and build
    (VERDICT r5 next 5): its batch on one stream, two resident input/output
    sets, per-launch time from HIP events (launch_windows), frac of 8 TB/s
    from B_alg, and the PMC traffic profiles/traffic.json records for it."""
    B = WORKLOADS[name]["batch"]
    sizes, geoms, f32 = make_workload(capi, name, B, 0)
    sets, out_total = device_sets(capi, dev, sizes, geoms, f32, 2, 3000)
    stream = capi.Stream(dev)
    hs = ctypes.c_void_p(stream.handle)
    mode = capi.MXD_F32_DIV255 if f32 else capi.MXD_U8
    L = capi.lib()

    def launch(i):
        _, _, imgs, n = sets[i % 2]
        capi.check(L.mxd_resize_crop_batch(imgs, n, mode, dev, hs))

    try:
        for i in range(6):
            launch(i)
        ms, host_ms, windows = launch_windows(capi, stream, launch, stream.synchronize)
    finally:
        stream.synchronize()
        for src, dst, _, _ in sets:
            src.free()
            dst.free()
        stream.close()
    alg = sum(footprint_bytes(capi, sw, sh, C, *g[:6]) for (sw, sh), g in zip(sizes, geoms)) + out_total
    traffic = load_traffic(name)
    return {"images": B, "out": "f32" if f32 else "u8", "kernel_ms_per_launch": round(ms, 5),
            "kernel_ms_windows": windows, "images_per_s": round(B / (ms * 1e-3), 1),
            "alg_bytes_per_launch": int(alg), "achieved_gbs": round(alg / (ms * 1e-3) / 1e9, 1),
            "frac": round(alg / (ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4), "traffic": traffic,
            "traffic_over_alg": round(traffic / alg, 3) if traffic else None,
            "kernel": kernel_name(capi, sizes[0], geoms[0], f32, 0), "desc": WORKLOADS[name]["desc"]}


def split_run(capi, args, ranks, sizes, geoms, f32, B):
    """--split-devices D: one process drives D devices; every step is one
    global batch of D x B images whose contiguous slices (B each, one per
    device, op/Shard.cpp:11-20) are launched on each device's own HIP stream
    from this thread (launches are asynchronous); no collective."""
    env = os.environ.get("MXD_BENCH_SPLIT_DEVICES", "")
    devs = [int(d) for d in env.split(",") if d] or list(range(args.split_devices))
    devs = devs[:args.split_devices]
    D = len(devs)
    L = capi.lib()
    mode = capi.MXD_F32_DIV255 if f32 else capi.MXD_U8
    per = []
    for k, d in enumerate(devs):
        sets, _ = device_sets(capi, d, sizes, geoms, f32, 2, 2000 + k)
        st = capi.Stream(d)
        per.append((d, sets, st, ctypes.c_void_p(st.handle)))

    def step(i):
        for d, sets, _, hs in per:
            _, _, imgs, n = sets[i % 2]
            capi.check(L.mxd_resize_crop_batch(imgs, n, mode, d, hs))

    def sync_all():
        for _, _, st, _ in per:
            st.synchronize()

    for i in range(args.warmup + 2):
        step(i)
    wall, _ = timed_steps(ranks, step, sync_all, args.steps)
    line = bench_line(args.workload, D, B, args.steps, args.warmup, wall, None, None, None, manifest(capi, devs[0]))
    line["config"]["parallelism"] = (f"split{D} (one process; each step one global batch of {D} x {B} images, one "
                                     f"contiguous slice per device on its own HIP stream; no collective)")
    line["config"]["devices"] = devs
    for _, sets, _, _ in per:
        for src, dst, _, _ in sets:
            src.free()
            dst.free()
    print(json.dumps(line), flush=True)


def e2e_host(capi, args, sizes, geoms, f32, host, offs, pitches, dev):
    """The product host path (mxd_resize_crop_host): host sources in, host
    batch out, synchronous per call."""
    elem = 4 if f32 else 1
    outs = np.empty(sum(g[4] * g[5] * C for g in geoms), np.float32 if f32 else np.uint8)
    o = 0
    entries = []
    for (sw, sh), so, pt, g in zip(sizes, offs, pitches, geoms):
        entries.append(dict(src=host.ctypes.data + so, src_stride=pt, src_w=sw, src_h=sh, channels=C,
                            resize_w=g[0], resize_h=g[1], crop_x=g[2], crop_y=g[3], crop_w=g[4], crop_h=g[5],
                            flip=g[6], dst=outs.ctypes.data + o * elem, dst_stride=g[4] * C * elem))
        o += g[4] * g[5] * C
    imgs, n = capi.make_images(entries)
    mode = capi.MXD_F32_DIV255 if f32 else capi.MXD_U8
    capi.resize_crop_host(imgs, n, mode, dev)

    def timed(call, min_s=1.0):
        # whole calls until >= min_s (host-side rates scatter run to run; a
        # handful of calls measured 10-16 k img/s for the same C2 code)
        k, t0 = 0, time.perf_counter()
        while k < 3 or time.perf_counter() - t0 < min_s:
            call()
            k += 1
        return k, time.perf_counter() - t0

    k, dt_pageable = timed(lambda: capi.resize_crop_host(imgs, n, mode, dev))
    B = len(sizes)
    # The same call with the host images and the host batch in page-locked
    # memory (what a decoder writing into pinned buffers hands over): the
    # footprint rows and the results are DMA'd in place, no staging copies.
    L = capi.lib()
    pin_in, pin_out = ctypes.c_void_p(), ctypes.c_void_p()
    capi.check(L.mxd_malloc_pinned(ctypes.byref(pin_in), ctypes.c_size_t(host.nbytes)))
    capi.check(L.mxd_malloc_pinned(ctypes.byref(pin_out), ctypes.c_size_t(outs.nbytes)))
    try:
        hin = np.ctypeslib.as_array((ctypes.c_uint8 * host.nbytes).from_address(pin_in.value))
        hin[:] = host
        pentries = [dict(e, src=pin_in.value + (e["src"] - host.ctypes.data), dst=pin_out.value + (e["dst"] - outs.ctypes.data))
                    for e in entries]
        pimgs, pn = capi.make_images(pentries)
        capi.resize_crop_host(pimgs, pn, mode, dev)
        kp, dt_pinned = timed(lambda: capi.resize_crop_host(pimgs, pn, mode, dev))
        hout = np.ctypeslib.as_array((ctypes.c_uint8 * outs.nbytes).from_address(pin_out.value))
        same = bool(np.array_equal(hout, outs.view(np.uint8)))
    finally:
        capi.check(L.mxd_free_pinned(pin_in))
        capi.check(L.mxd_free_pinned(pin_out))
    return {"value": round(B * k / dt_pageable, 1), "unit": "images/s", "steps": k, "seconds": round(dt_pageable, 3),
            "pinned_value": round(B * kp / dt_pinned, 1), "pinned_steps": kp, "pinned_matches_pageable": same,
            "note": "mxd_resize_crop_host: each image's source footprint staged into page-locked memory by "
                    "helper threads and read by the fused kernel over PCIe, results written over PCIe into "
                    "page-locked staging and copied out; chunks overlapped over two slots; synchronous per call. "
                    "pinned_value: host images and batch in page-locked memory, read and written in place by the "
                    "kernel (zero copy)"}


def e2e_jpeg_hwq16(timeout=300):
    """The device-batch leg of e2e_jpeg in a child process with 16 hardware
    queues per process (GPU_MAX_HW_QUEUES is read once per process, when HIP
    initialises): the pipeline's 16 workers' streams then map to 16 queues
    instead of the box's 4."""
    env = dict(os.environ, GPU_MAX_HW_QUEUES="16", MXD_HW_QUEUES="16")
    try:
        r = subprocess.run([sys.executable, os.path.abspath(__file__), "--e2e-jpeg-child"], env=env, timeout=timeout,
                           capture_output=True, text=True)
    except subprocess.TimeoutExpired:
        return {"error": "timeout"}
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    if r.returncode != 0 or not lines:
        return {"error": f"rc {r.returncode}", "stderr": r.stderr[-400:]}
    return json.loads(lines[-1])


def e2e_jpeg(dev, workers=16, batch=128, min_s=3.0, no_cpu=False, device_only=False):
    """configs[3]'s chain on one GPU's slice (see the module docstring).
    Returns images/s of the device batch (Huffman decode on the GPU), the same
    with the Huffman decode on the host, the host-ending form, the
    progressive files, the device leg at 16 hardware queues, and the CPU
    restatement (device_only: the device batch rate alone)."""
    try:
        from PIL import Image  # noqa: F401  (the synthetic files and the CPU leg)
    except ImportError:
        return None
    import tempfile

    sys.path.insert(0, os.path.join(REPO, "tools"))
    import bench_pipeline as bp
    from mlx_data_amd import capi
    from mlx_data_amd import data as dx

    cores = host_cores()
    workers = min(workers, cores)
    with tempfile.TemporaryDirectory() as root:
        files = bp.make_files(root, "c4", batch)  # seed 2: ImageNet shapes 500x375 / 375x500 / 500x333
        mb = sum(os.path.getsize(f) for f in files) / 1e6

        def leg(variant):
            bp.run_surface(files, batch, workers, variant, 2 * workers)  # warm: contexts, pools, tables
            repeat = 4 * workers
            for _ in range(4):
                capi.host_stats(reset=True)
                bp._pipe_stats(True)
                n, dt = bp.run_surface(files, batch, workers, variant, repeat)
                if dt >= min_s:
                    break
                repeat = int(np.ceil(repeat * 1.2 * min_s / max(dt, 1e-3)))
            return round(n / dt, 1), n, round(dt, 3), host_split(n, dt)

        def device_us_per_image(variant, repeat=3):
            prev = capi.set_tuning(capi.MXD_TUNE_DEVICE_TIMING, 1)
            try:
                capi.device_stats(reset=True)
                k, _ = bp.run_surface(files, batch, 1, variant, repeat)
                ds = capi.device_stats(reset=True)
            finally:
                capi.set_tuning(capi.MXD_TUNE_DEVICE_TIMING, prev)
            return ds["device_s"] / max(k, 1) * 1e6

        def bound_of(sp, busy):
            """What limits the timed run: the device (its kernels' isolated
            time x the rate fills >= 85 % of the GPU), the worker threads
            (>= 85 % busy with little device wait), device calls (workers
            busy, mostly waiting on the device), or the feed."""
            if busy is not None and busy >= 0.85:
                return "device"
            if sp["worker_busy"] >= 0.85:
                return "host workers" if sp["device_wait_share"] < 0.5 else "device calls"
            return "feed (workers idle)"

        def host_split(n, dt):
            """Where the worker threads' time went in the timed run (microseconds
            per image, summed over threads): what bounds the pipeline."""
            hs = capi.host_stats(reset=True)
            ps = bp._pipe_stats(True)
            fetch, merge = ps[2] / n / 1e3, ps[3] / n / 1e3  # batch_fetch includes load_image + transforms
            busy = (fetch + merge) * n * 1e-6 / (workers * dt)
            wait = hs["wait_s"] / n * 1e6
            sp = {"load_image_us": round(ps[0] / n / 1e3, 2), "fetch_us": round(fetch, 2),
                  "batch_call_us": round(merge, 2), "device_wait_us": round(wait, 2),
                  "worker_busy": round(busy, 3), "device_wait_share": round(wait / max(fetch + merge, 1e-9), 3)}
            sp["bound"] = bound_of(sp, None)
            return sp

        value, n, dt, split = leg("device")
        # device time per image of the same call, isolated (one worker, the
        # chunks' first-kernel-to-last spans, MXD_TUNE_DEVICE_TIMING): times
        # the rate = the share of the GPU the 16-worker run keeps busy
        dev_us = device_us_per_image("device")
        busy = round(dev_us * 1e-6 * value, 3)
        split["device_us_per_image"] = round(dev_us, 2)
        split["device_busy"] = busy
        split["bound"] = bound_of(split, busy)
        if device_only:
            return {"value": value, "images": n, "seconds": dt, "host_split": split,
                    "hw_queues": os.environ.get("GPU_MAX_HW_QUEUES")}
        hostent, n2, dt2, split2 = leg("device_hostent")
        # host-ending form (north_star: the path starts and ends in host
        # memory): the f32 batch written to host memory -- page-locked
        # staging, D2H inside the timed run -- the reference consumer's numpy
        # batch (benchmarks/comparative/caltech101/mlx_data.py:40-51)
        capi.narrow_returns(reset=True)
        hvalue, hn, hdt, hsplit = leg("fused")
        hsplit["bound"] = bound_of(hsplit, None)
        # ABI 7: the f32 results cross the link as their u8 bytes and the host
        # writes u8 / 255 into the batch (MXD_TUNE_F32_LINK 0, the default)
        narrowed = capi.narrow_returns(reset=True)
        out_b = 224 * 224 * C * (1 if narrowed else 4)
        host_out = {"value": hvalue, "images": hn, "seconds": hdt, "d2h_gbs": round(hvalue * out_b / 1e9, 2),
                    "d2h_bytes_per_image": out_b, "narrow_return": bool(narrowed), "host_split": hsplit,
                    "chain": "as `chain`, but batch(128) into host memory (no device=): the batch's results are "
                             "copied device -> page-locked staging (as u8 when narrow_return: the host then "
                             "writes u8 / 255) -> the f32 batch array inside the timed run"}
        # the same leg with the f32 results over the link (MXD_TUNE_F32_LINK 1,
        # the pre-ABI-7 form), for the comparison
        prev_link = capi.set_tuning(capi.MXD_TUNE_F32_LINK, 1)
        try:
            wvalue, _, _, wsplit = leg("fused")
        finally:
            capi.set_tuning(capi.MXD_TUNE_F32_LINK, prev_link)
        host_out["f32_link"] = {"value": wvalue, "d2h_gbs": round(wvalue * 224 * 224 * C * 4 / 1e9, 2),
                                "worker_busy": wsplit["worker_busy"]}
        # the same files saved progressive: entropy-decoded on the host
        # (round 6 retired the device decode of progressive scans), finished
        # and resized on the GPU
        files_c4 = files
        files = bp.make_files(root, "c4p", batch)
        pvalue, pn, pdt, psplit = leg("device")
        progressive = {"value": pvalue, "images": pn, "seconds": pdt, "host_split": psplit,
                       "files": "the e2e files saved progressive (libjpeg's default progression); Huffman decode "
                                "of every scan on the host, IDCT + colour + resize on the GPU"}
        files = files_c4
        hwq16 = e2e_jpeg_hwq16()
        cpu = None
        if not no_cpu:
            sys.path.insert(0, os.path.join(REPO, "oracle"))
            import oracle as O

            lib = O.lib()
            u8p = ctypes.POINTER(ctypes.c_uint8)
            per = 8

            def cpu_batch(b):
                crops = np.empty((per, 224, 224, C), np.uint8)
                for i in range(per):
                    f = files[(b * per + i) % len(files)]
                    img = np.ascontiguousarray(np.asarray(Image.open(f).convert("RGB")))
                    h, w = img.shape[:2]
                    assert lib.orc_resize_smallest_side_center_crop(img.ctypes.data_as(u8p), w, h, C, 256, 224, 224,
                                                                    crops[i].ctypes.data_as(u8p)) == 0
                return crops.astype("float32") / 255

            nb = max(cores, int(np.ceil(2 * len(files) / per)))
            t = _pool_rate(cores, nb, cpu_batch)
            cpu = {"value": round(nb * per / t, 1), "unit": "images/s", "cores": cores, "kind": "port",
                   "sample": f"{nb * per} decodes of the same files on {cores} threads: Pillow (libjpeg-turbo) decode "
                             f"-> oracle C stbir resize 256 -> crop 224 -> astype(float32)/255"}
    return {"value": value, "unit": "images/s", "images": n, "seconds": dt, "workers": workers, "cores": cores,
            "batch": batch, "files": len(files), "file_mb": round(mb, 2),
            "host_entropy_value": hostent, "host_entropy_seconds": dt2, "cpu_restatement": cpu,
            "host_split": split, "host_entropy_split": split2, "progressive": progressive,
            "device_busy": split["device_busy"], "host_out": host_out, "hwq16": hwq16,
            "hw_queues": os.environ.get("GPU_MAX_HW_QUEUES"), "devices": dx.devices(),
            "device_entropy": dx.device_entropy(), "abi": capi.lib().mxd_abi_version(),
            "chain": "files -> load_image -> image_resize_smallest_side(256) -> image_center_crop(224, 224) -> "
                     "image_to_float -> batch(128, device=0) -> prefetch(workers, workers); Huffman + IDCT + "
                     "upsampling + colour + resize + crop + normalize on the GPU, markers parsed on the host; "
                     "host_entropy_value: the Huffman decode on the host (set_device_entropy(False))"}


if __name__ == "__main__":
    main()
