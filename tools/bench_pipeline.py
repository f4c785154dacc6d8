"""End-to-end pipeline benchmark through the operator surface (SURVEY.md §8d
C1 / C4; VERDICT r1 missing 6): JPEG files on disk -> load_image (native
decoder) -> image_resize_smallest_side 256 -> image_center_crop 224 -> batch
-> f32 / 255 -> prefetch(workers, workers), timed like the reference's
harness (benchmarks/comparative/caltech101/mlx_data.py:23-72: whole-dataset
iteration at 1, 8 and 16 workers), beside the reference-algorithm CPU
restatement of the same chain on the same files and threads.

Variants per worker count:
  ref_form   the reference chain verbatim (batch, then
             key_transform(lambda x: x.astype("float32") / 255))
  fused      image_to_float before batch: the kernel writes the f32 batch
  device     fused + batch(..., device=0): the batch stays in HBM (DLPack)
  *_hostdec  the same with set_device_decode(False): the whole JPEG decode on
             the host (default with a device: the whole decode of sequential
             files in the batch launch -- Huffman, IDCT, upsampling, colour)
  *_hostent  the same with set_device_entropy(False): the Huffman decode on
             the host, the rest in the batch launch (round 3's split)
  cpu        Pillow (libjpeg-turbo) decode -> oracle C stbir restatement ->
             crop per batch on a pool of that many worker processes, numpy
             /255 of each batch in the consumer
Datasets (synthetic stand-ins, seeded smooth noise, Pillow q=90 JPEGs):
  c1  300x200 / 200x300 (Caltech-101-like), batch 32
  c4  500x375 / 375x500 / 500x333 (ImageNet-like), batch 128
  c4p the c4 files saved progressive
Each surface point iterates the file list as many times as it takes to run
>= --min-seconds (default 5 s) with >= --min-batches (16) batches per worker.
Prints one JSON line per (dataset, variant, workers)."""
import argparse
import ctypes
import json
import multiprocessing
import os
import sys
import tempfile
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "mlx-data_amd"), os.path.join(REPO, "oracle")]

DATASETS = {
    "c1": dict(sizes=[(300, 200), (300, 200), (200, 300)], batch=32),
    "c4": dict(sizes=[(500, 375), (375, 500), (500, 333)], batch=128),
    # c4's files saved progressive (libjpeg's default progression, optimised tables)
    "c4p": dict(sizes=[(500, 375), (375, 500), (500, 333)], batch=128, progressive=True),
}


def smooth(rng, h, w):
    gh, gw = h // 24 + 2, w // 24 + 2
    grid = rng.integers(0, 256, (gh, gw, 3)).astype(np.float32)
    yi = np.minimum(np.arange(h) * (gh - 1) // max(1, h - 1), gh - 2)
    xi = np.minimum(np.arange(w) * (gw - 1) // max(1, w - 1), gw - 2)
    f = grid[yi][:, xi] * 0.6 + grid[yi + 1][:, xi + 1] * 0.4 + rng.normal(0, 12, (h, w, 3))
    return np.clip(f, 0, 255).astype(np.uint8)


def make_files(root, name, n):
    from PIL import Image

    rng = np.random.default_rng({"c1": 11, "c4": 2, "c4p": 2}[name])
    sizes = DATASETS[name]["sizes"]
    files = []
    for i in range(n):
        w, h = sizes[int(rng.integers(0, len(sizes)))]
        d = os.path.join(root, name, f"class{i % 16}")
        os.makedirs(d, exist_ok=True)
        p = os.path.join(d, f"img{i}.jpg")
        Image.fromarray(smooth(rng, h, w)).save(p, quality=90, progressive=DATASETS[name].get("progressive", False))
        files.append(p)
    return files


def _pipe_stats(reset):
    from mlx_data_amd import _pipeline
    return _pipeline._pipe_stats(reset)


def run_surface(files, batch, workers, variant, repeat=1):
    from mlx_data_amd import data as dx

    hostdec = variant.endswith("_hostdec")
    hostent = variant.endswith("_hostent")
    variant = variant.rsplit("_", 1)[0] if hostdec or hostent else variant
    prev, prev_ent = dx.device_decode(), dx.device_entropy()
    dx.set_device_decode(not hostdec)
    dx.set_device_entropy(not hostent)
    try:
        return _run_surface(dx, files, batch, workers, variant, repeat)
    finally:
        dx.set_device_decode(prev)
        dx.set_device_entropy(prev_ent)


def _run_surface(dx, files, batch, workers, variant, repeat=1):
    samples = [dict(image=f.encode("ascii"), label=i) for i, f in enumerate(files)] * repeat
    d = (dx.buffer_from_vector(samples).shuffle().to_stream().load_image("image")
         .image_resize_smallest_side("image", 256).image_center_crop("image", 224, 224))
    if variant == "ref_form":
        d = d.batch(batch).key_transform("image", lambda x: x.astype("float32") / 255)
    elif variant == "fused":
        d = d.image_to_float("image").batch(batch)
    else:
        d = d.image_to_float("image").batch(batch, device=0)
    d = d.prefetch(workers, workers)
    n = 0
    t0 = time.perf_counter()
    for s in d:
        n += len(s["label"])
    return n, time.perf_counter() - t0


def _cpu_batch(args):
    """One batch of the reference chain on the CPU (a worker process):
    libjpeg-turbo decode (Pillow), the oracle's stbir restatement + crop."""
    files, = args
    from PIL import Image
    import oracle as O

    lib = O.lib()
    u8p = ctypes.POINTER(ctypes.c_uint8)
    crops = np.empty((len(files), 224, 224, 3), np.uint8)
    for k, f in enumerate(files):
        img = np.ascontiguousarray(np.asarray(Image.open(f).convert("RGB")))
        h, w = img.shape[:2]
        rc = lib.orc_resize_smallest_side_center_crop(img.ctypes.data_as(u8p), w, h, 3, 256, 224, 224,
                                                      crops[k].ctypes.data_as(u8p))
        assert rc == 0
    return crops


def run_cpu(files, batch, workers, min_seconds=0.0):
    """The reference's CPU path restated on `workers` processes (the reference
    runs it on a C++ thread pool; processes keep Python's GIL out of the
    measurement): decode + resize + crop per batch in a worker, the batch's
    astype(float32) / 255 in the consumer like the reference's key_transform."""
    from concurrent.futures import ProcessPoolExecutor

    order = np.random.default_rng(0).permutation(len(files))
    chunks = [[files[i] for i in order[b:b + batch]] for b in range(0, len(files), batch)]
    # fork: main() runs every CPU leg before this process touches the GPU
    with ProcessPoolExecutor(max_workers=workers, mp_context=multiprocessing.get_context("fork")) as ex:
        list(ex.map(_cpu_batch, [(c[:2],) for c in chunks[:workers]]))  # warm the workers
        t0 = time.perf_counter()
        n = 0
        while True:  # whole passes over the files until >= min_seconds
            for crops in ex.map(_cpu_batch, [(c,) for c in chunks]):
                x = crops.astype("float32") / 255
                n += len(x)
            dt = time.perf_counter() - t0
            if dt >= min_seconds:
                break
    return n, dt


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--datasets", default="c1,c4")
    ap.add_argument("--images", type=int, default=2048)
    ap.add_argument("--workers", default="1,8,16")
    ap.add_argument("--variants", default="ref_form,fused,device,cpu")
    ap.add_argument("--cpu-images", type=int, default=512, help="files the CPU restatement runs over")
    ap.add_argument("--min-seconds", type=float, default=5.0, help="least duration of a timed surface run")
    ap.add_argument("--min-batches", type=int, default=16, help="least batches per worker of a timed surface run")
    ap.add_argument("--stats", action="store_true", help="add mxd_host_stats of the timed run to GPU legs' lines")
    ap.add_argument("--tune", default="", help="tuning knobs for the GPU legs, e.g. HUFF_GLOBAL=1,HUFF_BITS=1024 "
                    "(capi.set_tuning; MXD_TUNE_<name>)")
    args = ap.parse_args()
    tune = {}
    for kv in filter(None, args.tune.split(",")):
        k, v = kv.split("=")
        tune[k] = int(v)
    workers = [int(w) for w in args.workers.split(",")]
    variants = args.variants.split(",")
    # CPU legs first: their worker processes fork before any GPU call here
    order = [v for v in variants if v == "cpu"] + [v for v in variants if v != "cpu"]
    with tempfile.TemporaryDirectory() as root:
        files = {name: make_files(root, name, args.images) for name in args.datasets.split(",")}
        for v in order:
            for name, fl in files.items():
                B = DATASETS[name]["batch"]
                for w in workers:
                    if v == "cpu":
                        n, dt = run_cpu(fl[:args.cpu_images], B, w, args.min_seconds)
                    else:
                        if tune:
                            from mlx_data_amd import capi
                            for k, val in tune.items():
                                capi.set_tuning(getattr(capi, "MXD_TUNE_" + k), val)
                        # warm-up with every worker busy twice over: tap tables, host-path
                        # contexts and the recycled batch buffers reach their steady state;
                        # its rate sizes the timed run: the file list repeated until the run
                        # lasts >= --min-seconds and gives every worker >= --min-batches
                        nw, tw = run_surface(fl[:min(len(fl), 2 * B * w)], B, w, v)
                        want = max(args.min_seconds * nw / tw, args.min_batches * B * w)
                        repeat = max(1, int(np.ceil(want / len(fl))))
                        if args.stats:
                            from mlx_data_amd import capi
                            capi.host_stats(reset=True)
                            _pipe_stats(True)
                        n, dt = run_surface(fl, B, w, v, repeat)
                        # the warm-up's rate underestimates the steady one: rerun
                        # longer until the timed run itself lasts >= --min-seconds
                        for _ in range(3):
                            if dt >= args.min_seconds:
                                break
                            repeat = max(repeat + 1, int(np.ceil(repeat * 1.25 * args.min_seconds / dt)))
                            if args.stats:
                                capi.host_stats(reset=True)
                                _pipe_stats(True)
                            n, dt = run_surface(fl, B, w, v, repeat)
                    rec = dict(dataset=name, variant=v, workers=w, images=n, seconds=round(dt, 3),
                               images_per_s=round(n / dt, 1), batch=B)
                    if tune and v != "cpu":
                        rec["tune"] = tune
                    if args.stats and v != "cpu":
                        hs = capi.host_stats(reset=True)
                        # per image, microseconds (summed over worker threads)
                        rec["host_us_per_image"] = {k: round(hs[k] / max(1, n) * 1e6, 2)
                                                    for k in ("call_s", "wait_s", "parse_s")}
                        rec["host_calls"] = hs["calls"]
                        ps = _pipe_stats(True)
                        rec["pipe_us_per_image"] = {k: round(ps[i] / max(1, n) / 1e3, 2) for i, k in enumerate(
                            ("load_image", "transforms", "batch_fetch", "batch_merge", "from_buffer"))}
                    print(json.dumps(rec), flush=True)


if __name__ == "__main__":
    main()
