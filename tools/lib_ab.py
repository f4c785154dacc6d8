"""In-process A/B of library builds: the product libmxd_amd.so and compile-time
variants (tools/variants.sh build NAME FLAGS) loaded side by side in ONE
process, timed round-robin on the same resident inputs, so box-to-box and
process-to-process spread cannot decide the comparison.

  python tools/lib_ab.py --workloads c2,c3,c4,c5 --variants product,ntl,sc1 \
      [--launches 20] [--reps 5]

Each variant is a separate shared object (its own code objects registered with
the HIP runtime); inputs, outputs, streams and events come from the product
library and are used by every variant (one HIP runtime, one device).  For
every workload: two resident source/output sets (bench.py's synthetic inputs),
then per rep and per variant 3 untimed launches and `launches` timed ones
(HIP events on one stream).  Prints one JSON line per (workload, variant):
median ms per launch, frac of 8 TB/s from B_alg, every rep; and checks that
each variant's output equals the product's byte for byte.
"""
import argparse
import ctypes
import json
import os
import statistics
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "mlx-data_amd"))
sys.path.insert(0, os.path.join(REPO, "tools"))

import numpy as np  # noqa: E402

import band_sweep  # noqa: E402


# "NAME@knob=v,knob=v": a library with tuning knobs set around its runs
KNOBS = {"load": 12, "policy": -1}  # -1: mxd_set_kernel_policy


def parse_variant(spec):
    name, _, knobs = spec.partition("@")
    kv = {}
    for item in filter(None, knobs.split(",")):
        k, _, v = item.partition("=")
        kv[KNOBS[k]] = int(v)
    return name, kv


def load_variant(name, capi):
    name = parse_variant(name)[0]
    if name == "product":
        return capi.lib()
    path = os.path.join(REPO, "tools", f"libmxd_amd_var_{name}.so")
    L = ctypes.CDLL(path, mode=os.RTLD_LOCAL | os.RTLD_NOW)
    L.mxd_last_error.restype = ctypes.c_char_p
    rc = L.mxd_set_device(0)
    if rc != 0:
        raise RuntimeError(f"{name}: mxd_set_device -> {rc}")
    return L


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--workloads", default="c2,c3,c4,c5")
    ap.add_argument("--variants", default="product")
    ap.add_argument("--launches", type=int, default=20)
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--policy", type=int, default=0, help="mxd_set_kernel_policy for every variant (256: prefer band)")
    args = ap.parse_args()
    names = args.variants.split(",")
    for wl in args.workloads.split(","):
        # "c3:640x480" = C3's batch drawn from that one size
        name, _, only = wl.partition(":")
        c3 = [tuple(int(v) for v in only.split("x"))] if only else None
        capi, PL, stream, sets, mode, alg, sizes, geoms, f32 = band_sweep.setup(name, c3_sizes=c3)
        libs = {n: load_variant(n, capi) for n in names}
        for L in libs.values():
            L.mxd_set_kernel_policy(args.policy)
        hs = ctypes.c_void_p(stream.handle)
        e0, e1 = capi.Event(), capi.Event()

        knobs = {n: parse_variant(n)[1] for n in names}
        cur = {"n": None}

        def run(L, i, n=None):
            if n is not None and cur["n"] != n:
                # the previous variant's knobs back to 0, this one's set
                if cur["n"] is not None:
                    for k in knobs[cur["n"]]:
                        if k < 0:
                            libs[cur["n"]].mxd_set_kernel_policy(args.policy)
                        else:
                            libs[cur["n"]].mxd_set_tuning(k, 0)
                for k, v in knobs[n].items():
                    if k < 0:
                        L.mxd_set_kernel_policy(v)
                    else:
                        L.mxd_set_tuning(k, v)
                cur["n"] = n
            rc = L.mxd_resize_crop_batch(sets[i % 2][2], sets[i % 2][3], mode, 0, hs)
            if rc != 0:
                raise RuntimeError(L.mxd_last_error().decode())

        # equality with the product's output, then warm-up of every variant
        out_bytes = sets[0][1].nbytes
        ref = None
        same = {}
        for n, L in libs.items():
            sets[0][1].memset(0, stream=stream)
            run(L, 0, n)
            stream.synchronize()
            got = sets[0][1].download((out_bytes,), np.uint8, stream=stream)
            if ref is None:
                ref = got
            same[n] = bool(np.array_equal(got, ref))
            for i in range(20):
                run(L, i, n)
        stream.synchronize()
        times = {n: [] for n in names}
        for _ in range(args.reps):
            for n, L in libs.items():
                for i in range(3):
                    run(L, i, n)
                stream.synchronize()
                e0.record(stream)
                for i in range(args.launches):
                    run(L, i, n)
                e1.record(stream)
                stream.synchronize()
                times[n].append(e0.elapsed_ms(e1) / args.launches)
        for n in names:
            ms = statistics.median(times[n])
            print(json.dumps({"workload": wl, "variant": n, "ms_per_launch": round(ms, 5),
                              "frac": round(alg / (ms * 1e-3) / 8e12, 4), "equal_to_first": same[n],
                              "reps": [round(t, 5) for t in times[n]]}), flush=True)
        for s in sets:
            s[0].free()
            s[1].free()


if __name__ == "__main__":
    main()
