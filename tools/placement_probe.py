"""Does buffer placement change the per-launch time?  One process allocates
--allocs independent copies of bench.py's input/output sets (all kept alive,
so each lands elsewhere in HBM) and times each round-robin (HIP events
around --launches back-to-back launches, --reps rounds, median), after a
warm-up.  Prints one JSON line per allocation with its buffers' virtual
addresses.  python tools/placement_probe.py --workload c2 --allocs 6"""
import argparse
import ctypes
import json
import os
import statistics
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "tools"))

import band_sweep  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--workload", default="c2")
    ap.add_argument("--allocs", type=int, default=6)
    ap.add_argument("--launches", type=int, default=20)
    ap.add_argument("--reps", type=int, default=5)
    args = ap.parse_args()
    allocs = [band_sweep.setup(args.workload) for _ in range(args.allocs)]
    capi, L, stream = allocs[0][0], allocs[0][1], allocs[0][2]
    mode, alg = allocs[0][4], allocs[0][5]
    hs = ctypes.c_void_p(stream.handle)
    e0, e1 = capi.Event(), capi.Event()

    def run(sets, k):
        for i in range(k):
            capi.check(L.mxd_resize_crop_batch(sets[i % 2][2], sets[i % 2][3], mode, 0, hs))

    t_end = time.time() + 1.0
    while time.time() < t_end:
        for a in allocs:
            run(a[3], 5)
        stream.synchronize()
    times = [[] for _ in allocs]
    for _ in range(args.reps):
        for j, a in enumerate(allocs):
            run(a[3], 3)
            stream.synchronize()
            e0.record(stream)
            run(a[3], args.launches)
            e1.record(stream)
            stream.synchronize()
            times[j].append(e0.elapsed_ms(e1) / args.launches)
    for j, a in enumerate(allocs):
        ms = statistics.median(times[j])
        srcs = [hex(s[0].ptr) for s in a[3]]
        dsts = [hex(s[1].ptr) for s in a[3]]
        print(json.dumps({"workload": args.workload, "alloc": j, "ms_per_launch": round(ms, 5),
                          "frac": round(alg / (ms * 1e-3) / 8e12, 4), "reps": [round(t, 5) for t in times[j]],
                          "src": srcs, "dst": dsts}), flush=True)


if __name__ == "__main__":
    main()
