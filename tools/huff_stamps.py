"""Summarises the entropy decode's phase stamps (diagnostic build
-DMXD_HUFF_STAMPS, tools/r05_stamps.sh): per launch size, the median and
max over jobs of each phase's shader cycles, the synchronisation rounds and
the lanes of rounds 2..4, and the spread of the jobs' start times.
  python tools/huff_stamps.py FILE [skip]"""
import json
import struct
import sys
from collections import defaultdict

import numpy as np


def read(path):
    out = []
    with open(path, "rb") as f:
        b = f.read()
    i = 0
    while i < len(b):
        (n,) = struct.unpack_from("<q", b, i)
        i += 8
        w = np.frombuffer(b, np.uint64, 3 * n, i).reshape(n, 3)
        i += 24 * n
        jobs = np.frombuffer(b, np.int32, 10 * n, i).reshape(n, 10)
        i += 40 * n
        out.append((w, jobs))
    return out


def main():
    recs = read(sys.argv[1])
    skip = int(sys.argv[2]) if len(sys.argv) > 2 else 3
    by = defaultdict(list)
    for w, jobs in recs[skip:]:
        by[len(w)].append((w, jobs))
    for n, runs in sorted(by.items()):
        ph = defaultdict(list)
        spread, rnd, nact = [], [], []
        for w, jobs in runs:
            m = (1 << 21) - 1
            w5, w6, w7 = w[:, 0], w[:, 1], w[:, 2]
            cols = dict(load=w5 & m, rounds=(w5 >> 21) & m, pred=(w5 >> 42) & m, write=w6 & m, tail=(w6 >> 21) & m)
            for k, v in cols.items():
                ph[k].append(v.astype(np.int64) * 16)
            ph["total"].append(sum(v.astype(np.int64) for v in cols.values()) * 16)
            rnd.append(((w6 >> 42) & 63).astype(np.int64))
            ph["rounds_fix"].append(((w6 >> 48) & 63).astype(np.int64))
            nact.append(np.stack([(w7 >> s) & 2047 for s in (0, 11, 22)], 1).astype(np.int64))
            rt = ((w7 >> 33) & 0x3ffffff).astype(np.int64)
            spread.append(int(rt.max() - rt.min()) * 10)  # ns (100 MHz)
        line = dict(jobs=n, launches=len(runs))
        for k, v in ph.items():
            a = np.concatenate(v)
            line[k] = dict(med=int(np.median(a)), p90=int(np.percentile(a, 90)), max=int(a.max()))
        r = np.concatenate(rnd)
        line["rounds_hist"] = {int(k): int(c) for k, c in zip(*np.unique(r, return_counts=True))}
        line["nact_med"] = [int(x) for x in np.median(np.concatenate(nact), 0)]
        line["nsub_med"] = int(np.median(np.concatenate([j[:, 5] for _, j in runs])))
        line["start_spread_ns_med"] = int(np.median(spread))
        print(json.dumps(line))


if __name__ == "__main__":
    main()
