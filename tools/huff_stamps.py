"""Summarises the entropy decode's phase stamps (diagnostic build
-DMXD_HUFF_STAMPS, tools/r05_stamps.sh): per launch size, over jobs, the
median / p90 / max shader cycles of each phase (load, rounds, predecessor,
thread 0's write pass, the rest), the median cycles and lanes of each
synchronisation round, the rounds histogram and the spread of the jobs'
start times.
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
        n, nw = struct.unpack_from("<qq", b, i)
        i += 16
        w = np.frombuffer(b, np.uint64, nw * n, i).reshape(n, nw).astype(np.int64)
        i += 8 * nw * n
        jobs = np.frombuffer(b, np.int32, 10 * n, i).reshape(n, 10)
        i += 40 * n
        out.append((w, jobs))
    return out


def stat(a):
    a = np.asarray(a)
    return dict(med=int(np.median(a)), p90=int(np.percentile(a, 90)), max=int(a.max()))


def main():
    recs = read(sys.argv[1])
    skip = int(sys.argv[2]) if len(sys.argv) > 2 else 3
    by = defaultdict(list)
    for w, jobs in recs[skip:]:
        by[len(w)].append((w, jobs))
    for n, runs in sorted(by.items()):
        W = np.concatenate([w for w, _ in runs])
        st = W[:, 0:6]
        names = ["load", "rounds", "pred", "write0", "rest"]
        line = dict(jobs=n, launches=len(runs))
        for i, k in enumerate(names):
            line[k] = stat(st[:, i + 1] - st[:, i])
        line["total"] = stat(st[:, 5] - st[:, 0])
        rounds = W[:, 7] & 255
        line["rounds_hist"] = {int(k): int(c) for k, c in zip(*np.unique(rounds, return_counts=True))}
        R = W[:, 8:24]
        t_end = R & ((1 << 40) - 1)
        lanes = R >> 40
        per = []
        for r in range(1, 12):
            ok = rounds > r
            if ok.sum() < len(W) // 2:
                break
            prev = np.where(r == 1, st[:, 1], 0) if False else t_end[:, r - 1]
            d = (t_end[:, r] - t_end[:, r - 1])[ok]
            per.append(dict(round=r, lanes=int(np.median(lanes[ok, r - 1])), cycles=int(np.median(d))))
        line["per_round"] = per
        pred = np.concatenate([j[:, 9] for _, j in runs]) != 0
        dcw = W[:, 7] >> 32
        for name, sel in (("pred_jobs", pred), ("first_jobs", ~pred)):
            if sel.any():
                line[name] = dict(n=int(sel.sum()), total=stat((st[:, 5] - st[:, 0])[sel]),
                                  rounds=stat((st[:, 2] - st[:, 1])[sel]), after_rounds=stat((st[:, 5] - st[:, 3])[sel]),
                                  dc_wait=stat(dcw[sel]))
        line["first_scan"] = int(np.median(t_end[:, 0] - st[:, 1]))
        rt = W[:, 6]
        line["start_spread_ns_med"] = int(np.median([(w[:, 6].max() - w[:, 6].min()) * 10 for w, _ in runs]))
        line["nsub_med"] = int(np.median(np.concatenate([j[:, 5] for _, j in runs])))
        print(json.dumps(line))


if __name__ == "__main__":
    main()
