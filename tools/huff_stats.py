"""Synchronisation statistics and phase durations of the device entropy decode (diagnostic; needs
the -DMXD_HUFF_STATS=1 variant library in place of libmxd_amd.so,
tools/variants.sh build hstats "-DMXD_HUFF_STATS=1" jpeghuff): per job the
rounds until no subsequence's start state changed, the subsequences, and the
symbols decoded in the rounds and in the write pass, for C4- and C1-shaped
files at the default and at forced subsequence lengths."""
import ctypes
import json
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "mlx-data_amd"), os.path.join(REPO, "tools")]

import jpeg_batch_bench as J  # noqa: E402
from mlx_data_amd import capi  # noqa: E402


def main():
    L = capi.lib()
    capi.check(L.mxd_set_device(0))
    for name in ("c4", "c1"):
        datas = J.files(name, 64)
        for bits in (0, 1024, 2048, 4096):
            capi.set_tuning(capi.MXD_TUNE_HUFF_BITS, bits)
            coefs = [capi.JpegCoefs(d, True) for d in datas]
            dst = capi.DeviceBuffer(len(datas) * 224 * 224 * 3, 0)
            entries = []
            for i, c in enumerate(coefs):
                rw, rh = capi.resize_smallest_side_dims(c.width, c.height, 256)
                cx, cy = capi.center_crop_origin(rw, rh, 224, 224)
                entries.append(dict(coefs=c, win_x=0, win_y=0, win_w=c.width, win_h=c.height, resize_w=rw,
                                    resize_h=rh, crop_x=cx, crop_y=cy, crop_w=224, crop_h=224, flip=0,
                                    dst=dst.ptr + i * 224 * 224 * 3, dst_stride=224 * 3))
            arr, n = capi.make_jpeg_images(entries)
            capi.jpeg_resize_crop_to_device(arr, n, capi.MXD_U8, 0)
            st = np.zeros((len(datas), 16), np.int32)
            assert L.mxd_debug_huff_stats(st.ctypes.data_as(ctypes.c_void_p), len(datas)) == 0
            print(json.dumps(dict(dataset=name, min_bits=bits, rounds_mean=round(float(st[:, 0].mean()), 2),
                                  rounds_max=int(st[:, 0].max()), subsequences_mean=round(float(st[:, 1].mean()), 1),
                                  sync_symbols_per_write_symbol=round(float(st[:, 2].sum() / st[:, 3].sum()), 3),
                                  # phase durations, us (mean / max over jobs): staging, sync rounds, write, DC
                                  us_stage=[round(float(st[:, 7].mean()) / 100, 1), round(float(st[:, 7].max()) / 100, 1)],
                                  us_sync=[round(float(st[:, 4].mean()) / 100, 1), round(float(st[:, 4].max()) / 100, 1)],
                                  us_write=[round(float(st[:, 5].mean()) / 100, 1), round(float(st[:, 5].max()) / 100, 1)],
                                  us_dc=[round(float(st[:, 6].mean()) / 100, 1), round(float(st[:, 6].max()) / 100, 1)],
                                  syms_per_sub_round=round(float(st[:, 2].sum() / max(1, (st[:, 1] * st[:, 0]).sum())), 1),
                                  # write pass: shader cycles per step of the busiest thread, and the
                                  # shader clock (cycles / real-time ticks of 10 ns)
                                  write_cycles_per_step=round(float((st[:, 8] / np.maximum(st[:, 9], 1)).mean()), 1),
                                  write_max_syms=round(float(st[:, 9].mean()), 1),
                                  write_t0_syms=round(float(st[:, 10].mean()), 1),
                                  clock_ghz=round(float((st[:, 8] / np.maximum(st[:, 11], 1)).mean()) / 10, 3),
                                  # start-state changes after round 0, and the shares that kept the
                                  # bit position (phase only) and the position and coefficient index
                                  changes=int(st[:, 12].sum()),
                                  share_same_pos=round(float(st[:, 13].sum() / max(1, st[:, 12].sum())), 3),
                                  share_same_pos_k=round(float(st[:, 14].sum() / max(1, st[:, 12].sum())), 3))),
                  flush=True)
            dst.free()
    capi.set_tuning(capi.MXD_TUNE_HUFF_BITS, 0)


if __name__ == "__main__":
    main()
