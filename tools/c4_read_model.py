"""Line-level model of the source bytes C4's wave kernel reads (DESIGN §5,
VERDICT r3 next 4): bench.py's C4 workload (128 ImageNet shapes, seed 2, rows
at 16-byte-rounded pitches, images 256-byte aligned), the narrow kernel's two
strips per crop row (112 output columns each, each lane a 12-byte dwordx3 of
4 pixels from the 4-pixel-aligned window start), bands of `ty` output rows
reading their tap rows; counts the distinct 64- and 128-byte lines each band
touches per row and sums them over bands (no L2 reuse between bands), against
the byte footprint of bench.footprint_bytes.

    python tools/c4_read_model.py
"""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "mlx-data_amd")]

import bench  # noqa: E402
from mlx_data_amd import capi  # noqa: E402


def main():
    sizes, geoms, _ = bench.make_workload(capi, "c4", 128, 0)
    foot = sum(bench.footprint_bytes(capi, sw, sh, 3, *g[:6]) for (sw, sh), g in zip(sizes, geoms))
    print(f"byte footprint {foot / 1e6:.1f} MB")
    for ty in (10, 16, 23, 32, 224):
        for line in (64, 128):
            tot, off = 0, 0
            for (sw, sh), g in zip(sizes, geoms):
                rw, rh, cx, cy, cw, ch, _ = g
                pitch = (sw * 3 + 15) // 16 * 16
                fx, nx, _ = capi.axis_taps(sw, rw, cx, cw)
                fy, ny, _ = capi.axis_taps(sh, rh, cy, ch)
                spans = []
                for ox0 in (0, cw // 2):
                    ox1 = ox0 + cw // 2 - 1
                    lo, hi = fx[ox0], fx[ox1] + nx[ox1] - 1
                    wp0 = lo & ~3
                    spans.append((wp0 * 3, wp0 * 3 + 12 * ((hi + 1 - wp0 + 3) // 4)))
                for y0 in range(0, ch, ty):
                    y1 = min(ch, y0 + ty)
                    r0, r1 = fy[y0], (fy[y0:y1] + ny[y0:y1] - 1).max()
                    for r in range(r0, r1 + 1):
                        lines = set()
                        for b0, b1 in spans:
                            a, e = off + r * pitch + b0, off + r * pitch + b1
                            lines.update(range(a // line, (e - 1) // line + 1))
                        tot += len(lines) * line
                off += (pitch * sh + 255) // 256 * 256
            print(f"band rows {ty:3d}  {line:3d}-byte lines: {tot / 1e6:.1f} MB = {tot / foot:.3f} x footprint")


if __name__ == "__main__":
    main()
