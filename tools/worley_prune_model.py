"""CPU model of Worley-F1 cell pruning for the procedural march (config 2:
1080p x 128, reference camera, Worley frequency .03 on q = P * 128).

cellular() takes the minimum squared distance over the 27 cells around
rint(q).  Feature points sit at distance `jitter` (0.396) from their cell's
integer corner, so a cell whose corner is >= D from the sample cannot come
closer than D - jitter.  The model evaluates the 8 cells of the sample's
near octant first (per axis the centre cell and the one on the sample's
side), then asks, per wave of the sorted schedule and per step, whether ANY
lane could still find a closer point in each group of far cells -- the
wave-uniform branch a kernel would take.

    python tools/worley_prune_model.py [--every K] [--groups 2|7]
"""
import argparse

import numpy as np

from ta_model import rays

JIT = 0.39614353
KPX, KPY, KPZ = 501125321, 1136930381, 1720413743
W, H = 1920, 1080


def wrap(v):
    return ((v + 2**31) % 2**32) - 2**31


def feature(ix, iy, iz, seed=2):
    h = wrap((seed ^ wrap(ix * KPX) ^ wrap(iy * KPY) ^ wrap(iz * KPZ)) * 0x27d4eb2d)
    h = h & 0xffffffff
    xd = (h & 0x3ff) - 511.5
    yd = ((h >> 10) & 0x3ff) - 511.5
    zd = ((h >> 20) & 0x3ff) - 511.5
    inv = JIT / np.sqrt(xd * xd + yd * yd + zd * zd)
    return np.stack([ix + xd * inv, iy + yd * inv, iz + zd * inv], -1)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--every", type=int, default=8, help="model every K-th wave")
    ap.add_argument("--freq", type=float, default=0.03)
    ap.add_argument("--tight", action="store_true")
    args = ap.parse_args()
    n, p0, st = rays()
    # sorted schedule: n descending, 64x64 regions, row-major inside a region
    yy, xx = np.mgrid[0:H, 0:W]
    region = (yy // 64) * ((W + 63) // 64) + xx // 64
    inreg = (yy % 64) * 64 + xx % 64
    live = n.ravel() > 0
    order = np.lexsort((inreg.ravel()[live], region.ravel()[live], -n.ravel()[live]))
    pix = np.flatnonzero(live)[order]
    nw = len(pix) // 64
    waves = pix[:nw * 64].reshape(nw, 64)[::args.every]
    s = 128.0 * args.freq
    tot = {k: 0 for k in ("steps", "near_only", "single", "double", "triple", "any", "ax0", "ax1", "ax2", "cells")}
    offs = np.array([(a, b, c) for a in (-1, 0, 1) for b in (-1, 0, 1) for c in (-1, 0, 1)])
    for w in waves:
        nn = n.ravel()[w]
        P0 = p0.reshape(-1, 3)[w]
        ST = st.reshape(-1, 3)[w]
        for i in range(nn.max()):
            act = i < nn
            q = (P0 + ST * i)[act] * s
            r = np.rint(q)
            f = q - r
            sg = np.where(f >= 0, 1, -1)
            cells = r[:, None, :] + offs[None, :, :]                    # [L, 27, 3]
            fp = feature(cells[..., 0].astype(np.int64), cells[..., 1].astype(np.int64),
                         cells[..., 2].astype(np.int64))
            d2 = ((fp - q[:, None, :]) ** 2).sum(-1)                   # [L, 27]
            far = (offs[None, :, :] == -sg[:, None, :])                  # axes on the far side
            nfar = far.sum(-1)
            near_min = np.where(nfar == 0, d2, np.inf).min(1)
            e2 = (np.sqrt(near_min) + JIT) ** 2
            # corner distances of the far cells: the far axes at 1 + |f|, the others >= 0
            # (--tight: the near axes at |f| (offset 0) or 1 - |f| (offset toward the sample))
            if args.tight:
                ax = np.where(far, 1 + np.abs(f)[:, None, :],
                              np.where(offs[None] == 0, np.abs(f)[:, None, :], 1 - np.abs(f)[:, None, :]))
                cd2 = (ax ** 2).sum(-1)
            else:
                cd2 = np.where(far, (1 + np.abs(f))[:, None, :] ** 2, 0).sum(-1)
            need = (cd2 < e2[:, None]) & (nfar > 0)
            assert (d2.min(1) == np.where(need | (nfar == 0), d2, np.inf).min(1)).all()
            tot["steps"] += 1
            for a in range(3):
                tot[f"ax{a}"] += (need & (nfar == 1) & far[..., a]).any()
            tot["cells"] += need.any(0).sum()
            ns = (need & (nfar == 1)).any()
            nd = (need & (nfar == 2)).any()
            nt = (need & (nfar == 3)).any()
            tot["single"] += ns
            tot["double"] += nd
            tot["triple"] += nt
            tot["any"] += ns or nd or nt
            tot["near_only"] += not (ns or nd or nt)
    S = tot["steps"]
    print(f"{len(waves)} waves, {S} wave-steps")
    for k in ("near_only", "single", "double", "triple", "ax0", "ax1", "ax2"):
        print(f"  {k:10s} {tot[k] / S:.3f}")
    cells = 8 + 12 * tot["single"] / S + 6 * tot["double"] / S + tot["triple"] / S
    print(f"  mean cells evaluated per wave-step (groups 1/2/3-axis-far) {cells:.2f} of 27")
    print(f"  per-axis groups of 4: {8 + 4 * (tot['ax0'] + tot['ax1'] + tot['ax2']) / S:.2f}; "
          f"per cell: {8 + tot['cells'] / S:.2f}")


if __name__ == "__main__":
    main()
