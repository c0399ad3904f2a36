"""CPU model of an exact fBm early-out for the procedural march (config 2).

density = max(fbm * (1 - F1), 0) * scale.  After octave o the remaining
octaves add at most B * sum_{k>o} amp_k in magnitude (|Perlin| <= B:
0.9649 x a convex combination of corner dots, each |dot| <= 2, so B = 1.93).
Once fbm_o + that bound < 0 with 1 - F1 > 0 (or > 0 with 1 - F1 < 0) the
density is exactly 0 and the remaining octaves can be skipped.  A wave of the
sorted schedule saves an octave only when all its lanes can.

    python tools/fbm_exit_model.py [--every K] [--bound B]
"""
import argparse

import numpy as np

from ta_model import rays
from worley_prune_model import W, H, feature, wrap, KPX, KPY, KPZ

M = 0x27d4eb2d


def grad_dot(h, fx, fy, fz):
    h13 = h & 13
    u = np.where(h13 < 8, fx, fy)
    v = np.where(h13 < 2, fy, np.where(h13 == 12, fx, fz))
    u = np.where(h & 1, -u, u)
    v = np.where(h & 2, -v, v)
    return u + v


def perlin(seed, x, y, z):
    xs, ys, zs = np.floor(x), np.floor(y), np.floor(z)
    x0, y0, z0 = wrap(xs.astype(np.int64) * KPX), wrap(ys.astype(np.int64) * KPY), wrap(zs.astype(np.int64) * KPZ)
    x1, y1, z1 = wrap(x0 + KPX), wrap(y0 + KPY), wrap(z0 + KPZ)
    fx0, fy0, fz0 = x - xs, y - ys, z - zs
    fx1, fy1, fz1 = fx0 - 1, fy0 - 1, fz0 - 1
    q = lambda t: t * t * t * (t * (t * 6 - 15) + 10)
    u, v, w = q(fx0), q(fy0), q(fz0)

    def hs(a, b, c):
        h = wrap((seed ^ a ^ b ^ c) * M) & 0xffffffff
        return ((h >> 15) ^ h) & 0xffffffff

    lerp = lambda a, b, t: a + t * (b - a)
    l00 = lerp(grad_dot(hs(x0, y0, z0), fx0, fy0, fz0), grad_dot(hs(x1, y0, z0), fx1, fy0, fz0), u)
    l10 = lerp(grad_dot(hs(x0, y1, z0), fx0, fy1, fz0), grad_dot(hs(x1, y1, z0), fx1, fy1, fz0), u)
    l01 = lerp(grad_dot(hs(x0, y0, z1), fx0, fy0, fz1), grad_dot(hs(x1, y0, z1), fx1, fy0, fz1), u)
    l11 = lerp(grad_dot(hs(x0, y1, z1), fx0, fy1, fz1), grad_dot(hs(x1, y1, z1), fx1, fy1, fz1), u)
    return 0.964921414852142333984375 * lerp(lerp(l00, l10, v), lerp(l01, l11, v), w)


def f1(q):
    r = np.rint(q)
    offs = np.array([(a, b, c) for a in (-1, 0, 1) for b in (-1, 0, 1) for c in (-1, 0, 1)])
    cells = r[:, None, :] + offs[None]
    fp = feature(cells[..., 0].astype(np.int64), cells[..., 1].astype(np.int64), cells[..., 2].astype(np.int64))
    return ((fp - q[:, None, :]) ** 2).sum(-1).min(1)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--every", type=int, default=64)
    ap.add_argument("--bound", type=float, default=1.93)
    args = ap.parse_args()
    n, p0, st = rays()
    yy, xx = np.mgrid[0:H, 0:W]
    region = (yy // 64) * ((W + 63) // 64) + xx // 64
    inreg = (yy % 64) * 64 + xx % 64
    live = n.ravel() > 0
    order = np.lexsort((inreg.ravel()[live], region.ravel()[live], -n.ravel()[live]))
    pix = np.flatnonzero(live)[order]
    nw = len(pix) // 64
    waves = pix[:nw * 64].reshape(nw, 64)[::args.every]
    amps = [1.0, 0.5, 0.25, 0.125]
    rem = [args.bound * sum(amps[k + 1:]) for k in range(4)]
    lane_oct = wave_oct = steps = zero = 0
    for w in waves:
        nn = n.ravel()[w]
        P0, ST = p0.reshape(-1, 3)[w], st.reshape(-1, 3)[w]
        for i in range(nn.max()):
            act = i < nn
            q = (P0 + ST * i)[act] * 128.0
            omf = 1.0 - f1(q * 0.03)
            fbm = np.zeros(len(q))
            done = np.zeros(len(q), bool)
            need = np.zeros(4)
            f = 0.19
            for o in range(4):
                need[o] = (~done).sum()
                fbm = fbm + amps[o] * perlin(3, q[:, 0] * f, q[:, 1] * f, q[:, 2] * f) * (~done)
                f *= 2.0
                done |= ((omf > 0) & (fbm < -rem[o])) | ((omf < 0) & (fbm > rem[o])) | (omf == 0)
            steps += 1
            lane_oct += need.sum() / len(q)
            wave_oct += (need > 0).sum()
            zero += (np.maximum(fbm * omf, 0) == 0).mean()
    print(f"{len(waves)} waves, {steps} wave-steps; zero-density share {zero / steps:.3f}")
    print(f"octaves per lane {lane_oct / steps:.3f} of 4, per wave {wave_oct / steps:.3f} of 4")


if __name__ == "__main__":
    main()
