"""CPU model of the shadow-ray compaction of config 3 (1080p x 128, 8 shadow
steps toward normalize(1, 1, 2)): per wave of the sorted schedule and per
primary step, the (lane, shadow step) pairs to deal (lanes with density > 0,
in-box shadow samples only) and the 64-lane rounds they take -- and the
rounds if two consecutive primary steps were dealt together.

    python tools/shadow_rounds_model.py [--every K]
"""
import argparse

import numpy as np

from fbm_exit_model import f1, perlin
from ta_model import rays
from worley_prune_model import H, W


def density(q):
    fbm = np.zeros(len(q))
    f, amp = 0.19, 1.0
    for _ in range(4):
        fbm = fbm + amp * perlin(3, q[:, 0] * f, q[:, 1] * f, q[:, 2] * f)
        f *= 2.0
        amp *= 0.5
    return np.maximum(fbm * (1.0 - f1(q * 0.03)), 0.0)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--every", type=int, default=128)
    a = ap.parse_args()
    n, p0, st = rays()
    yy, xx = np.mgrid[0:H, 0:W]
    region = (yy // 64) * ((W + 63) // 64) + xx // 64
    live = n.ravel() > 0
    order = np.lexsort(((yy * W + xx).ravel()[live], -n.ravel()[live]))   # shadow: row-major within n
    pix = np.flatnonzero(live)[order]
    nw = len(pix) // 64
    waves = pix[:nw * 64].reshape(nw, 64)[::a.every]
    L = np.array([1.0, 1.0, 2.0]) / np.sqrt(6.0) / 64.0
    pairs = rounds = rounds2 = events = 0
    for w in waves:
        nn = n.ravel()[w]
        P0, ST = p0.reshape(-1, 3)[w], st.reshape(-1, 3)[w]
        carry = None
        for i in range(nn.max()):
            act = i < nn
            P = (P0 + ST * i)[act]
            need = density(P * 128.0) > 0
            q = P[need][:, None, :] + L[None, None, :] * np.arange(1, 9)[None, :, None]
            cnt = ((q >= 0) & (q <= 1)).all(-1).sum(1)
            p = int(cnt.sum())
            if p == 0:
                continue
            events += 1
            pairs += p
            rounds += -(-p // 64)
            if carry is None:
                carry = p
            else:
                rounds2 += -(-(carry + p) // 64)
                carry = None
        if carry is not None:
            rounds2 += -(-carry // 64)
    print(f"{len(waves)} waves, {events} events, {pairs / max(events, 1):.1f} pairs per event")
    print(f"rounds per event {rounds / max(events, 1):.2f}, lane use {pairs / (64 * max(rounds, 1)):.3f}; "
          f"two steps per deal: lane use {pairs / (64 * max(rounds2, 1)):.3f}")


if __name__ == "__main__":
    main()
