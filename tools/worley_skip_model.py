"""CPU model: how often could a wave of config 2's sorted schedule skip the
Worley evaluation because every live lane's fBm is <= 0 (density is then
max(fbm * (1 - F1), 0) = 0 whenever 1 - F1 >= 0)?  Reuses the fbm/F1
restatements of tools/fbm_exit_model.py.

    python tools/worley_skip_model.py [--every K]
"""
import argparse

import numpy as np

from fbm_exit_model import perlin, f1
from ta_model import rays
from worley_prune_model import W, H


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--every", type=int, default=64)
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
    steps = lanes_neg = wave_neg = wave_skip = 0
    for w in waves:
        nn = n.ravel()[w]
        P0, ST = p0.reshape(-1, 3)[w], st.reshape(-1, 3)[w]
        for i in range(nn.max()):
            act = i < nn
            q = (P0 + ST * i)[act] * 128.0
            fbm = np.zeros(len(q))
            f = 0.19
            for o in range(4):
                fbm = fbm + amps[o] * perlin(3, q[:, 0] * f, q[:, 1] * f, q[:, 2] * f)
                f *= 2.0
            omf = 1.0 - f1(q * 0.03)
            neg = fbm <= 0
            steps += 1
            lanes_neg += neg.mean()
            wave_neg += neg.all()
            wave_skip += (neg & (omf >= 0)).all()
    print(f"{len(waves)} waves, {steps} wave-steps")
    print(f"lanes with fbm <= 0: {lanes_neg / steps:.3f}; waves with all lanes fbm <= 0: {wave_neg / steps:.3f}"
          f" (and 1 - F1 >= 0: {wave_skip / steps:.3f})")


if __name__ == "__main__":
    main()
