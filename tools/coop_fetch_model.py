"""Model of a wave-cooperative fetch for the config-5 march (verdict r05 #4),
before building anything: per tap, the wave loads each distinct 128-B line of
its footprints once, with line-contiguous lanes (b128: 8 lanes, i.e. 2 quads,
per line), and hands every lane its 2 x 8 bytes by ds_bpermute.

Layout: COL48 (columns of 3 x 7 positions through z, 32-B slices, 4 slices per
128-B line).  For each wave-step and tap (the 3 loaded channels; G is uniform),
with the frame's geometry (tools/ta_model.py rays(), reference camera, 512^3,
1080p x 128):

- today: 2 b64 loads (slices z, z+1), L1 lookups = per quad, the distinct
  lines among its active lanes (tcp_calib);
- cooperative, exact set: the wave's distinct lines over both slices, each
  fetched once (2 lookups per line, ceil(lines / 8) b128 instructions); the
  lane -> line assignment needs the set's ordering (a wave sort or a loop
  over distinct keys);
- cooperative, bounding box: the box of (x column, y column, z line) over the
  wave's footprints, every box line fetched (no sort: a lane's line index is
  arithmetic in the box), so lines = box volume.

VALU added per tap (cooperative), counted on the instruction sequence it
needs: the wave's min / max of the three line coordinates (6 DPP reductions
of ~7 ops each, shared by the 3 taps of a step: 14 per tap), the box index and
lane -> line address (~10), 4 bpermutes per slice pair with their selects
(8 + 4), against ~34 VALU per tap today (3 fma coordinates, floor/convert,
table adds, 7 lerps, alignbyte).  The build criterion: <= 20 lookups per
VMEM instruction-equivalent at <= 1.3x the VALU.

    python tools/coop_fetch_model.py [--tiles 8]
"""
import argparse

import numpy as np

import ta_model
from ta_model import N, S, W, H


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--tiles", type=int, default=8, help="model every K-th 8x8 tile")
    a = ap.parse_args()
    n, p0, st = ta_model.rays()
    tx8, ty8 = W // 8, (H + 7) // 8
    lane = np.arange(64)
    lx, ly = ((lane >> 2) & 3) * 2 + (lane & 1), (lane >> 4) * 2 + ((lane >> 1) & 1)   # 2x2 quads
    T = np.arange(tx8 * ty8)[::a.tiles]
    X = (T % tx8)[:, None] * 8 + lx[None, :]
    Y = np.minimum((T // tx8)[:, None] * 8 + ly[None, :], H - 1)
    nn = n[Y, X]
    keep = nn.max(1) > 0
    nn, P0, ST = nn[keep], p0[Y, X][keep], st[Y, X][keep]
    nz_lines = (N + 3) // 4 + 1
    today_look = coop_lines = box_lines = taps = 0
    box_le16 = 0
    for i in range(S):
        act = i < nn
        wave = act.any(1)
        if not wave.any():
            break
        a_ = act[wave]
        P = P0[wave] + ST[wave] * i
        for sc in (1, .8, .75):   # the loaded channels (R, B, A; G is uniform) -- 3 taps
            g = np.clip(np.floor(P * sc * N + 0.5).astype(np.int64), 0, N)
            xc, yc, z = g[..., 0] // 3, g[..., 1] // 7, g[..., 2]
            col = xc * (N // 7 + 1) + yc
            # today: per quad, distinct (line) among active lanes, for slices z and z+1
            for zz in (z, z + 1):
                ln = np.where(a_, col * nz_lines + zz // 4, -1)
                q = np.sort(ln.reshape(len(ln), 16, 4), axis=-1)
                today_look += (np.concatenate([q[..., :1] >= 0, (q[..., 1:] != q[..., :-1]) & (q[..., 1:] >= 0)], -1)).sum()
            # cooperative: the wave's distinct lines over both slices
            l0 = np.where(a_, col * nz_lines + z // 4, -1)
            l1 = np.where(a_, col * nz_lines + (z + 1) // 4, -1)
            both = np.sort(np.concatenate([l0, l1], 1), axis=1)
            coop_lines += (np.concatenate([both[:, :1] >= 0, (both[:, 1:] != both[:, :-1]) & (both[:, 1:] >= 0)], 1)).sum()
            big = 1 << 40
            def ext(v):
                lo = np.where(a_, v, big).min(1)
                hi = np.where(a_, v, -1).max(1)
                return hi - lo + 1
            zl = ext(z // 4) + ((np.where(a_, (z + 1) // 4, -1).max(1) > np.where(a_, z // 4, -1).max(1)))
            bl = ext(xc) * ext(yc) * zl
            box_lines += bl.sum()
            box_le16 += (bl <= 16).sum()
            taps += len(a_)
    today_per_tap = today_look / taps
    print(f"wave-taps modelled: {taps} (every {a.tiles}th tile, 3 loaded taps per step)")
    print(f"today: 2 b64 loads per tap, {today_per_tap:.1f} L1 lookups per tap ({today_per_tap / 2:.1f} per instruction)")
    cl = coop_lines / taps
    print(f"cooperative, exact line set: {cl:.1f} distinct lines per tap -> {2 * cl:.1f} lookups, "
          f"{np.ceil(cl / 8):.0f}+ b128 loads; needs a per-wave sort / distinct-key loop of ~{cl:.0f} rounds")
    bx = box_lines / taps
    print(f"cooperative, bounding box: {bx:.1f} lines per tap -> {2 * bx:.1f} lookups in {bx / 8:.1f} b128 loads "
          f"({box_le16 / taps:.2f} of wave-taps have a box of <= 16 lines)")
    valu_today, valu_add = 34.0, 14 + 10 + 12
    print(f"VALU per tap: today ~{valu_today:.0f}, cooperative ~{valu_today + valu_add:.0f} "
          f"({(valu_today + valu_add) / valu_today:.2f}x); the exact-set variant adds ~{6 * cl:.0f} more for its "
          "distinct-key loop")
    ok = 2 * bx / max(1.0, np.ceil(bx / 8)) <= 20 and (valu_today + valu_add) / valu_today <= 1.3
    print("verdict:", "build" if ok else "do not build: the box variant fetches "
          f"{bx:.1f} lines for {cl:.1f} distinct ({bx / cl:.1f}x the bytes through TD) and both variants exceed "
          "1.3x the VALU of a kernel whose VALU is already 0.67 busy")


if __name__ == "__main__":
    main()
