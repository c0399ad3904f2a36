"""CPU model of the LDS-slab fill for the grid march at config 5 (512^3,
1080p x 128, reference camera; geometry from tools/ta_model.py, which
reproduces the measured L1 lookups of the shipped kernel to 3 %).

Per wave (8x8 tile) and step, per channel: the bounding box of the padded
base positions (a, b, c) = floor(P * s_t * N + 0.5) of the live rays, mapped
to 64-B chunks of a brick layout (one chunk = the bytes a quad of lanes
fetches with one 16-B LDS-DMA load each, one L1 lookup).  Reports chunks per
channel-step (= L1 lookups of the fill), the fill instructions (64 lanes x
16 B each), and how often a per-channel capacity is exceeded.

    python tools/slab_fill_model.py [--tiles K] [--chunk brick4832|b4416|b4432]
"""
import argparse

import numpy as np

from ta_model import rays, W, H, N, S


def chunk_box(lo, hi, geo):
    """lo/hi: (..., 3) int base positions.  geo = (Bx, By, Bz_positions, slices
    per chunk): x positions per brick, y positions per brick, z positions per
    brick (slices = Bz + 1), slices per 64-B chunk.  Returns chunk counts."""
    Bx, By, Bz, cs = geo
    nbx = hi[..., 0] // Bx - lo[..., 0] // Bx + 1
    nby = hi[..., 1] // By - lo[..., 1] // By + 1
    # z: slice index s = (c // Bz) * (Bz + 1) + c % Bz, the footprint needs s and s + 1
    s_lo = (lo[..., 2] // Bz) * (Bz + 1) + lo[..., 2] % Bz
    s_hi = (hi[..., 2] // Bz) * (Bz + 1) + hi[..., 2] % Bz + 1
    nk = s_hi // cs - s_lo // cs + 1
    return nbx * nby * nk, nbx, nby, nk


GEOS = {
    # name: (x positions, y positions, z positions per brick, slices per 64-B chunk)
    "brick4832": (3, 7, 31, 2),    # 4x8x32 B bricks, chunk = 2 slices of 32 B
    "brick4416": (3, 3, 15, 4),    # 4x4x16 B bricks (1.83x bytes), chunk = 4 slices of 16 B
    "brick4432": (3, 3, 31, 4),
    "brick4864": (3, 7, 63, 2),
}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--tiles", type=int, default=4, help="model every K-th tile")
    ap.add_argument("--chunk", default="brick4832")
    ap.add_argument("--cap", type=int, default=16, help="chunks per channel a slab holds")
    args = ap.parse_args()
    geo = GEOS[args.chunk]
    n, p0, st = rays()
    tx8, ty8 = W // 8, (H + 7) // 8
    lane = np.arange(64)
    lx, ly = ((lane >> 2) & 3) * 2 + (lane & 1), (lane >> 4) * 2 + ((lane >> 1) & 1)
    T = np.arange(tx8 * ty8)[::args.tiles]
    X = (T % tx8)[:, None] * 8 + lx[None, :]
    Y = (T // tx8)[:, None] * 8 + ly[None, :]
    ok = Y < H
    Y = np.minimum(Y, H - 1)
    nn = np.where(ok, n[Y, X], 0)
    keep = nn.max(1) > 0
    nn, P0, ST = nn[keep], p0[Y, X][keep], st[Y, X][keep]
    tot_chunks = []
    tot_steps = 0
    wave_steps = 0
    fills = 0
    over = 0
    for i in range(S):
        act = i < nn
        wave = act.any(1)
        if not wave.any():
            break
        a_ = act[wave]
        P = P0[wave] + ST[wave] * i
        tot_steps += a_.sum()
        wave_steps += wave.sum()
        for sc in (1, .8, .75, .7):
            g = np.clip(np.floor(P * sc * N + 0.5).astype(np.int64), 0, N)
            big = np.iinfo(np.int64).max
            lo = np.where(a_[..., None], g, big).min(1)
            hi = np.where(a_[..., None], g, -1).max(1)
            ch, _, _, _ = chunk_box(lo, hi, geo)
            tot_chunks.append(ch)
            fills += np.ceil(ch / 16).sum()
            over += (ch > args.cap).sum()
    ch = np.concatenate(tot_chunks)
    print(f"{args.chunk}: {keep.sum()} tiles with rays (every {args.tiles}th), {tot_steps} lane-steps, "
          f"{wave_steps} wave-steps, {tot_steps / wave_steps:.1f} live lanes per wave-step")
    print(f"  chunks per channel-step: mean {ch.mean():.1f}, p50 {np.percentile(ch, 50):.0f}, "
          f"p90 {np.percentile(ch, 90):.0f}, p99 {np.percentile(ch, 99):.0f}, max {ch.max()}")
    print(f"  fill L1 lookups per wave-step {4 * ch.mean():.1f} (shipped kernel: 8 x 26.6 = 213)")
    print(f"  fill instructions per wave-step {fills / wave_steps:.2f} (16 chunks each)")
    print(f"  channel-steps over {args.cap} chunks: {over / len(ch) * 100:.2f} %")
    for cap in (8, 16, 24, 32, 48):
        print(f"    <= {cap}: {np.mean(ch <= cap) * 100:.1f} %")


if __name__ == "__main__":
    main()
