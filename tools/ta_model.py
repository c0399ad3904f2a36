"""CPU model of the vector-memory work of the grid march at config 5
(512^3, 1080p x 128, reference camera): for every wave load instruction
(8x8 tile, step, tap, z-slice) the L1 tag lookups it costs, counted as the
TA calibration (tools/tcp_calib.hip) found them: a
b64/b96/b128 load is looked up per quad of 4 lanes, once per distinct 128-B
line among the quad's active lanes.  Also: distinct lines per wave
instruction (what an LDS-staged fill would have to fetch) and the 16-B chunks
of a tile's per-step bounding box.

    python tools/ta_model.py [--layout brick4832] [--quad 2x2|4x1|1x4] [--tiles K]

Geometry: frag.glsl:42-55 (step counts, box-normalised points), taps at
scales 1/.8/.75/.7 (frag.glsl:66-69), padded base a = floor(P*s*N + .5).
"""
import argparse

import numpy as np

W, H, N, S = 1920, 1080, 512, 128


def rays():
    eye = np.array([3., 3., 3.])
    f = -eye / np.linalg.norm(eye)
    up = np.array([0, 0, 1.])
    s = np.cross(f, up); s /= np.linalg.norm(s)
    u = np.cross(s, f)
    th = np.tan(np.radians(45) / 2)
    asp = 1280 / 720
    X, Y = np.meshgrid((np.arange(W) + .5) / W * 2 - 1, (np.arange(H) + .5) / H * 2 - 1)
    d = f[None, None, :] + X[..., None] * th * asp * s + (-Y[..., None]) * th * u
    d /= np.linalg.norm(d, axis=-1, keepdims=True)
    with np.errstate(divide="ignore"):
        ta, tb = (-1 - eye) / d, (1 - eye) / d
    tn, tf = np.minimum(ta, tb).max(-1), np.maximum(ta, tb).min(-1)
    ds = 4 / S
    n = np.where(tn <= tf, np.minimum(S, ((tf - tn) / ds).astype(int)), 0)
    p0 = (eye + d * tn[..., None] + 1) / 2
    st = (ds * d) / 2
    return n, p0, st


def brick8_offset(Ry, Rz):
    """8-B rows (7 x positions), Ry rows per slice, Rz slices per brick: a
    z-slice of a footprint is one dword-aligned 16-B load (rows y, y+1), the
    z+1 slice 8*Ry bytes on (BRICK8's scheme).  Returns the load's first and
    last byte offsets for both slices."""
    By, Bz, brick = Ry - 1, Rz - 1, 8 * Ry * Rz
    nbx, nby = N // 7 + 1, N // By + 1

    def off(a, b, c):
        o = (a // 7) * brick + (b // By) * brick * nbx + (c // Bz) * brick * nbx * nby \
            + (b % By) * 8 + (c % Bz) * 8 * Ry + (a % 7)
        o = o & ~3
        return o, o + 8 * Ry
    return off


def brick_offset(layout):
    """(a, b, c) -> byte offset of the z-slice row load (off & ~3) and the
    z+1 slice's, for BRICK4-family geometries (4-B rows, x positions 0..2)."""
    geo = {"brick4": (3, 3, 4, 4, 64), "brick448": (3, 7, 4, 8, 128), "brick488": (7, 7, 8, 8, 256),
           "brick4816": (7, 15, 8, 16, 512), "brick4832": (7, 31, 8, 32, 1024),
           "brick4864": (7, 63, 8, 64, 2048), "brick41616": (15, 15, 16, 16, 1024)}[layout]
    By, Bz, Ry, Rz, brick = geo
    nbx, nby = N // 3 + 1, N // By + 1

    def off(a, b, c):
        o = (a // 3) * brick + (b // By) * brick * nbx + (c // Bz) * brick * nbx * nby \
            + (b % By) * 4 + (c % Bz) * 4 * Ry
        return o, o + 4 * Ry
    return off


def generic_b4(Ry, Rz):
    """A BRICK4-family geometry of 4-B rows (3 x positions), Ry rows per slice
    and Rz slices per brick (the bricks overlap by one position per axis)."""
    By, Bz, brick = Ry - 1, Rz - 1, 4 * Ry * Rz
    nbx, nby = N // 3 + 1, N // By + 1

    def off(a, b, c):
        o = (a // 3) * brick + (b // By) * brick * nbx + (c // Bz) * brick * nbx * nby \
            + (b % By) * 4 + (c % Bz) * 4 * Ry
        return o, o + 4 * Ry
    return off, (4 * Ry * Rz) / (3 * By * Bz)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--layout", default="brick4832")
    ap.add_argument("--quad", default="2x2")
    ap.add_argument("--tiles", type=int, default=0, help="model every K-th tile (0: all)")
    ap.add_argument("--b32", action="store_true",
                    help="4-B row loads (rows y, y+1 of each slice: 4 per tap), looked up per 16-lane group and line")
    args = ap.parse_args()
    n, p0, st = rays()
    tx8, ty8 = W // 8, (H + 7) // 8
    # lanes of each tile: lane -> (x, y); quads are lanes 4q..4q+3
    lane = np.arange(64)
    if args.quad == "2x2":
        lx, ly = ((lane >> 2) & 3) * 2 + (lane & 1), (lane >> 4) * 2 + ((lane >> 1) & 1)
    elif args.quad == "4x1":
        lx, ly = lane & 7, lane >> 3
    else:  # 1x4: four rows of one column
        lx, ly = (lane >> 2) & 7, (lane >> 5) * 4 + (lane & 3)
    T = np.arange(tx8 * ty8)
    if args.tiles:
        T = T[::args.tiles]
    X = (T % tx8)[:, None] * 8 + lx[None, :]
    Y = (T // tx8)[:, None] * 8 + ly[None, :]
    ok = Y < H
    Y = np.minimum(Y, H - 1)
    nn = np.where(ok, n[Y, X], 0)
    keep = nn.max(1) > 0
    nn, P0, ST = nn[keep], p0[Y, X][keep], st[Y, X][keep]
    print(f"{args.layout} quad {args.quad}: {keep.sum()} tiles with rays, {nn.sum()} executed steps")
    if args.layout.startswith("b4_"):   # b4_<Ry>_<Rz>: tools/ta_model.py --search
        _, ry, rz = args.layout.split("_")
        off, ratio = generic_b4(int(ry), int(rz))
        print(f"  bytes {ratio:.3f}x the volume")
        span = 8
    elif args.layout.startswith("r8_"):
        _, ry, rz = args.layout.split("_")
        off = brick8_offset(int(ry), int(rz))
        span = 16
    else:
        off = brick_offset(args.layout)
        span = 8
    look = insts = lines_w = steps = 0
    bbox_chunks = 0
    for i in range(S):
        act = i < nn
        wave = act.any(1)
        if not wave.any():
            break
        a_ = act[wave]
        P = P0[wave] + ST[wave] * i
        steps += a_.sum()
        for sc in (1, .8, .75, .7):
            g = np.clip(np.floor(P * sc * N + 0.5).astype(np.int64), 0, N)
            offs = off(g[..., 0], g[..., 1], g[..., 2])
            if args.b32:
                offs = [o + d for o in offs for d in (0, 4)]   # rows y, y+1 of each slice
            for o in offs:
                ln = np.where(a_, o // 128, -1)
                if args.b32:
                    q = np.sort(ln.reshape(len(ln), 4, 16), axis=-1)
                    new = np.concatenate([q[..., :1] >= 0, (q[..., 1:] != q[..., :-1]) & (q[..., 1:] >= 0)], -1)
                    look += new.sum()
                    insts += len(ln)
                    continue
                ln2 = np.where(a_ & ((o // 128) != ((o + span - 1) // 128)), (o + span - 1) // 128, -1)
                q = np.sort(np.concatenate([ln.reshape(len(ln), 16, 4), ln2.reshape(len(ln), 16, 4)], -1), axis=-1)
                new = np.concatenate([q[..., :1] >= 0, (q[..., 1:] != q[..., :-1]) & (q[..., 1:] >= 0)], -1)
                look += new.sum()
                w = np.sort(ln, axis=-1)
                lines_w += (np.concatenate([w[:, :1] >= 0, (w[:, 1:] != w[:, :-1]) & (w[:, 1:] >= 0)], -1)).sum()
                insts += len(ln)
            # planar bounding box of the tile's footprints (rows of x, 16-B chunks)
            big = np.iinfo(np.int64).max
            lo = np.where(a_[..., None], g, big).min(1)
            hi = np.where(a_[..., None], g, -1).max(1) + 1
            rows = (hi[:, 1] - lo[:, 1] + 1) * (hi[:, 2] - lo[:, 2] + 1)
            chunks = (hi[:, 0] // 16) - (lo[:, 0] // 16) + 1
            bbox_chunks += (rows * chunks).sum()
    print(f"  wave load instructions {insts}, lane-steps {steps}, "
          f"{insts * 64 / steps:.2f} lane loads/step (incl. idle lanes)")
    per_step = insts / (steps / 64) if steps else 0
    print(f"  L1 lookups per instruction {look / insts:.2f}, per wave-step {look / insts * (16 if args.b32 else 8):.1f}")
    print(f"  distinct 128-B lines per instruction (wave) {lines_w / insts:.2f}")
    print(f"  planar bbox 16-B chunks per tap-step {bbox_chunks / (insts / 2):.1f} "
          f"(= {bbox_chunks / (insts / 2) / 64:.2f} b128 wave loads)")


if __name__ == "__main__":
    main()
