"""Count the 128-B brick5 lines a 1080p x 128 frame of the 512^3 volume reads,
in total and per XCD (the sum over the eight L2s of their distinct lines), for
a tile -> XCD mapping.  A CPU model of the regions schedule's premise
(DESIGN.md sec. 5.3): with an L2 that kept every line, FETCH would equal the
per-XCD figure.  Reference camera (TestMain.cpp:219-245), frag.glsl:42-55
step counts, taps at scales 1/.8/.75/.7 (frag.glsl:66-69).

    python tools/xcd_lines_sim.py        # ~1 min, ~10 GB RAM
"""
import numpy as np

W, H, N, S = 1920, 1080, 512, 128
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
py, px = np.nonzero(n > 0)
nn = n[py, px]
print("executed steps", nn.sum())
tx8, ty8 = (W + 7) // 8, (H + 7) // 8
cx, cy = tx8 // 2, ty8 // 2


def ring_index(dx, dy):
    r = np.maximum(abs(dx), abs(dy))
    base = (2 * r - 1) ** 2
    k = np.where(dy == -r, base + (dx + r), np.where(dx == r, base + 2 * r + (dy + r),
                 np.where(dy == r, base + 4 * r + (r - dx), base + 6 * r + (r - dy))))
    return np.where(r == 0, 0, k)


rep = np.repeat(np.arange(len(nn)), nn)
i = np.arange(nn.sum()) - np.repeat(np.cumsum(nn) - nn, nn)
P = ((eye + d[py, px] * tn[py, px][:, None] + 1) / 2)[rep] + ((ds * d[py, px]) / 2)[rep] * i[:, None]
nb = (N + 1 + 3) // 4
lines = []
for sc in (1, .8, .75, .7):
    b = np.clip(np.floor(P * sc * N - 0.5).astype(np.int64) + 1, 0, N) // 4
    lines.append((b[:, 0] * nb + b[:, 1]) * nb + b[:, 2])
del P
print("distinct lines, all XCDs together: %.1f MB" % (sum(np.unique(l).size for l in lines) * 128 / 1e6))

TX, TY = np.meshgrid(np.arange(tx8), np.arange(ty8))
TX, TY = TX.ravel(), TY.ravel()
tid = (py // 8) * tx8 + px // 8
tmax = np.zeros(tx8 * ty8)
np.maximum.at(tmax, tid, nn)
k = ring_index(TX - cx, TY - cy)
R = max(cx, tx8 - 1 - cx, cy, ty8 - 1 - cy)
nw = 4 * ((((2 * R + 1) ** 2 + 1) // 2 + 3) // 4)
rings = ((np.where(k < nw, k, k - nw) // 4) % 8)          # ring positions, 2 per wave, WG % 8
ang = np.arctan2(TY - cy + .01, TX - cx + .01) + np.pi


def wedges(per_xcd):
    """equal-work angular wedges, wedge j -> XCD j % 8 (build_regions)"""
    order = np.argsort(ang)
    cum = np.cumsum(tmax[order]) - tmax[order] / 2
    K = 8 * per_xcd
    w = np.empty(len(ang), int)
    w[order] = np.minimum(K - 1, (cum / tmax.sum() * K).astype(int)) % 8
    return w


for name, xm in [("rings (round-robin)", rings), ("regions, 1 wedge/XCD", wedges(1)),
                 ("regions, 2 wedges/XCD", wedges(2)), ("regions, 4 wedges/XCD", wedges(4))]:
    per = sum(np.unique(l * 8 + xm[tid][rep]).size for l in lines)
    work = np.bincount(xm, weights=tmax, minlength=8)
    print(f"{name:24s} per-XCD distinct lines {per * 128 / 1e6:7.1f} MB, work max/mean {work.max() / work.mean():.3f}")
