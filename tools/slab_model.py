"""CPU model of per-wave LDS slabs for the grid march (config 5 experiment).

For each 8x8 tile (one wave) and each step, the box of padded texel
positions the wave's live rays touch per channel: floor(g) .. floor(g)+1
with g = P*S_t + T_t.  Reports the slab extents, the
(row, dword) pairs a fill needs, and how often a capacity is exceeded.
Usage: python tools/slab_model.py [N] [W H steps]
"""
import sys, os
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
sys.path.insert(0, os.path.join(ROOT, "tests"))
import vr_oracle as o
import glsl_f64 as g

N = int(sys.argv[1]) if len(sys.argv) > 1 else 512
W, H, S = (int(v) for v in sys.argv[2:5]) if len(sys.argv) > 4 else (1920, 1080, 128)
obj, glob = o.reference_shader_data(W / H)
m = o.march(S)
# ray setup: reuse the f64 restatement's front half by running it on a 1^3 volume
# is too slow at 1080p; restate the few lines here instead
M, V, P = g._m(obj, 0), g._m(obj, 1), g._m(obj, 2)
L = g._m(glob, 0)
cam = np.asarray(glob[16:19], np.float64)
bmin = np.array(m.box_min[:]); bmax = np.array(m.box_max[:])
PV = P @ V; inv_pv = np.linalg.inv(PV)
eye_h = np.linalg.inv(V) @ np.array([0, 0, 0, 1.0]); eye = eye_h[:3] / eye_h[3]
xs = (np.arange(W) + 0.5) / W * 2 - 1; ys = (np.arange(H) + 0.5) / H * 2 - 1
X, Y = np.meshgrid(xs, ys)
ndc = np.stack([X.ravel(), Y.ravel(), np.ones(X.size), np.ones(X.size)])
wp = inv_pv @ ndc; far = (wp[:3] / wp[3]).T
Minv = np.linalg.inv(M)
eye_l = (Minv @ np.append(eye, 1))[:3]
far_l = (Minv @ np.vstack([far.T, np.ones(len(far))]))[:3].T
v = far_l - eye_l
with np.errstate(divide="ignore", invalid="ignore"):
    t0 = (bmin - eye_l) / v; t1 = (bmax - eye_l) / v
tn = np.max(np.minimum(t0, t1), 1); tf = np.min(np.maximum(t0, t1), 1)
hit = tn <= tf
frag_l = eye_l + v * np.where(hit, tn, 0)[:, None]
fw = (M @ np.vstack([frag_l.T, np.ones(len(frag_l))]))[:3].T
c = (L @ np.append(cam, 1))[:3]
fr = (L @ np.vstack([fw.T, np.ones(len(fw))]))[:3].T
d = fr - c; d /= np.linalg.norm(d, axis=1, keepdims=True)
with np.errstate(divide="ignore", invalid="ignore"):
    a0 = (bmin - c) / d; a1 = (bmax - c) / d
tnear = np.max(np.minimum(a0, a1), 1); tfar = np.min(np.maximum(a0, a1), 1)
step = (1.0 / S) * 4
pin = c + d * tnear[:, None]; pout = c + d * tfar[:, None]
n = np.minimum(S, np.trunc(np.linalg.norm(pout - pin, axis=1) / step))
n = np.where(hit, n, 0).astype(int)
pin = (pin - bmin) / (bmax - bmin); sv = step * d / (bmax - bmin)
scale = [1.0, 0.8, 0.75, 0.7]
print(f"N={N} {W}x{H}x{S}: executed steps {n.sum()}")
# tiles
TX, TY = (W + 7) // 8, (H + 7) // 8
stats = []
cap_fail = 0; tot = 0
rows_hist = []; pairs_hist = []; ent_hist = []
for ty in range(0, TY, 2):          # half the tile rows (speed)
    for tx in range(TX):
        ys_ = np.arange(ty * 8, min(ty * 8 + 8, H)); xs_ = np.arange(tx * 8, min(tx * 8 + 8, W))
        idx = (ys_[:, None] * W + xs_[None, :]).ravel()
        nn = n[idx]
        if nn.max() <= 0: continue
        for i in range(nn.max()):
            act = idx[nn > i]
            p = pin[act] + i * sv[act]
            lo = p.min(0); hi = p.max(0)
            for t in range(4):
                glo = np.floor(lo * scale[t] * N + 0.5); ghi = np.floor(hi * scale[t] * N + 0.5)
                e = (ghi - glo + 2).astype(int)
                ndw = ((glo[0] % 4) + e[0] + 1 + 3) // 4   # dwords per row incl. the pair's x+1 byte
                rows = e[1] * e[2]
                rows_hist.append(rows); pairs_hist.append(rows * ndw); ent_hist.append(rows * ndw * 4)
                tot += 1
stats = np.array(pairs_hist); rows = np.array(rows_hist); ent = np.array(ent_hist)
for q in (50, 90, 99, 99.9, 100):
    print(f"p{q}: rows {np.percentile(rows, q):.0f} (row,dword) pairs {np.percentile(stats, q):.0f} entries {np.percentile(ent, q):.0f}")
for cap in (64, 128, 192, 256):
    print(f"pairs <= {cap}: {np.mean(stats <= cap) * 100:.2f} %  (load instr per channel-step mean {np.mean(np.ceil(stats / 64)):.2f})")
