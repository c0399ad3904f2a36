"""Where the oracle's distance to the float64 restatement comes from (verdict
r02 #7; test infrastructure, CPU only).

tests/glsl_f64.py reads frag.glsl literally but in float64 throughout.  The
reference itself runs in fp32: Pin += stepVec (frag.glsl:74) accumulates in
fp32, and the tap coordinate Pin*s_t + MediaScroll*w_t (:66-69) is an fp32
expression before the sampler's u*N - 0.5.  This script re-runs the float64
restatement with those two pieces switched to fp32, one at a time, and
reports the oracle's max |d grey| and step-count flips against each:

  f64            the restatement as tests/glsl_f64.py has it
  p32            ray point accumulated in fp32 (GLSL's own drift)
  p32+tap_glsl   and the tap coordinate as GLSL writes it: u = fl(fl(P*s)+o),
                 t = fl(u*N) - 0.5
  p32+tap_fma    and the tap coordinate as the spec:
                 g = fma(P, s*N, o*N + 0.5)

    python tools/tap_form_study.py
"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
sys.path.insert(0, os.path.join(ROOT, "tests"))
import glsl_f64 as g  # noqa: E402
import vr_oracle as oracle  # noqa: E402

f32 = np.float32


def render_variant(vol, obj48, glob36, march, width, height, p32=False, tap=None):
    """glsl_f64.render with the ray point and/or the tap coordinate in fp32."""
    vol = np.ascontiguousarray(vol)
    nz, ny, nx, _ = vol.shape
    # reuse the literal restatement for everything before the loop: run it on
    # the rows, but redo the loop here (a copy of its last part, with switches)
    grey64, n = g.render(vol, obj48, glob36, march, width, height)
    src = g.render.__code__  # noqa: F841  (documentation: the loop below mirrors glsl_f64.render's)
    M, V, P = g._m(obj48, 0), g._m(obj48, 1), g._m(obj48, 2)
    L = g._m(glob36, 0)
    cam = np.asarray(glob36[16:19], np.float64)
    ms = np.asarray(glob36[20:36], np.float64).reshape(4, 4)
    max_steps = int(march.max_steps)
    bmin = np.array(march.box_min[:], np.float64)
    bmax = np.array(march.box_max[:], np.float64)
    scale = float(f32(march.scale))
    density = float(f32(march.density))
    tap_s = [float(v) for v in march.tap_scale]
    tap_w = [float(v) for v in march.tap_weight]
    rows = np.arange(height)
    PV = P @ V
    inv_pv = np.linalg.inv(PV)
    eye_h = np.linalg.inv(V) @ np.array([0.0, 0.0, 0.0, 1.0])
    eye = eye_h[:3] / eye_h[3]
    xs = (np.arange(width) + 0.5) / width * 2.0 - 1.0
    ys = (rows + 0.5) / height * 2.0 - 1.0
    X, Y = np.meshgrid(xs, ys)
    ndc = np.stack([X.ravel(), Y.ravel(), np.ones(X.size), np.ones(X.size)])
    wp = inv_pv @ ndc
    far = (wp[:3] / wp[3]).T
    Minv = np.linalg.inv(M)
    eye_l = (Minv @ np.append(eye, 1.0))[:3]
    far_l = (Minv @ np.vstack([far.T, np.ones(far.shape[0])]))[:3].T
    v = far_l - eye_l[None, :]
    with np.errstate(divide="ignore", invalid="ignore"):
        t0 = (bmin[None, :] - eye_l[None, :]) / v
        t1 = (bmax[None, :] - eye_l[None, :]) / v
    tn = np.max(np.minimum(t0, t1), axis=1)
    hit = tn <= np.min(np.maximum(t0, t1), axis=1)
    frag_l = eye_l[None, :] + v * np.where(hit, tn, 0.0)[:, None]
    frag_world = (M @ np.vstack([frag_l.T, np.ones(frag_l.shape[0])]))[:3].T
    c = (L @ np.append(cam, 1.0))[:3]
    fr = (L @ np.vstack([frag_world.T, np.ones(frag_world.shape[0])]))[:3].T
    d = fr - c[None, :]
    d /= np.linalg.norm(d, axis=1, keepdims=True)
    with np.errstate(divide="ignore", invalid="ignore"):
        tmin = (bmin[None, :] - c[None, :]) / d
        tmax = (bmax[None, :] - c[None, :]) / d
    tnear = np.max(np.minimum(tmin, tmax), axis=1)
    step = (1.0 / max_steps) * float(f32(march.step_scale))
    pin = c[None, :] + d * tnear[:, None]
    step_vec = step * d
    rng = np.abs(bmax - bmin)
    pin = (pin - bmin[None, :]) / rng[None, :]
    step_vec = step_vec / rng[None, :]
    n = n.ravel()
    idx = np.nonzero(n > 0)[0]
    p = pin[idx].copy()
    sv = step_vec[idx]
    if p32:
        p, sv = p.astype(f32), sv.astype(f32)
    nn = n[idx]
    acc = np.zeros(idx.size)
    planes = [vol[..., ch] for ch in range(4)]
    dims = np.array([nx, ny, nz], np.float64)
    off = [np.array([ms[0][t], ms[1][t], ms[2][t]]) * tap_w[t] for t in range(4)]
    for i in range(int(nn.max()) if idx.size else 0):
        act = np.nonzero(i < nn)[0]
        pa = p[act]
        s = []
        for t in range(4):
            if tap == "glsl":     # u = fl(fl(P*s) + o) in fp32, then texel space fl(u*N) - 0.5
                u = (pa.astype(f32) * f32(tap_s[t]) + off[t].astype(f32)[None, :]).astype(f32)
                tex = (u * dims.astype(f32)[None, :]).astype(f32).astype(np.float64) - 0.5
                s.append(texture_texel(planes[t], nx, ny, nz, tex))
            elif tap == "fma":    # the spec: g = fma(P, s*N, o*N + 0.5), texel space g - 1
                S = (f32(tap_s[t]) * dims.astype(f32)).astype(f32)
                T = (off[t].astype(f32) * dims.astype(f32) + f32(0.5)).astype(f32)
                gg = (pa.astype(np.float64) * S.astype(np.float64)[None, :] + T.astype(np.float64)[None, :]).astype(f32)
                s.append(texture_texel(planes[t], nx, ny, nz, gg.astype(np.float64) - 1.0))
            else:
                s.append(g._texture(planes[t], nx, ny, nz, pa.astype(np.float64) * tap_s[t] + off[t][None, :]))
        acc[act] += (s[0] * s[1]) * (s[2] + s[3]) * scale
        if p32:
            p[act] = (p[act] + sv[act]).astype(f32)
        else:
            p[act] += sv[act]
    total = np.zeros(n.size)
    total[idx] = acc
    grey = 1.0 - np.exp(density * np.minimum(-total * step, 0.0))
    grey = np.where(n >= 0, grey, np.nan)
    return grey.reshape(height, width), n.reshape(height, width)


def texture_texel(vol_c, nx, ny, nz, t):
    """The LINEAR filter at texel-space coordinate t (= u*N - 0.5), float64."""
    i0, al = [], []
    for ax in range(3):
        f = np.floor(t[:, ax])
        i0.append(f.astype(np.int64))
        al.append(t[:, ax] - f)
    dims = (nx, ny, nz)
    ix = [g._vk_mirrored_repeat(i0[0], dims[0]), g._vk_mirrored_repeat(i0[0] + 1, dims[0])]
    iy = [g._vk_mirrored_repeat(i0[1], dims[1]), g._vk_mirrored_repeat(i0[1] + 1, dims[1])]
    iz = [g._vk_mirrored_repeat(i0[2], dims[2]), g._vk_mirrored_repeat(i0[2] + 1, dims[2])]
    acc = np.zeros(t.shape[0])
    for kz in (0, 1):
        wz = al[2] if kz else 1.0 - al[2]
        for ky in (0, 1):
            wy = al[1] if ky else 1.0 - al[1]
            for kx in (0, 1):
                wx = al[0] if kx else 1.0 - al[0]
                acc += (wx * wy * wz) * (vol_c[iz[kz], iy[ky], ix[kx]].astype(np.float64) / 255.0)
    return acc


def compare(vol, obj, glob, m, W, H, **kw):
    ref, steps = oracle.render(vol, obj, glob, m, W, H, 0)
    ox = ref[..., 0].astype(np.float64)
    on = oracle.step_counts(obj, glob, m, W, H) if hasattr(oracle, "step_counts") else None
    grey, n = render_variant(vol, obj, glob, m, W, H, **kw)
    cov = n >= 0
    same = cov if on is None else cov & (on == n)
    dmax = float(np.nanmax(np.abs(ox[same] - grey[same]))) if same.any() else 0.0
    flips = float(((on != n) & cov).sum() / max(1, cov.sum())) if on is not None else float("nan")
    return dmax, flips


def main():
    cases = []
    rng = np.random.default_rng(7)
    vol_rand = rng.integers(0, 256, size=(23, 50, 37, 4), dtype=np.uint8)
    obj, glob = oracle.reference_shader_data(1.5, 35.0, -20.0)
    m = oracle.march(96)
    m.density, m.scale, m.step_scale = 2.5, 0.35, 3.0
    m.tap_scale[:] = [0.9, 1.1, 0.5, 1.0]
    cases.append(("random bytes, odd constants (test_odd_volume_and_constants)", vol_rand, obj, glob, m, 240, 160))
    vol48 = oracle.build_volume(48)
    obj2, glob2 = oracle.reference_shader_data(16 / 9, 20.0, 10.0)
    glob2 = np.array(glob2, np.float32)
    glob2[16:19] = (4.0, 2.0, 2.5)
    cases.append(("recipe 48^3, CameraPosition (4, 2, 2.5) off the eye", vol48, obj2, glob2, oracle.march(128), 320, 180))
    obj3, glob3 = oracle.reference_shader_data(16 / 9)
    cases.append(("recipe 48^3, reference camera", vol48, obj3, glob3, oracle.march(128), 320, 180))
    for name, vol, o, gl, mm, W, H in cases:
        print(name)
        for label, kw in [("f64", {}), ("p32", {"p32": True}), ("p32+tap_glsl", {"p32": True, "tap": "glsl"}),
                          ("p32+tap_fma", {"p32": True, "tap": "fma"})]:
            dmax, flips = compare(vol, o, gl, mm, W, H, **kw)
            print(f"  {label:14s} max |d grey| {dmax:.3g}   step flips {flips:.3g}")


if __name__ == "__main__":
    main()
