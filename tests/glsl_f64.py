"""An independent float64 restatement of the reference hot path -- TEST ONLY.

This is a second, separately written statement of what the reference computes
per pixel, used to check the C oracle (oracle/vr_oracle.c) rather than the
product.  It shares no code, no ray basis and no padded-texel trick with the
oracle or the HIP library: it follows the GLSL and the Vulkan rules literally,
in float64 numpy.

* Coverage / fragPosition (vert.glsl:17-22 + rasterisation).  The reference
  draws the 12-triangle cube of TestMain.cpp:94-112 (vertices +-1) through
  Projection*View*Model, culls back faces (VulkanPipeline.cpp:107-108, CCW
  front; the y-flip of TestMain.cpp:228 keeps outward faces CCW on screen),
  depth test LESS (:132).  So a pixel is covered iff the View eye's ray
  through the pixel centre hits the cube in front of the eye, and the hit
  survives clipping (0 <= z_clip <= w_clip).  fragPosition is that hit point
  (world), the nearest front face.
* frag.glsl:36-80, line by line: cameraInBoxLocal = W2L * CameraPosition,
  fragmentInBoxLocal = W2L * fragPosition, rayDirection = normalize(...),
  IntersectAABB (:18-27), stepSize = (1/maxSteps)*4, Pin/Pout,
  actualSteps = min(maxSteps, int(distance/stepSize)), normalise to [0,1],
  the four texture() taps at Pin*s_t + MediaScroll-column * w_t
  (:66-69), currentSample = (s1*s2)*(s3+s4)*scale, Pin += stepVec,
  Beer-Lambert 1 - exp(density*min(-acc*stepSize, 0)).
* texture() (VulkanCore.cpp:676-710, VulkanTexture.cpp:111-156): R8G8B8A8
  UNORM (c/255), LINEAR filter: texel space u*N - 0.5, i0 = floor, alpha =
  frac, and VK_SAMPLER_ADDRESS_MODE_MIRRORED_REPEAT as the Vulkan spec writes
  it: i' = (N-1) - mirror(mod(i, 2N) - N), mirror(a) = a >= 0 ? a : -(1+a).
  LOD 0 (maxLod 0, magnification at the reference footprint).

Matrices are column-major float32 arrays as in the C ABI (obj48 = Model, View,
Projection; glob36 = WorldToLocal, CameraPosition + pad, MediaScroll), taken
to float64 once.
"""
from __future__ import annotations

import numpy as np


def _m(a, k):
    """k-th column-major 4x4 matrix of a flat float array -> float64 (row, col)."""
    return np.asarray(a[16 * k:16 * k + 16], np.float64).reshape(4, 4).T


def _vk_mirrored_repeat(i, n):
    """Vulkan spec texel-coordinate wrapping, MIRRORED_REPEAT."""
    two = 2 * n
    m = i - two * np.floor_divide(i, two)          # mod(i, 2N), floored
    a = m - n
    mir = np.where(a >= 0, a, -(1 + a))
    return (n - 1) - mir


def _texture(vol_c, nx, ny, nz, u):
    """texture(sampler3D, u).channel: trilinear LINEAR filter, float64."""
    dims = (nx, ny, nz)
    i0, al = [], []
    for ax in range(3):
        t = u[:, ax] * dims[ax] - 0.5
        f = np.floor(t)
        i0.append(f.astype(np.int64))
        al.append(t - f)
    ix = [_vk_mirrored_repeat(i0[0], nx), _vk_mirrored_repeat(i0[0] + 1, nx)]
    iy = [_vk_mirrored_repeat(i0[1], ny), _vk_mirrored_repeat(i0[1] + 1, ny)]
    iz = [_vk_mirrored_repeat(i0[2], nz), _vk_mirrored_repeat(i0[2] + 1, nz)]
    acc = np.zeros(u.shape[0])
    for kz in (0, 1):
        wz = al[2] if kz else 1.0 - al[2]
        for ky in (0, 1):
            wy = al[1] if ky else 1.0 - al[1]
            for kx in (0, 1):
                wx = al[0] if kx else 1.0 - al[0]
                texel = vol_c[iz[kz], iy[ky], ix[kx]].astype(np.float64) / 255.0
                acc += (wx * wy * wz) * texel
    return acc


def render(vol, obj48, glob36, march, width, height, rows=None):
    """Grey value and step count per pixel of the given rows (default all):
    (grey float64 (len(rows), W) with NaN where uncovered, n int (-1 uncovered))."""
    vol = np.ascontiguousarray(vol)
    nz, ny, nx, _ = vol.shape
    M, V, P = _m(obj48, 0), _m(obj48, 1), _m(obj48, 2)
    L = _m(glob36, 0)
    cam = np.asarray(glob36[16:19], np.float64)
    ms = np.asarray(glob36[20:36], np.float64).reshape(4, 4)   # ms[col][row] = MediaScroll[col][row]
    max_steps = int(march.max_steps)
    bmin = np.array(march.box_min[:], np.float64)
    bmax = np.array(march.box_max[:], np.float64)
    scale = float(np.float32(march.scale))
    density = float(np.float32(march.density))
    tap_s = [float(v) for v in march.tap_scale]
    tap_w = [float(v) for v in march.tap_weight]
    rows = np.arange(height) if rows is None else np.asarray(rows)

    # --- rasterisation: the View eye's ray through each pixel centre, world space
    PV = P @ V
    PVM = PV @ M
    inv_pv = np.linalg.inv(PV)
    eye_h = np.linalg.inv(V) @ np.array([0.0, 0.0, 0.0, 1.0])
    eye = eye_h[:3] / eye_h[3]
    xs = (np.arange(width) + 0.5) / width * 2.0 - 1.0
    ys = (rows + 0.5) / height * 2.0 - 1.0
    X, Y = np.meshgrid(xs, ys)
    ndc = np.stack([X.ravel(), Y.ravel(), np.ones(X.size), np.ones(X.size)])   # far-plane point
    wp = inv_pv @ ndc
    far = (wp[:3] / wp[3]).T
    Minv = np.linalg.inv(M)   # mesh (local) space of the cube vertices
    eye_l = (Minv @ np.append(eye, 1.0))[:3]
    far_l = (Minv @ np.vstack([far.T, np.ones(far.shape[0])]))[:3].T
    v = far_l - eye_l[None, :]
    with np.errstate(divide="ignore", invalid="ignore"):
        # the mesh cube (TestMain.cpp:94-103, +-1) is the march box (frag.glsl:31-32, +-1);
        # vr_march_params moves both together
        t0 = (bmin[None, :] - eye_l[None, :]) / v
        t1 = (bmax[None, :] - eye_l[None, :]) / v
    tn = np.max(np.minimum(t0, t1), axis=1)
    tf = np.min(np.maximum(t0, t1), axis=1)
    hit = tn <= tf
    frag_l = eye_l[None, :] + v * np.where(hit, tn, 0.0)[:, None]
    clip = (PVM @ np.vstack([frag_l.T, np.ones(frag_l.shape[0])])).T
    covered = hit & (clip[:, 3] > 0) & (clip[:, 2] >= 0) & (clip[:, 2] <= clip[:, 3])
    frag_world = (M @ np.vstack([frag_l.T, np.ones(frag_l.shape[0])]))[:3].T

    # --- frag.glsl:36-55
    c = (L @ np.append(cam, 1.0))[:3]                                         # :36
    fr = (L @ np.vstack([frag_world.T, np.ones(frag_world.shape[0])]))[:3].T   # :37
    d = fr - c[None, :]
    d /= np.linalg.norm(d, axis=1, keepdims=True)                             # :38
    with np.errstate(divide="ignore", invalid="ignore"):
        tmin = (bmin[None, :] - c[None, :]) / d                                # :20
        tmax = (bmax[None, :] - c[None, :]) / d                                # :21
    tnear = np.max(np.minimum(tmin, tmax), axis=1)                            # :22-24
    tfar = np.min(np.maximum(tmin, tmax), axis=1)                             # :25
    step = (1.0 / max_steps) * float(np.float32(march.step_scale))             # :42 (the constant 4)
    pin = c[None, :] + d * tnear[:, None]                                     # :43
    pout = c[None, :] + d * tfar[:, None]                                     # :44
    step_vec = step * d                                                       # :45
    with np.errstate(invalid="ignore"):
        n = np.minimum(max_steps, np.trunc(np.linalg.norm(pout - pin, axis=1) / step))   # :46
    rng = np.abs(bmax - bmin)                                                 # :51
    pin = (pin - bmin[None, :]) / rng[None, :]                                # :49, :52
    step_vec = step_vec / rng[None, :]                                        # :54
    ok = covered & np.isfinite(n)
    n = np.where(ok, n, -1).astype(np.int64)

    # --- frag.glsl:57-75 over the covered pixels
    idx = np.nonzero(n > 0)[0]
    p = pin[idx].copy()
    sv = step_vec[idx]
    nn = n[idx]
    acc = np.zeros(idx.size)
    planes = [vol[..., ch] for ch in range(4)]
    off = [np.array([ms[0][t], ms[1][t], ms[2][t]]) * tap_w[t] for t in range(4)]   # MediaScroll[0..2].x/y/z/w
    for i in range(int(nn.max()) if idx.size else 0):
        act = np.nonzero(i < nn)[0]
        pa = p[act]
        s = [_texture(planes[t], nx, ny, nz, pa * tap_s[t] + off[t][None, :]) for t in range(4)]   # :66-69
        acc[act] += (s[0] * s[1]) * (s[2] + s[3]) * scale                    # :71-73
        p[act] += sv[act]                                                     # :74
    total = np.zeros(n.size)
    total[idx] = acc
    grey = 1.0 - np.exp(density * np.minimum(-total * step, 0.0))             # :76-79
    grey = np.where(n >= 0, grey, np.nan)
    return grey.reshape(len(rows), width), n.reshape(len(rows), width)
