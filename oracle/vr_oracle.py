"""ctypes wrapper of oracle/libvr_oracle.so -- TEST INFRASTRUCTURE ONLY.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may use
this module, and only as the checker or the CPU baseline.  The product path
(volumetricrenderer_amd) never imports it.  Parity unpinned against reference
outputs: see vr_oracle.h.
"""
from __future__ import annotations

import ctypes
import math
import os

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "libvr_oracle.so")

FMT_RGBA32F, FMT_RGBA8_UNORM, FMT_RGBA8_SRGB = 0, 1, 2
NOISE_CELLULAR, NOISE_PERLIN, NOISE_SIMPLEX = 0, 1, 2


class March(ctypes.Structure):
    _fields_ = [("max_steps", ctypes.c_int32), ("step_scale", ctypes.c_float), ("density", ctypes.c_float),
                ("scale", ctypes.c_float), ("box_min", ctypes.c_float * 3), ("box_max", ctypes.c_float * 3),
                ("tap_scale", ctypes.c_float * 4), ("tap_weight", ctypes.c_float * 4),
                ("early_out", ctypes.c_float), ("reserved", ctypes.c_int32 * 3)]


class Recipe(ctypes.Structure):
    _fields_ = [("size", ctypes.c_int32), ("freq", ctypes.c_float * 4), ("seed", ctypes.c_int32 * 4),
                ("literal_overwrite", ctypes.c_int32)]


class Procedural(ctypes.Structure):
    _fields_ = [("enabled", ctypes.c_int32), ("grid_scale", ctypes.c_float), ("octaves", ctypes.c_int32),
                ("freq0", ctypes.c_float), ("lacunarity", ctypes.c_float), ("gain", ctypes.c_float),
                ("seed_fbm", ctypes.c_int32), ("worley_freq", ctypes.c_float), ("seed_worley", ctypes.c_int32),
                ("shadow_steps", ctypes.c_int32), ("sun_dir", ctypes.c_float * 3), ("reserved", ctypes.c_int32)]


_fp = ctypes.POINTER(ctypes.c_float)
_vp = ctypes.c_void_p
_lib = None


def lib() -> ctypes.CDLL:
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise ImportError(f"oracle not built: {LIB_PATH} (make -C oracle)")
        L = ctypes.CDLL(LIB_PATH)
        L.vro_perlin3.restype = L.vro_simplex3.restype = L.vro_cellular3.restype = ctypes.c_float
        for f in (L.vro_perlin3, L.vro_simplex3, L.vro_cellular3):
            f.argtypes = [ctypes.c_int32, ctypes.c_float, ctypes.c_float, ctypes.c_float]
        L.vro_gen_uniform_grid3d.argtypes = [ctypes.c_int, _vp, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                             ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_float,
                                             ctypes.c_int32, _fp, _fp]
        L.vro_gen_uniform_grid3d.restype = None
        L.vro_build_volume.argtypes = [ctypes.POINTER(Recipe), _vp]
        L.vro_reference_shader_data.argtypes = [ctypes.c_float] * 4 + [_fp, _fp]
        L.vro_reference_shader_data.restype = None
        L.vro_sample.argtypes = [_vp, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                 ctypes.c_float, ctypes.c_float, ctypes.c_float]
        L.vro_sample.restype = ctypes.c_float
        L.vro_mirror.argtypes = [ctypes.c_int, ctypes.c_int]
        L.vro_expf.argtypes = [ctypes.c_float]
        L.vro_expf.restype = ctypes.c_float
        L.vro_render.argtypes = [_vp, ctypes.c_int, ctypes.c_int, ctypes.c_int, _fp, _fp, ctypes.POINTER(March),
                                 ctypes.c_int, ctypes.c_int, ctypes.c_int, _vp, ctypes.c_size_t,
                                 ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.POINTER(ctypes.c_int64),
                                 ctypes.c_int]
        L.vro_render_procedural.argtypes = [ctypes.POINTER(Procedural), _fp, _fp, ctypes.POINTER(March),
                                            ctypes.c_int, ctypes.c_int, ctypes.c_int, _vp, ctypes.c_size_t,
                                            ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                            ctypes.POINTER(ctypes.c_int64), ctypes.POINTER(ctypes.c_int64),
                                            ctypes.POINTER(ctypes.c_int64), ctypes.c_int]
        L.vro_worley_cells.argtypes = [ctypes.POINTER(Procedural), ctypes.c_float, ctypes.c_float, ctypes.c_float]
        L.vro_procedural_density.argtypes = [ctypes.POINTER(Procedural), ctypes.c_float, ctypes.c_float,
                                             ctypes.c_float, ctypes.c_float]
        L.vro_procedural_density.restype = ctypes.c_float
        L.vro_step_counts.argtypes = [_fp, _fp, ctypes.POINTER(March), ctypes.c_int, ctypes.c_int, _vp]
        _lib = L
    return _lib


def march(max_steps=128, **kw) -> March:
    """frag.glsl constants (same defaults as vr_march_defaults)."""
    m = March(max_steps=max_steps, step_scale=4.0, density=1.0, scale=0.2)
    m.box_min[:] = [-1, -1, -1]
    m.box_max[:] = [1, 1, 1]
    m.tap_scale[:] = [1.0, 0.8, 0.75, 0.7]
    m.tap_weight[:] = [0.0, 0.2, 0.25, 0.3]
    for k, v in kw.items():
        if isinstance(v, (list, tuple)):
            getattr(m, k)[:] = list(v)
        else:
            setattr(m, k, v)
    return m


def from_params(p) -> March:
    """Copy a volumetricrenderer_amd MarchParams (same field layout)."""
    m = March()
    ctypes.memmove(ctypes.byref(m), ctypes.byref(p), ctypes.sizeof(March))
    return m


def reference_shader_data(aspect=1280.0 / 720.0, phi=0.0, theta=0.0, frame_time=0.0):
    obj = np.zeros(48, np.float32)
    glob = np.zeros(36, np.float32)
    lib().vro_reference_shader_data(aspect, phi, theta, frame_time, obj.ctypes.data_as(_fp),
                                    glob.ctypes.data_as(_fp))
    return obj, glob


def build_volume(size=128, freq=(0.01, 0.03, 0.19, 0.15), seed=(1, 2, 3, 4), literal=True) -> np.ndarray:
    r = Recipe(size=size, literal_overwrite=int(literal))
    r.freq[:] = list(freq)
    r.seed[:] = list(seed)
    out = np.empty((size, size, size, 4), np.uint8)
    if lib().vro_build_volume(ctypes.byref(r), out.ctypes.data_as(_vp)) != 0:
        raise MemoryError("vro_build_volume failed")
    return out


def noise_grid(kind, nx, ny, nz, freq, seed, origin=(0, 0, 0)):
    out = np.empty((nz, ny, nx), np.float32)
    mn, mx = ctypes.c_float(), ctypes.c_float()
    lib().vro_gen_uniform_grid3d(kind, out.ctypes.data_as(_vp), origin[0], origin[1], origin[2], nx, ny, nz,
                                 freq, seed, ctypes.byref(mn), ctypes.byref(mx))
    return out, mn.value, mx.value


def render(volume: np.ndarray, obj, glob, m: March, width, height, fmt=FMT_RGBA32F, band_rows=0,
           band_stride=1, band_first=0, threads=0):
    """Render with the CPU restatement -> (image (rows, width, 4), executed steps)."""
    vol = np.ascontiguousarray(volume, dtype=np.uint8)
    nz, ny, nx, _ = vol.shape
    if band_rows > 0:
        nb = (height + band_rows - 1) // band_rows
        rows = len(range(band_first, nb, band_stride)) * band_rows
    else:
        rows = height
    dt = np.float32 if fmt == FMT_RGBA32F else np.uint8
    out = np.zeros((rows, width, 4), dt)
    steps = ctypes.c_int64()
    obj = np.ascontiguousarray(obj, np.float32)
    glob = np.ascontiguousarray(glob, np.float32)
    rc = lib().vro_render(vol.ctypes.data_as(_vp), nx, ny, nz, obj.ctypes.data_as(_fp), glob.ctypes.data_as(_fp),
                          ctypes.byref(m), width, height, fmt, out.ctypes.data_as(_vp), out.strides[0],
                          band_rows, band_stride, band_first, ctypes.byref(steps), threads)
    if rc != 0:
        raise ValueError(f"vro_render failed ({rc})")
    return out, steps.value


def step_counts(obj, glob, m: March, width, height) -> np.ndarray:
    n = np.empty((height, width), np.int32)
    obj = np.ascontiguousarray(obj, np.float32)
    glob = np.ascontiguousarray(glob, np.float32)
    lib().vro_step_counts(obj.ctypes.data_as(_fp), glob.ctypes.data_as(_fp), ctypes.byref(m), width, height,
                          n.ctypes.data_as(_vp))
    return n


def sample(volume: np.ndarray, channel, p):
    vol = np.ascontiguousarray(volume, dtype=np.uint8)
    nz, ny, nx, _ = vol.shape
    return lib().vro_sample(vol.ctypes.data_as(_vp), nx, ny, nz, channel, float(p[0]), float(p[1]), float(p[2]))


def procedural_from(p) -> Procedural:
    """Copy a volumetricrenderer_amd Procedural (same layout), normalising
    sun_dir in double and rounding once, as vr_set_procedural does."""
    q = Procedural()
    ctypes.memmove(ctypes.byref(q), ctypes.byref(p), ctypes.sizeof(Procedural))
    if q.enabled and q.shadow_steps > 0:
        d = [float(v) for v in q.sun_dir]
        ln = math.sqrt(d[0] * d[0] + d[1] * d[1] + d[2] * d[2])
        q.sun_dir[:] = [float(np.float32(v / ln)) for v in d]
    return q


def render_procedural(p: Procedural, obj, glob, m: March, width, height, fmt=FMT_RGBA32F, band_rows=0,
                      band_stride=1, band_first=0, threads=0, with_evals=False, with_cells=False):
    """BASELINE configs 2/3 with the CPU restatement -> (image, executed steps)
    or, with_evals, (image, steps, density evaluations); with_cells appends the
    Worley cells the device's pruned evaluation computes (vr "count" = 2)."""
    if band_rows > 0:
        nb = (height + band_rows - 1) // band_rows
        rows = len(range(band_first, nb, band_stride)) * band_rows
    else:
        rows = height
    dt = np.float32 if fmt == FMT_RGBA32F else np.uint8
    out = np.zeros((rows, width, 4), dt)
    steps, evals, cells = ctypes.c_int64(), ctypes.c_int64(), ctypes.c_int64()
    obj = np.ascontiguousarray(obj, np.float32)
    glob = np.ascontiguousarray(glob, np.float32)
    rc = lib().vro_render_procedural(ctypes.byref(p), obj.ctypes.data_as(_fp), glob.ctypes.data_as(_fp),
                                     ctypes.byref(m), width, height, fmt, out.ctypes.data_as(_vp), out.strides[0],
                                     band_rows, band_stride, band_first, ctypes.byref(steps), ctypes.byref(evals),
                                     ctypes.byref(cells) if with_cells else None, threads)
    if rc != 0:
        raise ValueError(f"vro_render_procedural failed ({rc})")
    res = (out, steps.value) + ((evals.value,) if with_evals else ()) + ((cells.value,) if with_cells else ())
    return res
