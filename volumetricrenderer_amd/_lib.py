"""ctypes binding of libvr.so, the C ABI of include/vr.h.

This module is plumbing: it declares the C structs and function signatures and
raises :class:`VRError` on a non-zero status.  The product code is the HIP
library.  If ``libvr.so`` is missing, ``load()`` raises immediately.  There is
no CPU fallback.

torch is imported before the library is opened.  torch ships its own
``libamdhip64.so`` with soname ``libamdhip64.so.7``.  Opening it first makes
libvr.so bind to that runtime instead of loading a second copy from
/opt/rocm/lib.
"""
from __future__ import annotations

import ctypes
import os

try:  # noqa: SIM105 - load order matters, see module docstring
    import torch  # noqa: F401
except ImportError:  # pragma: no cover - torch is always present in this image
    torch = None

HERE = os.path.dirname(os.path.abspath(__file__))
# VR_LIB overrides the library path (timing experiments with variant builds)
LIB_PATH = os.environ.get("VR_LIB") or os.path.join(HERE, "libvr.so")

VR_OK = 0
STATUS_NAMES = {
    0: "VR_OK", 1: "VR_ERR_INVALID", 2: "VR_ERR_HIP", 3: "VR_ERR_NO_VOLUME",
    4: "VR_ERR_NO_CAMERA", 5: "VR_ERR_OOM", 6: "VR_ERR_NO_DEVICE",
    7: "VR_ERR_TIMEOUT", 8: "VR_ERR_COMM",
}
FMT_RGBA32F, FMT_RGBA8_UNORM, FMT_RGBA8_SRGB = 0, 1, 2
# grey targets (include/vr.h): the R channel of the RGBA format, 1 value per pixel
FMT_R8_UNORM, FMT_R8_SRGB, FMT_R32F = 3, 4, 5
BYTES_PER_PIXEL = {FMT_RGBA32F: 16, FMT_RGBA8_UNORM: 4, FMT_RGBA8_SRGB: 4, FMT_R8_UNORM: 1, FMT_R8_SRGB: 1,
                   FMT_R32F: 4}
CHANNELS = {FMT_RGBA32F: 4, FMT_RGBA8_UNORM: 4, FMT_RGBA8_SRGB: 4, FMT_R8_UNORM: 1, FMT_R8_SRGB: 1, FMT_R32F: 1}
GREY_OF = {FMT_RGBA32F: FMT_R32F, FMT_RGBA8_UNORM: FMT_R8_UNORM, FMT_RGBA8_SRGB: FMT_R8_SRGB}
FLOAT_FORMATS = (FMT_RGBA32F, FMT_R32F)
# OR'ed into a target's format: bands written at their frame rows (include/vr.h)
TARGET_BANDS_IN_PLACE = 0x100
TARGET_ROW_RANGE = 0x200   # vr.h VR_TARGET_ROW_RANGE
ASSEMBLE_SERPENTINE = 0x400   # vr.h: OR'ed into vr_assemble_frame's frame format

c_float_p = ctypes.POINTER(ctypes.c_float)
c_int_p = ctypes.POINTER(ctypes.c_int)


class VRError(RuntimeError):
    """A libvr call returned a non-zero vr_status."""

    def __init__(self, status: int, func: str, msg: str):
        self.status = status
        super().__init__(f"{func} -> {STATUS_NAMES.get(status, status)}: {msg}")


class ObjectShaderData(ctypes.Structure):
    """binding 0 UBO, TestMain.cpp:27-32 / vert.glsl:4-9 (column-major)."""
    _fields_ = [("model", ctypes.c_float * 16), ("view", ctypes.c_float * 16),
                ("projection", ctypes.c_float * 16)]


class GlobalShaderData(ctypes.Structure):
    """binding 1 UBO, TestMain.cpp:34-39 / frag.glsl:9-14, std140 (144 B)."""
    _fields_ = [("world_to_local", ctypes.c_float * 16), ("camera_position", ctypes.c_float * 3),
                ("_pad0", ctypes.c_float), ("media_scroll", ctypes.c_float * 16)]


class MarchParams(ctypes.Structure):
    """frag.glsl:29-32, 42, 63-69 constants (vr_march_params)."""
    _fields_ = [("max_steps", ctypes.c_int32), ("step_scale", ctypes.c_float),
                ("density", ctypes.c_float), ("scale", ctypes.c_float),
                ("box_min", ctypes.c_float * 3), ("box_max", ctypes.c_float * 3),
                ("tap_scale", ctypes.c_float * 4), ("tap_weight", ctypes.c_float * 4),
                ("early_out", ctypes.c_float), ("reserved", ctypes.c_int32 * 3)]


class VolumeRecipe(ctypes.Structure):
    """TestMain.cpp:43-92 volume recipe (vr_volume_recipe)."""
    _fields_ = [("size", ctypes.c_int32), ("freq", ctypes.c_float * 4),
                ("seed", ctypes.c_int32 * 4), ("literal_overwrite", ctypes.c_int32)]


class Procedural(ctypes.Structure):
    """vr_procedural: BASELINE configs 2/3 (build-defined procedural medium)."""
    _fields_ = [("enabled", ctypes.c_int32), ("grid_scale", ctypes.c_float), ("octaves", ctypes.c_int32),
                ("freq0", ctypes.c_float), ("lacunarity", ctypes.c_float), ("gain", ctypes.c_float),
                ("seed_fbm", ctypes.c_int32), ("worley_freq", ctypes.c_float), ("seed_worley", ctypes.c_int32),
                ("shadow_steps", ctypes.c_int32), ("sun_dir", ctypes.c_float * 3), ("reserved", ctypes.c_int32)]


class Target(ctypes.Structure):
    """vr_target: device render target + band selection."""
    _fields_ = [("width", ctypes.c_int32), ("height", ctypes.c_int32), ("format", ctypes.c_int32),
                ("band_rows", ctypes.c_int32), ("band_stride", ctypes.c_int32),
                ("band_first", ctypes.c_int32), ("pixels", ctypes.c_void_p),
                ("row_pitch", ctypes.c_size_t), ("step_counter", ctypes.c_void_p),
                ("band_flip", ctypes.c_int32), ("reserved", ctypes.c_int32)]


_vp = ctypes.c_void_p
_SIGS = {
    "vr_create": (ctypes.c_int, [ctypes.c_int, ctypes.POINTER(_vp)]),
    "vr_destroy": (ctypes.c_int, [_vp]),
    "vr_last_error": (ctypes.c_char_p, []),
    "vr_abi_version": (ctypes.c_int, []),
    "vr_build_id": (ctypes.c_char_p, []),
    "vr_set_volume": (ctypes.c_int, [_vp, _vp, ctypes.c_int, ctypes.c_int, ctypes.c_int]),
    "vr_set_volume_device": (ctypes.c_int, [_vp, _vp, ctypes.c_int, ctypes.c_int, ctypes.c_int, _vp]),
    "vr_get_volume": (ctypes.c_int, [_vp, _vp]),
    "vr_volume_dims": (ctypes.c_int, [_vp, c_int_p, c_int_p, c_int_p]),
    "vr_volume_extent_ok": (ctypes.c_int, [ctypes.c_int, ctypes.c_int, ctypes.c_int]),
    "vr_volume_recipe_defaults": (ctypes.c_int, [ctypes.POINTER(VolumeRecipe)]),
    "vr_generate_volume": (ctypes.c_int, [_vp, ctypes.POINTER(VolumeRecipe), _vp]),
    "vr_noise_grid": (ctypes.c_int, [_vp, ctypes.c_int, _vp, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                     ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_float,
                                     ctypes.c_int32, c_float_p, c_float_p, _vp]),
    "vr_set_shader_data": (ctypes.c_int, [_vp, ctypes.POINTER(ObjectShaderData),
                                          ctypes.POINTER(GlobalShaderData)]),
    "vr_reference_shader_data": (ctypes.c_int, [ctypes.c_float, ctypes.c_float, ctypes.c_float,
                                                ctypes.c_float, ctypes.POINTER(ObjectShaderData),
                                                ctypes.POINTER(GlobalShaderData)]),
    "vr_march_defaults": (ctypes.c_int, [ctypes.POINTER(MarchParams)]),
    "vr_selftest": (ctypes.c_int, [_vp, ctypes.c_char_p, ctypes.POINTER(ctypes.c_longlong)]),
    "vr_procedural_defaults": (ctypes.c_int, [ctypes.POINTER(Procedural)]),
    "vr_set_procedural": (ctypes.c_int, [_vp, ctypes.POINTER(Procedural)]),
    "vr_set_march": (ctypes.c_int, [_vp, ctypes.POINTER(MarchParams)]),
    "vr_render": (ctypes.c_int, [_vp, ctypes.POINTER(Target), _vp]),
    "vr_render_sequence": (ctypes.c_int, [_vp, ctypes.POINTER(Target), ctypes.c_int, ctypes.POINTER(ObjectShaderData),
                                          ctypes.POINTER(GlobalShaderData), _vp]),
    "vr_assemble_bands": (ctypes.c_int, [_vp, _vp, ctypes.c_size_t, ctypes.c_int, ctypes.c_int,
                                         ctypes.c_int, ctypes.c_int, ctypes.c_int, _vp, _vp]),
    "vr_assemble_frame": (ctypes.c_int, [_vp, _vp, ctypes.c_int, ctypes.c_size_t, ctypes.c_int, ctypes.c_int,
                                         ctypes.c_int, ctypes.c_int, ctypes.c_int, _vp, _vp]),
    "vr_assemble_frame_ranks": (ctypes.c_int, [_vp, _vp, ctypes.c_int, ctypes.c_size_t, ctypes.c_int, ctypes.c_int,
                                               ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int, _vp, _vp]),
    "vr_band_rows_packed": (ctypes.c_int, [ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int]),
    "vr_row_partition": (ctypes.c_int, [_vp, ctypes.c_int, ctypes.c_int, ctypes.c_int, c_int_p]),
    "vr_row_work": (ctypes.c_int, [_vp, ctypes.c_int, ctypes.c_int, ctypes.POINTER(ctypes.c_double), ctypes.c_int]),
    "vr_row_partition_measured": (ctypes.c_int, [_vp, ctypes.c_int, ctypes.c_int, ctypes.c_int, c_int_p,
                                                 ctypes.POINTER(ctypes.c_double), c_int_p]),
    "vr_kernel_variant": (ctypes.c_char_p, [_vp]),
    "vr_set_layout_preference": (ctypes.c_int, [_vp, ctypes.c_int]),
    "vr_set_option": (ctypes.c_int, [_vp, ctypes.c_char_p, ctypes.c_int]),
    "vr_get_option": (ctypes.c_int, [_vp, ctypes.c_char_p]),
    "vr_measure_copy_bandwidth": (ctypes.c_int, [_vp, ctypes.c_size_t, ctypes.c_int, _vp,
                                                 ctypes.POINTER(ctypes.c_double), ctypes.POINTER(ctypes.c_double)]),
    "vr_measure_bandwidth": (ctypes.c_int, [_vp, ctypes.c_int, ctypes.c_int, ctypes.c_size_t, ctypes.c_int, _vp,
                                            ctypes.POINTER(ctypes.c_double), ctypes.POINTER(ctypes.c_double),
                                            ctypes.POINTER(ctypes.c_int)]),
}
# functions whose int return is a value, not a vr_status
_VALUE_RETURNS = {"vr_abi_version", "vr_band_rows_packed", "vr_get_option", "vr_volume_extent_ok"}

_lib = None


def load(path: str | None = None) -> ctypes.CDLL:
    """Open libvr.so and declare its signatures.  Fails loudly if absent."""
    global _lib
    if _lib is not None and path is None:
        return _lib
    p = path or LIB_PATH
    if not os.path.exists(p):
        raise ImportError(f"libvr.so not built: {p} is missing (run __graft_entry__.build() "
                          "or `make -C volumetricrenderer_amd/csrc`)")
    lib = ctypes.CDLL(p)
    for name, (res, args) in _SIGS.items():
        if os.environ.get("VR_LIB") and not hasattr(lib, name):
            continue   # an older build for a timing A/B (VR_LIB) may lack newer entry points
        f = getattr(lib, name)
        f.restype = res
        f.argtypes = args
    if path is None:
        _lib = lib
    return lib


def exported_symbols() -> list[str]:
    return sorted(_SIGS)


def check(status: int, func: str) -> None:
    if status != VR_OK:
        msg = load().vr_last_error()
        raise VRError(status, func, msg.decode(errors="replace") if msg else "")


def call(name: str, *args):
    """Call a vr_* function, raising VRError on a non-zero status."""
    f = getattr(load(), name)
    r = f(*args)
    if name in _VALUE_RETURNS or f.restype is not ctypes.c_int:
        return r
    check(r, name)
    return r


# ---- libvr_shard.so: the multi-GPU frame pipeline (include/vr_shard.h) ----
SHARD_LIB_PATH = os.environ.get("VR_SHARD_LIB") or os.path.join(HERE, "libvr_shard.so")
SHARD_ID_BYTES = 128
_SHARD_SIGS = {
    "vr_shard_last_error": (ctypes.c_char_p, []),
    "vr_shard_build_id": (ctypes.c_char_p, []),
    "vr_shard_unique_id": (ctypes.c_int, [_vp]),
    "vr_shard_create": (ctypes.c_int, [_vp, _vp, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                       ctypes.c_int, ctypes.c_int, ctypes.POINTER(_vp)]),
    "vr_shard_alloc": (ctypes.c_int, [_vp, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                      ctypes.c_int, ctypes.c_int, ctypes.POINTER(_vp)]),
    "vr_shard_connect": (ctypes.c_int, [_vp, _vp]),
    "vr_shard_destroy": (ctypes.c_int, [_vp]),
    "vr_shard_run": (ctypes.c_int, [_vp, ctypes.c_int, _vp, ctypes.c_int, c_float_p]),
    "vr_shard_run_frames": (ctypes.c_int, [_vp, ctypes.c_int, ctypes.POINTER(ObjectShaderData),
                                           ctypes.POINTER(GlobalShaderData), _vp, ctypes.c_int, c_float_p,
                                           ctypes.POINTER(ctypes.c_double)]),
    "vr_shard_frame": (ctypes.c_int, [_vp, ctypes.POINTER(_vp), ctypes.POINTER(ctypes.c_size_t), c_int_p]),
    "vr_shard_copy_frame": (ctypes.c_int, [_vp, _vp, ctypes.c_size_t, _vp]),
    "vr_shard_rows": (ctypes.c_int, [_vp, c_int_p, c_int_p]),
    "vr_shard_barrier": (ctypes.c_int, [_vp, _vp]),
    "vr_shard_share_volume": (ctypes.c_int, [_vp, _vp, ctypes.c_int, ctypes.c_int, ctypes.c_int, _vp]),
    "vr_shard_set_timeout": (ctypes.c_int, [_vp, ctypes.c_double]),
    "vr_shard_aborted": (ctypes.c_int, [_vp]),
    "vr_shard_sampled_busy": (ctypes.c_int, [_vp, ctypes.POINTER(ctypes.c_double), ctypes.POINTER(ctypes.c_double)]),
    "vr_shard_set_lead_rows": (ctypes.c_int, [_vp, ctypes.c_int]),
    "vr_shard_get_lead_rows": (ctypes.c_int, [_vp]),
    "vr_shard_balance_lead": (ctypes.c_int, [_vp, ctypes.c_int]),
    "vr_shard_set_render_streams": (ctypes.c_int, [_vp, ctypes.c_int]),
    "vr_shard_get_render_streams": (ctypes.c_int, [_vp]),
    "vr_shard_set_solo": (ctypes.c_int, [_vp, ctypes.c_int]),
    "vr_shard_set_host_threads": (ctypes.c_int, [_vp, ctypes.c_int]),
    "vr_shard_set_exchange_streams": (ctypes.c_int, [_vp, ctypes.c_int]),
    "vr_shard_set_compositor": (ctypes.c_int, [_vp, ctypes.c_int]),
    "vr_shard_get_compositor": (ctypes.c_int, [_vp]),
    "vr_shard_bands": (ctypes.c_int, [_vp, c_int_p, c_int_p, c_int_p]),
    "vr_shard_set_serpentine": (ctypes.c_int, [_vp, ctypes.c_int]),
    "vr_shard_get_serpentine": (ctypes.c_int, [_vp]),
    "vr_shard_set_rows": (ctypes.c_int, [_vp, c_int_p]),
    "vr_shard_balance_rows": (ctypes.c_int, [_vp]),
    "vr_shard_rebalance_rows": (ctypes.c_int, [_vp, ctypes.c_double]),
    "vr_shard_partition": (ctypes.c_int, [_vp]),
    "vr_shard_row_range": (ctypes.c_int, [_vp, ctypes.c_int, c_int_p, c_int_p]),
    "vr_shard_poll_selftest": (ctypes.c_int, [ctypes.c_int, ctypes.c_double, c_int_p]),
}
# shard functions whose int return is a value, not a vr_status
_SHARD_VALUE_RETURNS = {"vr_shard_aborted", "vr_shard_poll_selftest", "vr_shard_get_render_streams",
                        "vr_shard_get_compositor", "vr_shard_partition", "vr_shard_get_lead_rows",
                        "vr_shard_get_serpentine"}
_shard_lib = None


def load_shard() -> ctypes.CDLL:
    """Open libvr_shard.so (libvr + RCCL).  Only the multi-GPU path loads it,
    so single-GPU users never map RCCL.  Fails loudly if absent."""
    global _shard_lib
    if _shard_lib is not None:
        return _shard_lib
    load()   # libvr first: libvr_shard binds to the same copy
    if not os.path.exists(SHARD_LIB_PATH):
        raise ImportError(f"libvr_shard.so not built: {SHARD_LIB_PATH} is missing (run __graft_entry__.build())")
    lib = ctypes.CDLL(SHARD_LIB_PATH)
    for name, (res, args) in _SHARD_SIGS.items():
        f = getattr(lib, name)
        f.restype = res
        f.argtypes = args
    _shard_lib = lib
    return lib


def shard_exported_symbols() -> list[str]:
    return sorted(_SHARD_SIGS)


def shard_call(name: str, *args):
    """Call a vr_shard_* function, raising VRError on a non-zero status."""
    lib = load_shard()
    r = getattr(lib, name)(*args)
    if name in _SHARD_VALUE_RETURNS:
        return r
    if r != VR_OK:
        msg = lib.vr_shard_last_error()
        raise VRError(r, name, msg.decode(errors="replace") if msg else "")
    return r
