"""Host-side interface of the ray-march path, over the C ABI (include/vr.h).

This mirrors the part of the reference interface that feeds shaders/frag.glsl:

==========================================  =====================================
reference (file:line)                       here
==========================================  =====================================
``vkc::Texture3D(data, extent)``            :meth:`Renderer.set_volume`
(VulkanTexture.h:55-60)
noise -> pixelData loops                    :meth:`Renderer.generate_volume`
(TestMain.cpp:43-92)
``UniformBuffer<T>::Update`` x2             :meth:`Renderer.set_shader_data`
(TestMain.cpp:248-249)
Model/View/Projection/W2L producer          :func:`reference_shader_data`
(TestMain.cpp:219-245)
frag.glsl constants (:29-32, :42, :63-69)   :func:`march_defaults`, :meth:`Renderer.set_march`
``EnqueueRenderPass("BasePass")`` + draw    :meth:`Renderer.render`
(TestMain.cpp:194-217)
==========================================  =====================================

torch is used only for device memory and streams.  All arithmetic runs in
libvr.so, and a missing library raises at import.  Errors are raised as
:class:`VRError`.  The reference throws from ``Error()`` instead (Utils.h:22-29).
"""
from __future__ import annotations

import ctypes

import numpy as np
import torch

from . import _lib
from ._lib import (BYTES_PER_PIXEL, CHANNELS, FLOAT_FORMATS, FMT_RGBA8_SRGB, FMT_RGBA8_UNORM, FMT_RGBA32F,  # noqa: F401
                   GREY_OF, GlobalShaderData, MarchParams, ObjectShaderData, Procedural, Target, VolumeRecipe, VRError,
                   call)

_lib.load()  # fail at import if the HIP library is missing


def _stream_handle(stream) -> ctypes.c_void_p:
    if stream is None:
        stream = torch.cuda.current_stream()
    if isinstance(stream, torch.cuda.Stream):
        return ctypes.c_void_p(stream.cuda_stream)
    return ctypes.c_void_p(int(stream))


def march_defaults(**overrides) -> MarchParams:
    """The reference's frag.glsl constants, with field overrides."""
    m = MarchParams()
    call("vr_march_defaults", ctypes.byref(m))
    for k, v in overrides.items():
        if isinstance(v, (list, tuple)):
            getattr(m, k)[:] = list(v)
        else:
            setattr(m, k, v)
    return m


def volume_recipe_defaults(**overrides) -> VolumeRecipe:
    """TestMain.cpp:51-62: N=128, freqs (.01,.03,.19,.15), seeds 1..4, literal."""
    r = VolumeRecipe()
    call("vr_volume_recipe_defaults", ctypes.byref(r))
    for k, v in overrides.items():
        if isinstance(v, (list, tuple)):
            getattr(r, k)[:] = list(v)
        else:
            setattr(r, k, v)
    return r


def procedural_defaults(**overrides) -> Procedural:
    """BASELINE config 2 medium (enabled=1); shadow_steps=8 gives config 3."""
    p = Procedural()
    call("vr_procedural_defaults", ctypes.byref(p))
    p.enabled = 1
    for k, v in overrides.items():
        if isinstance(v, (list, tuple)):
            getattr(p, k)[:] = list(v)
        else:
            setattr(p, k, v)
    return p


def scaled_recipe(size: int, literal: bool = True) -> VolumeRecipe:
    """Reference recipe at N = size, with frequencies scaled by 128/size so that
    the continuous field matches the 128^3 one (BASELINE config 5)."""
    r = volume_recipe_defaults(size=size, literal_overwrite=int(literal))
    s = 128.0 / size
    r.freq[:] = [float(np.float32(f) * np.float32(s)) for f in (0.01, 0.03, 0.19, 0.15)]
    return r


def reference_shader_data(aspect: float = 1280.0 / 720.0, phi_deg: float = 0.0, theta_deg: float = 0.0,
                          frame_time: float = 0.0):
    """TestMain.cpp:219-245 computed by libvr's host code (GLM semantics)."""
    osd, gsd = ObjectShaderData(), GlobalShaderData()
    call("vr_reference_shader_data", ctypes.c_float(aspect), ctypes.c_float(phi_deg),
         ctypes.c_float(theta_deg), ctypes.c_float(frame_time), ctypes.byref(osd), ctypes.byref(gsd))
    return osd, gsd


def band_rows_packed(height: int, band_rows: int, band_stride: int = 1, band_first: int = 0,
                     band_flip: int = 0) -> int:
    """Rows vr_render writes for a band set (vr_band_rows_packed); band_flip
    shifts the set's odd bands (vr.h vr_target.band_flip)."""
    n = _lib.load().vr_band_rows_packed(height, band_rows, band_stride, band_first, band_flip)
    if n < 0:
        raise ValueError(f"bad band set: rows {band_rows}, stride {band_stride}, flip {band_flip}")
    return n


def shader_data_arrays(osd: ObjectShaderData, gsd: GlobalShaderData):
    """(obj48, glob36) float32 arrays, the layout the oracle takes."""
    obj = np.ctypeslib.as_array(ctypes.cast(ctypes.byref(osd), ctypes.POINTER(ctypes.c_float)), (48,)).copy()
    glob = np.ctypeslib.as_array(ctypes.cast(ctypes.byref(gsd), ctypes.POINTER(ctypes.c_float)), (36,)).copy()
    return obj, glob


class Renderer:
    """Offscreen ray-march renderer on one HIP device (one per process/rank)."""

    def __init__(self, device: int = 0):
        self._ctx = ctypes.c_void_p()
        call("vr_create", int(device), ctypes.byref(self._ctx))
        self.device = int(device)
        self.march = march_defaults()

    # -- lifetime --------------------------------------------------------
    def close(self) -> None:
        if self._ctx:
            _lib.load().vr_destroy(self._ctx)
            self._ctx = ctypes.c_void_p()

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    def __del__(self):  # pragma: no cover - best effort
        try:
            self.close()
        except Exception:
            pass

    # -- volume (Texture3D) ------------------------------------------------
    def set_volume(self, rgba) -> None:
        """Upload an RGBA8 volume shaped (nz, ny, nx, 4), x fastest (TestMain.cpp:69-87)."""
        if isinstance(rgba, torch.Tensor) and rgba.is_cuda:
            return self.set_volume_device(rgba)
        a = np.ascontiguousarray(rgba, dtype=np.uint8)
        if a.ndim != 4 or a.shape[3] != 4:
            raise ValueError("volume must be shaped (nz, ny, nx, 4)")
        nz, ny, nx, _ = a.shape
        call("vr_set_volume", self._ctx, a.ctypes.data_as(ctypes.c_void_p), nx, ny, nz)

    def set_volume_device(self, t: torch.Tensor, stream=None) -> None:
        if t.dtype != torch.uint8 or t.dim() != 4 or t.shape[3] != 4 or not t.is_contiguous():
            raise ValueError("device volume must be a contiguous uint8 tensor (nz, ny, nx, 4)")
        nz, ny, nx, _ = t.shape
        h = _stream_handle(stream)
        call("vr_set_volume_device", self._ctx, ctypes.c_void_p(t.data_ptr()), nx, ny, nz, h)
        (stream if stream is not None else torch.cuda.current_stream()).synchronize()

    def generate_volume(self, recipe: VolumeRecipe | None = None) -> None:
        """Build the TestMain.cpp:43-92 volume on the GPU."""
        r = recipe if recipe is not None else volume_recipe_defaults()
        call("vr_generate_volume", self._ctx, ctypes.byref(r), _stream_handle(None))

    def get_volume(self) -> np.ndarray:
        nx, ny, nz = self.volume_dims()
        out = np.empty((nz, ny, nx, 4), np.uint8)
        call("vr_get_volume", self._ctx, out.ctypes.data_as(ctypes.c_void_p))
        return out

    def volume_dims(self):
        nx, ny, nz = ctypes.c_int(), ctypes.c_int(), ctypes.c_int()
        call("vr_volume_dims", self._ctx, ctypes.byref(nx), ctypes.byref(ny), ctypes.byref(nz))
        return nx.value, ny.value, nz.value

    def noise_grid(self, kind: int, nx: int, ny: int, nz: int, freq: float, seed: int,
                   origin=(0, 0, 0), out: torch.Tensor | None = None):
        """One GenUniformGrid3D on the GPU -> (tensor or None, min, max)."""
        mn, mx = ctypes.c_float(), ctypes.c_float()
        ptr = ctypes.c_void_p(out.data_ptr()) if out is not None else None
        call("vr_noise_grid", self._ctx, int(kind), ptr, origin[0], origin[1], origin[2], nx, ny, nz,
             ctypes.c_float(freq), int(seed), ctypes.byref(mn), ctypes.byref(mx), _stream_handle(None))
        return out, mn.value, mx.value

    # -- uniforms / constants ----------------------------------------------
    def set_shader_data(self, osd: ObjectShaderData, gsd: GlobalShaderData) -> None:
        call("vr_set_shader_data", self._ctx, ctypes.byref(osd), ctypes.byref(gsd))
        self.osd, self.gsd = osd, gsd

    def set_march(self, m: MarchParams | None = None, **overrides) -> None:
        m = m if m is not None else march_defaults(**overrides)
        call("vr_set_march", self._ctx, ctypes.byref(m))
        self.march = m

    def selftest(self, name: str) -> int:
        """Mismatch count of a device arithmetic shortcut (vr_selftest)."""
        n = ctypes.c_longlong()
        call("vr_selftest", self._ctx, name.encode(), ctypes.byref(n))
        return int(n.value)

    def set_procedural(self, p: Procedural | None = None, **overrides) -> None:
        """Enable the procedural medium (configs 2/3); pass enabled=0 to return to the volume."""
        p = p if p is not None else procedural_defaults(**overrides)
        call("vr_set_procedural", self._ctx, ctypes.byref(p))
        self.procedural = p

    def set_layout_preference(self, pref: int) -> None:
        call("vr_set_layout_preference", self._ctx, int(pref))

    def set_option(self, name: str, value: int) -> None:
        """Tuning knobs of vr_set_option: "layout", "schedule", "waves_per_simd"."""
        call("vr_set_option", self._ctx, name.encode(), int(value))

    def get_option(self, name: str) -> int:
        return _lib.load().vr_get_option(self._ctx, name.encode())

    @property
    def kernel_variant(self) -> str:
        return _lib.load().vr_kernel_variant(self._ctx).decode()

    def measure_copy_bandwidth(self, nbytes: int = 2 << 30, reps: int = 10, stream=None) -> tuple[float, float]:
        """(best, median) GB/s of the device's 16-B-per-lane streaming copy
        (read + written bytes): the measured HBM roofline (vr.h)."""
        best, med = ctypes.c_double(), ctypes.c_double()
        _lib.call("vr_measure_copy_bandwidth", self._ctx, nbytes, reps, _stream_handle(stream), ctypes.byref(best),
                  ctypes.byref(med))
        return best.value, med.value

    def measure_bandwidth(self, kind: str = "read", loads_per_lane: int = 0, nbytes: int = 2 << 30, reps: int = 10,
                          stream=None) -> tuple[float, float, int]:
        """(best, median GB/s, loads per lane of the best) of a one-pass 16-B-per-lane
        stream over `nbytes` (vr_measure_bandwidth): kind "read" (loads only, bytes
        read / time) or "copy" (read + written bytes / time); loads_per_lane 4, 8,
        16, or 0 = each of them."""
        k = {"copy": 0, "read": 1}[kind]
        best, med, pl = ctypes.c_double(), ctypes.c_double(), ctypes.c_int()
        _lib.call("vr_measure_bandwidth", self._ctx, k, int(loads_per_lane), nbytes, reps, _stream_handle(stream),
                  ctypes.byref(best), ctypes.byref(med), ctypes.byref(pl))
        return best.value, med.value, pl.value

    # -- the hot path ------------------------------------------------------
    def alloc_target(self, width: int, height: int, fmt: int = FMT_RGBA8_UNORM, band_rows: int = 0,
                     band_stride: int = 1, band_first: int = 0, band_flip: int = 0) -> torch.Tensor:
        """(rows, width, 4) for the RGBA formats, (rows, width) for the grey ones."""
        rows = band_rows_packed(height, band_rows, band_stride, band_first, band_flip)
        dev = torch.device("cuda", self.device)
        if fmt not in BYTES_PER_PIXEL:
            raise ValueError(f"unknown format {fmt}")
        shape = (rows, width, 4) if CHANNELS[fmt] == 4 else (rows, width)
        return torch.empty(shape, dtype=torch.float32 if fmt in FLOAT_FORMATS else torch.uint8, device=dev)

    def _check_target(self, width: int, height: int, fmt: int, out: torch.Tensor, band_rows: int,
                      band_stride: int, band_first: int, step_counter: torch.Tensor | None = None,
                      band_flip: int = 0) -> None:
        """The kernel writes band_rows_packed(...) rows of `width` pixels of
        BYTES_PER_PIXEL[fmt] bytes through a raw pointer: refuse any tensor it
        would write past, or that lives on another device."""
        if fmt not in BYTES_PER_PIXEL:
            raise ValueError(f"unknown format {fmt}")
        if not isinstance(out, torch.Tensor) or not out.is_cuda or out.device.index != self.device:
            raise ValueError(f"render target must be a tensor on cuda:{self.device}")
        want_dtype = torch.float32 if fmt in FLOAT_FORMATS else torch.uint8
        if out.dtype != want_dtype:
            raise ValueError(f"format {fmt} needs a {want_dtype} target, got {out.dtype}")
        rows = band_rows_packed(height, band_rows, band_stride, band_first, band_flip)
        if CHANNELS[fmt] == 4:
            if out.dim() != 3 or out.shape[0] < rows or out.shape[1] != width or out.shape[2] != 4:
                raise ValueError(f"render target must be shaped ({rows}, {width}, 4) (at least {rows} rows), "
                                 f"got {tuple(out.shape)}")
            if out.stride(2) != 1 or out.stride(1) != 4 or out.stride(0) < 4 * width:
                raise ValueError("render target rows must be contiguous RGBA pixels (strides (>=4*width, 4, 1))")
        else:
            if out.dim() != 2 or out.shape[0] < rows or out.shape[1] != width:
                raise ValueError(f"grey render target must be shaped ({rows}, {width}) (at least {rows} rows), "
                                 f"got {tuple(out.shape)}")
            if out.stride(1) != 1 or out.stride(0) < width:
                raise ValueError("grey render target rows must be contiguous (strides (>=width, 1))")
        if step_counter is not None and (step_counter.dtype != torch.int64 or not step_counter.is_cuda
                                         or step_counter.device.index != self.device
                                         or step_counter.numel() < 1):
            raise ValueError(f"step_counter must be an int64 tensor on cuda:{self.device}")

    def render(self, width: int, height: int, fmt: int = FMT_RGBA8_UNORM, out: torch.Tensor | None = None,
               band_rows: int = 0, band_stride: int = 1, band_first: int = 0, stream=None,
               step_counter: torch.Tensor | None = None, band_flip: int = 0) -> torch.Tensor:
        """Launch the march kernel (asynchronous on `stream`); returns `out`.
        band_flip: the set's odd bands shifted (vr.h vr_target.band_flip)."""
        if out is None:
            out = self.alloc_target(width, height, fmt, band_rows, band_stride, band_first, band_flip)
        self._check_target(width, height, fmt, out, band_rows, band_stride, band_first, step_counter, band_flip)
        t = Target(width=width, height=height, format=fmt, band_rows=band_rows, band_stride=band_stride,
                   band_first=band_first, pixels=out.data_ptr(), row_pitch=out.stride(0) * out.element_size(),
                   step_counter=step_counter.data_ptr() if step_counter is not None else None,
                   band_flip=band_flip)
        call("vr_render", self._ctx, ctypes.byref(t), _stream_handle(stream))
        return out

    def render_rows(self, width: int, height: int, fmt: int, first_row: int, rows: int,
                    out: torch.Tensor | None = None, in_place: bool = False, stream=None) -> torch.Tensor:
        """Frame rows [first_row, first_row + rows) of the width x height frame
        (vr.h VR_TARGET_ROW_RANGE; first_row a multiple of 8): packed from row
        0 of `out`, or at their own rows of a whole-frame `out` (in_place)."""
        n = max(0, min(rows, height - first_row))
        if out is None:
            out = self.alloc_target(width, height if in_place else n, fmt)
        self._check_target(width, height if in_place else n, fmt, out, 0, 1, 0)
        flags = _lib.TARGET_ROW_RANGE | (_lib.TARGET_BANDS_IN_PLACE if in_place else 0)
        t = Target(width=width, height=height, format=fmt | flags, band_rows=rows, band_stride=1,
                   band_first=first_row, pixels=out.data_ptr(), row_pitch=out.stride(0) * out.element_size(),
                   step_counter=None)
        call("vr_render", self._ctx, ctypes.byref(t), _stream_handle(stream))
        return out

    def row_partition(self, width: int, height: int, parts: int) -> list[int]:
        """vr_row_partition: parts + 1 row starts of contiguous ranges of equal
        estimated march work for the current camera."""
        rb = (ctypes.c_int * (parts + 1))()
        call("vr_row_partition", self._ctx, width, height, parts, rb)
        return list(rb)

    def row_work(self, width: int, height: int) -> list[float]:
        """The estimated march work of every 8-row strip (vr_row_work: the
        model vr_row_partition splits and vr_shard_balance_lead sizes rank 0's
        lead rows from)."""
        ns = (height + 7) // 8
        out = (ctypes.c_double * ns)()
        call("vr_row_work", self._ctx, width, height, out, ns)
        return list(out)

    def row_partition_measured(self, width: int, height: int, prev: list[int], prev_ms: list[float]) -> list[int]:
        """vr_row_partition_measured: the split again, range k of `prev` having
        taken prev_ms[k]."""
        parts = len(prev) - 1
        rb = (ctypes.c_int * (parts + 1))()
        call("vr_row_partition_measured", self._ctx, width, height, parts, (ctypes.c_int * (parts + 1))(*prev),
             (ctypes.c_double * parts)(*prev_ms), rb)
        return list(rb)

    def render_sequence(self, width: int, height: int, fmt: int, out: torch.Tensor, cameras, band_rows: int = 0,
                        band_stride: int = 1, band_first: int = 0, stream=None) -> torch.Tensor:
        """The reference's frame loop with a moving camera (TestMain.cpp:173-256):
        one render per (ObjectShaderData, GlobalShaderData) of `cameras`, all
        into `out`, queued natively (vr_render_sequence) without host waits."""
        self._check_target(width, height, fmt, out, band_rows, band_stride, band_first)
        cams = list(cameras)
        osd = (ObjectShaderData * max(1, len(cams)))(*[c[0] for c in cams])
        gsd = (GlobalShaderData * max(1, len(cams)))(*[c[1] for c in cams])
        t = Target(width=width, height=height, format=fmt, band_rows=band_rows, band_stride=band_stride,
                   band_first=band_first, pixels=out.data_ptr(), row_pitch=out.stride(0) * out.element_size(),
                   step_counter=None)
        call("vr_render_sequence", self._ctx, ctypes.byref(t), len(cams), osd, gsd, _stream_handle(stream))
        return out

    def prepare_render(self, width: int, height: int, fmt: int, out: torch.Tensor, band_rows: int = 0,
                       band_stride: int = 1, band_first: int = 0, stream=None):
        """A zero-argument launcher for one fixed render (target, bands,
        stream): the ctypes arguments are built once, so a frame loop pays
        only the call (host time per frame bounds multi-GPU strong scaling)."""
        self._check_target(width, height, fmt, out, band_rows, band_stride, band_first)
        t = Target(width=width, height=height, format=fmt, band_rows=band_rows, band_stride=band_stride,
                   band_first=band_first, pixels=out.data_ptr(), row_pitch=out.stride(0) * out.element_size(),
                   step_counter=None)
        fn, ctx, tref, sh = _lib.load().vr_render, self._ctx, ctypes.byref(t), _stream_handle(stream)

        def launch():
            st = fn(ctx, tref, sh)
            if st:
                _lib.check(st, "vr_render")
        launch.target = t   # keep the struct and the target tensor alive with the closure
        launch.out = out
        return launch

    def prepare_assemble(self, gathered: torch.Tensor, nranks: int, width: int, height: int, band_rows: int,
                         frame: torch.Tensor, stream=None):
        """Zero-argument launcher for one fixed vr_assemble_bands call."""
        self._check_assemble(gathered, nranks, width, height, band_rows, frame)
        bpp = gathered.element_size() * gathered.shape[-1]
        args = (self._ctx, ctypes.c_void_p(gathered.data_ptr()), gathered.shape[1], nranks, width, height, band_rows,
                bpp, ctypes.c_void_p(frame.data_ptr()), _stream_handle(stream))
        fn = _lib.load().vr_assemble_bands

        def launch():
            st = fn(*args)
            if st:
                _lib.check(st, "vr_assemble_bands")
        launch.keep = (gathered, frame)
        return launch

    def _check_assemble_frame(self, gathered: torch.Tensor, gfmt: int, nranks: int, width: int, height: int,
                              frame: torch.Tensor, ffmt: int) -> None:
        for name, t in (("gathered", gathered), ("frame", frame)):
            if not t.is_cuda or t.device.index != self.device or not t.is_contiguous():
                raise ValueError(f"{name} must be a contiguous tensor on cuda:{self.device}")
        if gfmt != ffmt and GREY_OF.get(ffmt) != gfmt:
            raise ValueError(f"band sets in format {gfmt} do not expand into format {ffmt}")
        gshape = (width, 4) if CHANNELS[gfmt] == 4 else (width,)
        gdtype = torch.float32 if gfmt in FLOAT_FORMATS else torch.uint8
        if gathered.dim() != 2 + len(gshape) or gathered.shape[0] < nranks or tuple(gathered.shape[2:]) != gshape \
                or gathered.dtype != gdtype:
            raise ValueError(f"gathered must be a {gdtype} tensor shaped (>= {nranks}, rows, {gshape}), "
                             f"got {gathered.dtype} {tuple(gathered.shape)}")
        fdtype = torch.float32 if ffmt in FLOAT_FORMATS else torch.uint8
        fshape = (height, width, 4) if CHANNELS[ffmt] == 4 else (height, width)
        if frame.dtype != fdtype or tuple(frame.shape) != fshape:
            raise ValueError(f"frame must be a {fdtype} tensor shaped {fshape}")

    def assemble_frame(self, gathered: torch.Tensor, gathered_fmt: int, nranks: int, width: int, height: int,
                       band_rows: int, frame_fmt: int, frame: torch.Tensor | None = None, stream=None,
                       serpentine: bool = False) -> torch.Tensor:
        """vr_assemble_frame: [rank][packed rows] band sets in `gathered_fmt`
        (e.g. grey) scattered and expanded into a `frame_fmt` frame.
        serpentine: rank r rendered with band_flip nranks-1-2r
        (VR_ASSEMBLE_SERPENTINE)."""
        if frame is None:
            shape = (height, width, 4) if CHANNELS[frame_fmt] == 4 else (height, width)
            frame = torch.empty(shape, dtype=torch.float32 if frame_fmt in FLOAT_FORMATS else torch.uint8,
                                device=gathered.device)
        self._check_assemble_frame(gathered, gathered_fmt, nranks, width, height, frame, frame_fmt)
        call("vr_assemble_frame", self._ctx, ctypes.c_void_p(gathered.data_ptr()), gathered_fmt, gathered.shape[1],
             nranks, width, height, band_rows, frame_fmt | (_lib.ASSEMBLE_SERPENTINE if serpentine else 0),
             ctypes.c_void_p(frame.data_ptr()), _stream_handle(stream))
        return frame

    def prepare_assemble_frame(self, gathered: torch.Tensor, gathered_fmt: int, nranks: int, width: int, height: int,
                               band_rows: int, frame_fmt: int, frame: torch.Tensor, stream=None):
        """Zero-argument launcher for one fixed vr_assemble_frame call."""
        self._check_assemble_frame(gathered, gathered_fmt, nranks, width, height, frame, frame_fmt)
        args = (self._ctx, ctypes.c_void_p(gathered.data_ptr()), gathered_fmt, gathered.shape[1], nranks, width,
                height, band_rows, frame_fmt, ctypes.c_void_p(frame.data_ptr()), _stream_handle(stream))
        fn = _lib.load().vr_assemble_frame

        def launch():
            st = fn(*args)
            if st:
                _lib.check(st, "vr_assemble_frame")
        launch.keep = (gathered, frame)
        return launch

    def _check_assemble(self, gathered: torch.Tensor, nranks: int, width: int, height: int, band_rows: int,
                        frame: torch.Tensor) -> None:
        for name, t in (("gathered", gathered), ("frame", frame)):
            if not t.is_cuda or t.device.index != self.device or not t.is_contiguous():
                raise ValueError(f"{name} must be a contiguous tensor on cuda:{self.device}")
        if gathered.dim() != 4 or gathered.shape[0] < nranks or gathered.shape[2] != width or gathered.shape[3] != 4:
            raise ValueError(f"gathered must be shaped (>= {nranks}, rows, {width}, 4), got {tuple(gathered.shape)}")
        if frame.dtype != gathered.dtype or tuple(frame.shape) != (height, width, 4):
            raise ValueError(f"frame must be a {gathered.dtype} tensor shaped ({height}, {width}, 4)")

    def assemble_bands(self, gathered: torch.Tensor, nranks: int, width: int, height: int, band_rows: int,
                       frame: torch.Tensor | None = None, stream=None) -> torch.Tensor:
        """Scatter [rank][packed rows] band sets into one frame (SURVEY.md e)."""
        bpp = gathered.element_size() * gathered.shape[-1]
        rows_per_rank = gathered.shape[1]
        if frame is None:
            frame = torch.empty((height, width, gathered.shape[-1]), dtype=gathered.dtype, device=gathered.device)
        self._check_assemble(gathered, nranks, width, height, band_rows, frame)
        call("vr_assemble_bands", self._ctx, ctypes.c_void_p(gathered.data_ptr()), rows_per_rank, nranks,
             width, height, band_rows, bpp, ctypes.c_void_p(frame.data_ptr()), _stream_handle(stream))
        return frame
