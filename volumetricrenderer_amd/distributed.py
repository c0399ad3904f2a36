"""Multi-GPU frame sharding: interleaved screen bands + gather to rank 0.

SURVEY.md sec. 8e.  Pixels are independent: a1-a6 read only the uniforms and
a read-only volume.  So a frame shards by screen rows and the volume is
replicated on every rank.  The silhouette of the reference cube is a centred
hexagon, so contiguous strips are badly imbalanced (2.45x at 8 ranks).
Interleaved 16-row bands, where band b goes to rank b mod N, are balanced to
within 1-2 %.  The only exchange is one gather per frame.  Each rank's packed
band set goes to rank 0, over RCCL (torch.distributed "nccl") on GPUs or gloo
in the CPU tests.  Rank 0 then scatters the sets into the frame with
vr_assemble_frame.  The sets travel in the frame format's grey form (one value
per pixel: the shader writes vec4(vec3(c), 1), frag.glsl:79-80), a quarter of
the RGBA bytes; the assembly expands them.

One process per GPU; the reference has no distributed code at all.
"""
from __future__ import annotations

import ctypes

import numpy as np
import torch
import torch.distributed as dist

from . import _lib


def rows_for_rank(height: int, band_rows: int, world: int, rank: int) -> int:
    nb = (height + band_rows - 1) // band_rows
    return len(range(rank, nb, world)) * band_rows


def share_volume(renderer, vol=None, rank: int | None = None, group=None):
    """Collective (collective 1): rank 0's RGBA8 volume
    (nz, ny, nx, 4; numpy or tensor, ignored elsewhere) reaches every rank of
    the torch.distributed group once, and each rank's `renderer` installs it
    (``set_volume``).  The shape goes first, so the other ranks need nothing
    but the call.  Over gloo the bytes travel as a CPU tensor, over nccl
    (RCCL) as a device tensor.  Returns the volume as this rank received it.

    `rank` defaults to this process's rank in `group`.  A bad volume on rank 0
    is announced with a shape of -1s, so every rank raises together instead of
    the others waiting in the broadcast."""
    world = dist.get_world_size(group)
    if rank is None:
        rank = dist.get_rank(group)
    dev = "cuda" if dist.get_backend(group) == "nccl" else "cpu"
    shape = torch.full((4,), -1, dtype=torch.int64, device=dev)
    bad = None
    if rank == 0:
        if vol is None:
            bad = "share_volume: rank 0 needs the volume"
        else:
            t = vol if isinstance(vol, torch.Tensor) else torch.from_numpy(np.ascontiguousarray(vol, dtype=np.uint8))
            if t.dtype != torch.uint8 or t.dim() != 4 or t.shape[3] != 4 or min(t.shape) <= 0:
                bad = "share_volume: the volume must be uint8 shaped (nz, ny, nx, 4)"
            else:
                shape.copy_(torch.tensor(list(t.shape), dtype=torch.int64))
    if world > 1:
        dist.broadcast(shape, src=0, group=group)
    dims = [int(v) for v in shape.tolist()]
    if bad or min(dims) <= 0:
        raise ValueError(bad or "share_volume: rank 0 had no valid volume")
    if rank == 0:
        data = t.to(dev).contiguous()
    else:
        data = torch.empty(dims, dtype=torch.uint8, device=dev)
    if world > 1:
        dist.broadcast(data, src=0, group=group)
    renderer.set_volume(data if data.is_cuda else data.numpy())
    return data


class BandSharder:
    """Renders this rank's bands of a W x H frame and gathers them on rank 0.

    `renderer` provides ``alloc_target``, ``render`` and ``assemble_frame``
    (or only ``assemble_bands``: then the band sets keep the frame format).
    That is :class:`volumetricrenderer_amd.Renderer`, or a CPU stand-in in
    the gloo tests.  With several ranks the band sets are grey
    (``GREY_OF[fmt]``); :meth:`frame` returns rank 0's RGBA frame and the
    other ranks' grey band sets.
    """

    def __init__(self, renderer, width: int, height: int, fmt: int, band_rows: int = 16, world: int = 1,
                 rank: int = 0, group=None, inflight: int = 1):
        self.r = renderer
        self.inflight = inflight   # world 1, grid medium: 2 = frames alternate two streams (run_frames)
        self.width, self.height, self.fmt = width, height, fmt
        self.world, self.rank, self.group = world, rank, group
        self.band_rows = band_rows if world > 1 else 0
        grey = world > 1 and hasattr(renderer, "assemble_frame") and fmt in _lib.GREY_OF
        self.gfmt = _lib.GREY_OF[fmt] if grey else fmt   # format of the band sets (exchanged)
        if world > 1:
            self.my_rows = rows_for_rank(height, band_rows, world, rank)
            # every rank's buffer has rank 0's row count (the most rows), so
            # the gather moves equal-sized messages
            self.rows_per_rank = rows_for_rank(height, band_rows, world, 0)
            buf = renderer.alloc_target(width, height, self.gfmt, band_rows, world, 0)
            assert buf.shape[0] == self.rows_per_rank
            self.local = buf
            if rank == 0:
                self.gathered = torch.empty((world,) + tuple(buf.shape), dtype=buf.dtype, device=buf.device)
                self.frame_buf = renderer.alloc_target(width, height, fmt)
        else:
            self.my_rows = height
            self.rows_per_rank = height
            self.local = renderer.alloc_target(width, height, fmt)
            self.frame_buf = self.local

    def render_local(self, step_counter=None, events=None):
        """Launch this rank's bands (async on the current stream)."""
        if events is not None:
            events[0].record()
        if self.world > 1:
            self.r.render(self.width, self.height, self.gfmt, out=self.local[: self.my_rows],
                          band_rows=self.band_rows, band_stride=self.world, band_first=self.rank,
                          step_counter=step_counter)
        else:
            self.r.render(self.width, self.height, self.fmt, out=self.local, step_counter=step_counter)
        if events is not None:
            events[1].record()

    def frame(self, events=None):
        """One frame: render local bands, gather to rank 0, assemble there.
        Returns the full frame on rank 0 and the local band set elsewhere."""
        self.render_local(events=events)
        if self.world == 1:
            return self.frame_buf
        if self.local.is_cuda and dist.get_backend(self.group) == "gloo":
            # gloo moves host memory only: stage through the host (tests and
            # one-GPU rehearsals; RCCL gathers device buffers directly)
            loc = self.local.cpu()
            gl = [torch.empty_like(loc) for _ in range(self.world)] if self.rank == 0 else None
            dist.gather(loc, gather_list=gl, dst=0, group=self.group)
            if self.rank == 0:
                self.gathered.copy_(torch.stack(gl))
        else:
            gl = list(self.gathered.unbind(0)) if self.rank == 0 else None
            dist.gather(self.local, gather_list=gl, dst=0, group=self.group)
        if self.rank == 0:
            self._assemble(self.gathered, self.frame_buf)
            return self.frame_buf
        return self.local

    def _assemble(self, gathered, frame):
        if hasattr(self.r, "assemble_frame"):
            self.r.assemble_frame(gathered, self.gfmt, self.world, self.width, self.height, self.band_rows,
                                  self.fmt, frame=frame)
        else:
            self.r.assemble_bands(gathered, self.world, self.width, self.height, self.band_rows, frame=frame)

    def run_frames(self, k: int, events=None):
        """Render k frames with two in flight, mirroring the reference's
        2 frames in flight (VulkanRenderer.cpp:13).  Frame i's gather (RCCL
        stream) overlaps frame i+1's render (compute stream).  Band sets,
        gather buffers and frames are double-buffered.  Each buffer of a
        parity is reused only after the stream order has retired its last
        reader.  Returns the last frame (rank 0) or band set."""
        # (a procedural medium with deferred shadow rays overlaps too since
        # round 6: a frame that reuses the cost order writes only its
        # stream's deferred scratch set)
        if self.world == 1 and self.inflight == 2 and hasattr(self.r, "prepare_render"):
            # one rank, grid medium, inflight 2 (throughput mode): consecutive
            # frames alternate between two streams and two targets, so frame
            # i+1's waves fill the SIMDs while frame i's last, longest rays
            # finish (3-7 % more frames/s at config 5,
            # profiles/r04/inflight_ab.txt; each launch then overlaps the next,
            # so per-launch kernel times no longer measure one frame, and the
            # default stays one stream).  The grid render's only shared state
            # is the read-only region lists; a procedural frame that reuses the
            # cost order only reads the ctx's scratch, and vr_render orders a
            # writing frame after every reader.  Both streams start after
            # the caller's stream and the caller's stream waits for both.
            if getattr(self, "_launch2", None) is None:
                self._streams2 = [torch.cuda.Stream(self.local.device), torch.cuda.Stream(self.local.device)]
                self._targets2 = [self.local, torch.empty_like(self.local)]
                self._launch2 = [self.r.prepare_render(self.width, self.height, self.fmt, self._targets2[j],
                                                       stream=self._streams2[j]) for j in range(2)]
            cur = torch.cuda.current_stream(self.local.device)
            for st in self._streams2:
                st.wait_stream(cur)
            for i in range(k):
                j = i % 2
                ev = events[i] if events else None
                if ev is not None:
                    ev[0].record(self._streams2[j])
                self._launch2[j]()
                if ev is not None:
                    ev[1].record(self._streams2[j])
            for st in self._streams2:
                cur.wait_stream(st)
            # the last target, without moving self.frame_buf: the one-stream
            # paths (frame(), the procedural medium) render into self.local and
            # return self.frame_buf, which must stay that buffer
            return self._targets2[(k - 1) % 2] if k > 0 else self.frame_buf
        if self.world == 1 and hasattr(self.r, "prepare_render"):
            # one rank: one stream, a prepared launcher (ctypes arguments built once)
            if getattr(self, "_launch1", None) is None:
                self._launch1 = self.r.prepare_render(self.width, self.height, self.fmt, self.local)
            for i in range(k):
                ev = events[i] if events else None
                if ev is not None:
                    ev[0].record()
                self._launch1()
                if ev is not None:
                    ev[1].record()
            return self.frame_buf
        if self.world == 1 or (self.local.is_cuda and dist.get_backend(self.group) == "gloo"):
            out = None
            for i in range(k):
                out = self.frame(events=events[i] if events else None)
            return out
        if getattr(self, "_pipe", None) is None:
            self._pipe = {
                "local": [self.local, torch.empty_like(self.local)],
                "gathered": [self.gathered, torch.empty_like(self.gathered)] if self.rank == 0 else [None, None],
                "frame": [self.frame_buf, torch.empty_like(self.frame_buf)] if self.rank == 0 else [None, None],
            }
            # per-rank views of the gather buffers and the render / assemble
            # launchers, made once (host time per frame is what limits strong
            # scaling of a ~0.03 ms/rank frame)
            self._pipe["lists"] = ([list(g.unbind(0)) for g in self._pipe["gathered"]] if self.rank == 0
                                   else [None, None])
            if hasattr(self.r, "prepare_render"):
                self._pipe["render"] = [
                    self.r.prepare_render(self.width, self.height, self.gfmt, loc[: self.my_rows],
                                          band_rows=self.band_rows, band_stride=self.world, band_first=self.rank)
                    for loc in self._pipe["local"]]
                self._pipe["assemble"] = ([
                    self.r.prepare_assemble_frame(g, self.gfmt, self.world, self.width, self.height, self.band_rows,
                                                  self.fmt, fr)
                    for g, fr in zip(self._pipe["gathered"], self._pipe["frame"])] if self.rank == 0
                    else [None, None])
        P = self._pipe
        pending = None

        def finish(p):
            work, par = p
            work.wait()   # the current stream waits for the gather
            if self.rank == 0:
                if "assemble" in P:
                    P["assemble"][par]()
                else:
                    self._assemble(P["gathered"][par], P["frame"][par])

        last = None
        for i in range(k):
            par = i & 1
            loc = P["local"][par]
            ev = events[i] if events else None
            if ev is not None:
                ev[0].record()
            if "render" in P:
                P["render"][par]()
            else:
                self.r.render(self.width, self.height, self.gfmt, out=loc[: self.my_rows],
                              band_rows=self.band_rows, band_stride=self.world, band_first=self.rank)
            if ev is not None:
                ev[1].record()
            work = dist.gather(loc, gather_list=P["lists"][par], dst=0, group=self.group, async_op=True)
            if pending is not None:
                finish(pending)
            pending = (work, par)
            last = par
        finish(pending)
        return P["frame"][last] if self.rank == 0 else P["local"][last]

    def close(self):
        self._launch1 = None
        self.local = None
        self.gathered = None
        self.frame_buf = None
        self._pipe = None


# rank 0's lead rows beside its assembly when it is a compositor over band
# sets: it counts as this % of a renderer (vr_shard_balance_lead; DESIGN.md
# sec. 7.5).  With serpentine band sets, config 5 (1080p) at 8 ranks: 60
# chooses 304 rows, the measured best -- 0.0174-0.0179 ms per frame against
# 0.0179-0.0184 at 40 (288 rows) and 0.0225 at 80 (336 rows).  Config 4 (4K):
# 80 chooses 688 rows -- 0.0400-0.0406 against 0.0407 at 60, 0.0421 at 40 and
# 0.0464 at 95 -- so frames past 2560 x 1440 take AUTO_LEAD_PCT_LARGE.
AUTO_LEAD_PCT = 60
AUTO_LEAD_PCT_LARGE = 80


class RcclBandPipeline:
    """The native multi-GPU frame loop (libvr_shard.so, include/vr_shard.h):
    the same interleaved bands and gather to rank 0 as :class:`BandSharder`,
    but the exchange is this library's own RCCL communicator (grouped
    point-to-point sends/receives over xGMI) and the whole 2-in-flight frame
    loop runs in C++, so the host cost per frame is a few HIP/RCCL calls.

    `group` is any torch.distributed group (gloo is enough): it only carries
    the communicator id from rank 0 and the barriers."""

    def __init__(self, renderer, width: int, height: int, fmt: int, band_rows: int = 16, world: int = 1,
                 rank: int = 0, group=None, loopback: bool = False, timeout_s: float | None = None,
                 render_streams: int | None = None, solo: bool = False, host_threads: int = 1, exchange_on_render: bool = True,
                 compositor: bool | None = None, partition: str = "auto", rows: list[int] | None = None,
                 lead_pct: int | str | None = "auto", lead_rows: int | None = None,
                 serpentine: bool | None = None):
        """loopback: one process renders all `world` ranks' band sets on its
        GPU and assembles them (no communicator; tests and rehearsals).
        solo (loopback only, any rank): each frame renders only this rank's
        band set, without an exchange -- one rank's frame period on one GPU
        (vr_shard_set_solo; tools/band_scaling.py --native).
        render_streams: n = 2..4 consecutive frames render on n alternating
        streams and overlap; 1 = on the caller's stream, in turn
        (vr_shard_set_render_streams).  None (default): 3 for frames of more
        than 2560 x 1440 pixels (config 4 at 8 ranks: 0.0431 ms per frame
        against 0.0486 with 2; 4 streams exceed the process's 4 hardware
        queues and lose), else 2 (config 5: equal).
        host_threads: 2 = a worker thread issues every frame's exchange half
        (vr_shard_set_host_threads).
        compositor: rank 0 renders no bands and only assembles, ranks 1..N-1
        render the band sets of N-1 renderers (vr_shard_set_compositor; None =
        the library's default: on from 8 ranks; every rank the same).
        partition: "bands" = interleaved band sets of `band_rows` rows (stride
        = the renderers); "rows" = contiguous row ranges of equal estimated
        work for the camera set at the first run_frames (vr_shard_balance_rows,
        collective); "auto" (default) = "bands".  Row ranges were the 4K
        default at 8 ranks until serpentine band sets with rank 0's lead rows
        beat them (config 4: 0.0402-0.0406 ms per frame against 0.0431-0.0434,
        DESIGN.md sec. 7.5).
        rows: explicit row starts for partition "rows" (renderers + 1 entries,
        vr_shard_set_rows; every rank the same) instead of the balanced split.
        lead_pct / lead_rows (compositor over band sets only): rank 0 also
        renders the frame's first rows in place, beside its assembly, and the
        renderers' band sets cover the rest -- sized at the first run_frames
        for the camera with rank 0 counted as lead_pct % of a renderer
        (vr_shard_balance_lead, collective), or lead_rows explicit rows (a
        multiple of band_rows; vr_shard_set_lead_rows).  "auto" (default):
        lead_pct AUTO_LEAD_PCT (AUTO_LEAD_PCT_LARGE past 2560 x 1440 pixels)
        whenever rank 0 is a compositor over band sets (config 5 at 8 ranks,
        serpentine band sets: slowest rank 0.0174-0.0179 ms per frame;
        0.0203-0.0204 with no lead rows and the plain deal; config 4
        0.0400-0.0406), else none; None: none.
        serpentine: band sets dealt forwards and backwards in turn (vr.h
        vr_target.band_flip; vr_shard_set_serpentine; None = the library's
        default, on; every rank the same).
        exchange_on_render: True (default) = each frame's exchange follows its
        render on the frame's render stream, over a communicator per buffer
        parity, with no events; False = on a communication stream, ordered by
        events (vr_shard_set_exchange_streams; every rank the same).
        timeout_s: deadline of every host wait on a collective, from the
        communicator init on (vr_shard_set_timeout; default VR_SHARD_TIMEOUT_S
        or 120 s).  A rank whose peer fails gets VRError VR_ERR_TIMEOUT /
        VR_ERR_COMM instead of hanging."""
        self.r = renderer
        self.width, self.height, self.fmt = width, height, fmt
        self.world, self.rank, self.group, self.loopback = world, rank, group, loopback
        if solo and not loopback:
            raise ValueError("RcclBandPipeline: solo is a loopback rehearsal")
        uid = (ctypes.c_uint8 * _lib.SHARD_ID_BYTES)()
        err = None
        if loopback:
            if rank != 0 and not solo:
                raise ValueError("RcclBandPipeline: a loopback pipeline of rank > 0 needs solo=True")
            uid = None
        elif rank == 0:
            try:
                _lib.shard_call("vr_shard_unique_id", uid)
            except _lib.VRError as e:   # still broadcast, so no rank waits forever
                err = e
        if world > 1 and not loopback:
            backend = dist.get_backend(group)
            t = torch.tensor([0 if err else 1] + list(bytearray(uid)), dtype=torch.uint8,
                             device="cuda" if backend == "nccl" else "cpu")
            dist.broadcast(t, src=0, group=group)
            got = t.cpu().tolist()
            if not got[0]:
                raise err or _lib.VRError(2, "vr_shard_unique_id", "failed on rank 0")
            ctypes.memmove(uid, bytes(got[1:]), _lib.SHARD_ID_BYTES)
        elif err:
            raise err
        # Two phases, so that no rank enters the collective communicator init
        # while a peer has failed to allocate (it would block there forever):
        # allocate locally, agree over the torch group, then connect.
        h = ctypes.c_void_p()
        alloc_err = None
        try:
            _lib.shard_call("vr_shard_alloc", renderer._ctx, world, rank, width, height, fmt, band_rows,
                            ctypes.byref(h))
        except _lib.VRError as e:
            alloc_err = e
        if world > 1 and not loopback:
            ok = torch.tensor([0 if alloc_err else 1], dtype=torch.int64,
                              device="cuda" if dist.get_backend(group) == "nccl" else "cpu")
            dist.all_reduce(ok, op=dist.ReduceOp.MIN, group=group)
            if int(ok.item()) == 0:
                if h:
                    _lib.shard_call("vr_shard_destroy", h)
                raise alloc_err or _lib.VRError(2, "vr_shard_alloc", "failed on another rank")
        elif alloc_err:
            raise alloc_err
        if timeout_s is not None:
            _lib.shard_call("vr_shard_set_timeout", h, float(timeout_s))
        try:
            if render_streams is None:
                render_streams = 3 if width * height > 2560 * 1440 else 2
            _lib.shard_call("vr_shard_set_render_streams", h, int(render_streams))
            _lib.shard_call("vr_shard_set_host_threads", h, int(host_threads))
            _lib.shard_call("vr_shard_set_exchange_streams", h, 1 if exchange_on_render else 0)
            if compositor is not None:
                _lib.shard_call("vr_shard_set_compositor", h, 1 if compositor else 0)
            if serpentine is not None:
                _lib.shard_call("vr_shard_set_serpentine", h, 1 if serpentine else 0)
            if solo:
                _lib.shard_call("vr_shard_set_solo", h, 1)
        except _lib.VRError:
            _lib.shard_call("vr_shard_destroy", h)
            raise
        if not loopback:
            try:
                _lib.shard_call("vr_shard_connect", h, uid)
            except _lib.VRError:
                _lib.shard_call("vr_shard_destroy", h)
                raise
        self._h = h
        if partition not in ("auto", "bands", "rows"):
            raise ValueError(f"RcclBandPipeline: partition {partition!r}: 'auto', 'bands' or 'rows'")
        self.partition = "bands" if partition == "auto" else partition
        self._balanced = self.partition == "bands"
        if rows is not None:
            if self.partition != "rows":
                _lib.shard_call("vr_shard_destroy", h)
                raise ValueError("RcclBandPipeline: rows needs partition 'rows'")
            # vr_shard_set_rows reads renderers + 1 ints: the
            # renderer count is the band stride of the current geometry
            stride, first = ctypes.c_int(), ctypes.c_int()
            _lib.shard_call("vr_shard_bands", h, ctypes.byref(stride), ctypes.byref(first), None)
            if len(rows) != stride.value + 1:
                _lib.shard_call("vr_shard_destroy", h)
                raise ValueError(f"RcclBandPipeline: rows needs {stride.value + 1} entries (renderers + 1), "
                                 f"got {len(rows)}")
            _lib.shard_call("vr_shard_set_rows", h, (ctypes.c_int * len(rows))(*rows))
            self._balanced = True
        self._lead_pct = None
        if lead_pct == "auto":
            lead_pct = ((AUTO_LEAD_PCT_LARGE if width * height > 2560 * 1440 else AUTO_LEAD_PCT)
                        if lead_rows is None and self.partition == "bands"
                        and bool(_lib.shard_call("vr_shard_get_compositor", h)) else None)
        if lead_pct is not None or lead_rows is not None:
            if not bool(_lib.shard_call("vr_shard_get_compositor", h)) or self.partition != "bands":
                _lib.shard_call("vr_shard_destroy", h)
                raise ValueError("RcclBandPipeline: lead rows need rank 0 as a compositor over band sets")
            if lead_rows is not None:
                try:
                    _lib.shard_call("vr_shard_set_lead_rows", h, int(lead_rows))
                except _lib.VRError:
                    _lib.shard_call("vr_shard_destroy", h)
                    raise
            else:
                self._lead_pct = int(lead_pct)
        self._geometry()

    def _geometry(self) -> None:
        h = self._h
        mine, per = ctypes.c_int(), ctypes.c_int()
        _lib.shard_call("vr_shard_rows", h, ctypes.byref(mine), ctypes.byref(per))
        self.my_rows, self.rows_per_rank = mine.value, per.value
        stride, first, flip = ctypes.c_int(), ctypes.c_int(), ctypes.c_int()
        _lib.shard_call("vr_shard_bands", h, ctypes.byref(stride), ctypes.byref(first), ctypes.byref(flip))
        # this rank's band set (vr_render target)
        self.band_stride, self.band_first, self.band_flip = stride.value, first.value, flip.value
        self.serpentine = bool(_lib.shard_call("vr_shard_get_serpentine", h))
        self.compositor = bool(_lib.shard_call("vr_shard_get_compositor", h))
        self.lead_rows = _lib.shard_call("vr_shard_get_lead_rows", h)   # rank 0's lead rows (0: none)
        self.row_range = None   # (first frame row, rows) of this rank with row ranges
        if _lib.shard_call("vr_shard_partition", h) == 1:
            r0, n = ctypes.c_int(), ctypes.c_int()
            _lib.shard_call("vr_shard_row_range", h, self.rank, ctypes.byref(r0), ctypes.byref(n))
            self.row_range = (r0.value, n.value)

    def rebalance_rows(self, frames: int = 16, stream=None) -> list[int]:
        """Collective, with row ranges: render `frames` frames with every
        render sampled, then split the frame again by every rank's measured
        render time (vr_shard_rebalance_rows).  Returns the new row starts
        (this rank's view: its own range is self.row_range)."""
        if self.partition != "rows":
            raise ValueError("rebalance_rows: the pipeline renders band sets")
        # measured on one render stream: with frames in flight, a sampled
        # render's bracket also holds the overlapping frames' work
        streams = self.render_streams
        self.render_streams = 1
        try:
            ms = self.run_frames(frames, stream=stream, sample_every=1)
        finally:
            self.render_streams = streams
        _lib.shard_call("vr_shard_rebalance_rows", self._h, float(ms))
        self._geometry()
        return self.row_range

    def balance_rows(self) -> None:
        """Collective: contiguous row ranges of equal estimated work for the
        renderer's current camera (vr_shard_balance_rows: rank 0 computes,
        every rank receives).  run_frames calls it once with partition="rows"."""
        _lib.shard_call("vr_shard_balance_rows", self._h)
        self._balanced = True
        self._geometry()

    @property
    def render_streams(self) -> int:
        return _lib.shard_call("vr_shard_get_render_streams", self._h)

    @render_streams.setter
    def render_streams(self, n: int) -> None:
        _lib.shard_call("vr_shard_set_render_streams", self._h, int(n))

    def set_timeout(self, seconds: float) -> None:
        """Deadline (s) of every later host wait on a collective."""
        _lib.shard_call("vr_shard_set_timeout", self._h, float(seconds))

    @property
    def aborted(self) -> bool:
        """True once an error or a missed deadline aborted the communicator."""
        return bool(_lib.shard_call("vr_shard_aborted", self._h))

    def run_frames(self, k: int, stream=None, sample_every: int = 0, cameras=None):
        """Queue k frames (collective).  Returns the mean duration (ms) of the
        sampled renders when sample_every > 0, else None.  cameras: k
        (ObjectShaderData, GlobalShaderData) pairs, one per frame (a moving
        camera, vr_shard_run_frames; every rank passes the same); after the
        call self.host_ms is the host time per frame spent queueing them."""
        from .renderer import _stream_handle
        ms = ctypes.c_float()
        host = ctypes.c_double()
        if cameras is not None:
            cameras = list(cameras)
        if not self._balanced and k > 0:
            if cameras:   # the ranges follow the first frame's camera
                self.r.set_shader_data(*cameras[0])
            self.balance_rows()
        if self._lead_pct is not None and k > 0:   # rank 0's lead rows, for the first frame's camera
            if cameras:
                self.r.set_shader_data(*cameras[0])
            _lib.shard_call("vr_shard_balance_lead", self._h, self._lead_pct)
            self._lead_pct = None
            self._geometry()
        if cameras is None:
            _lib.shard_call("vr_shard_run_frames", self._h, k, None, None, _stream_handle(stream), sample_every,
                            ctypes.byref(ms) if sample_every > 0 else None, ctypes.byref(host))
        else:
            cams = list(cameras)
            if len(cams) != k:
                raise ValueError(f"run_frames: {k} frames need {k} cameras, got {len(cams)}")
            osd = (_lib.ObjectShaderData * max(1, k))(*[c[0] for c in cams])
            gsd = (_lib.GlobalShaderData * max(1, k))(*[c[1] for c in cams])
            _lib.shard_call("vr_shard_run_frames", self._h, k, osd, gsd, _stream_handle(stream), sample_every,
                            ctypes.byref(ms) if sample_every > 0 else None, ctypes.byref(host))
        self.host_ms = host.value
        return ms.value if sample_every > 0 else None

    def sampled_busy(self) -> tuple[float, float]:
        """(busy, span) in ms of the last run_frames call that sampled renders:
        the union of the sampled renders' intervals (overlapping renders count
        once) and first start -> last end, on the GPU's clock
        (vr_shard_sampled_busy).  With sample_every=1, busy / frames is the GPU
        time per frame."""
        busy, span = ctypes.c_double(), ctypes.c_double()
        _lib.shard_call("vr_shard_sampled_busy", self._h, ctypes.byref(busy), ctypes.byref(span))
        return busy.value, span.value

    def share_volume(self, vol=None, stream=None) -> None:
        """Collective, once per volume: rank 0's RGBA8 volume (a contiguous
        uint8 CUDA tensor (nz, ny, nx, 4); ignored on other ranks) is
        broadcast over this pipeline's own RCCL communicator and installed
        in every rank's renderer (vr_shard_share_volume).  The extent goes
        to the other ranks over the torch group first."""
        from .renderer import _stream_handle
        # -1s announce a bad volume on rank 0: every rank raises after the
        # broadcast, none is left waiting in it
        dims = torch.full((3,), -1, dtype=torch.int64)
        bad = None
        if self.rank == 0:
            if vol is None or not isinstance(vol, torch.Tensor) or not vol.is_cuda:
                bad = "share_volume: rank 0 needs the volume as a CUDA tensor"
            elif vol.dtype != torch.uint8 or vol.dim() != 4 or vol.shape[3] != 4 or not vol.is_contiguous():
                bad = "share_volume: the volume must be a contiguous uint8 tensor (nz, ny, nx, 4)"
            else:
                dims = torch.tensor([vol.shape[2], vol.shape[1], vol.shape[0]], dtype=torch.int64)
        if self.world > 1 and not self.loopback:
            t = dims.to("cuda" if dist.get_backend(self.group) == "nccl" else "cpu")
            dist.broadcast(t, src=0, group=self.group)
            dims = t.cpu()
        nx, ny, nz = (int(v) for v in dims.tolist())
        if bad or min(nx, ny, nz) <= 0:
            raise ValueError(bad or "share_volume: rank 0 had no valid volume")
        ptr = ctypes.c_void_p(vol.data_ptr()) if self.rank == 0 else None
        _lib.shard_call("vr_shard_share_volume", self._h, ptr, nx, ny, nz, _stream_handle(stream))

    def barrier(self, stream=None):
        """Collective: returns once every rank's queued frames (on `stream`
        and the exchange stream) have finished -- a device-side RCCL barrier
        plus a host wait (vr_shard_barrier)."""
        from .renderer import _stream_handle
        _lib.shard_call("vr_shard_barrier", self._h, _stream_handle(stream))

    def frame(self, stream=None) -> torch.Tensor:
        """A copy of the last frame (rank 0) or grey band set (other ranks)."""
        from .renderer import _stream_handle
        rows = self.height if self.rank == 0 else self.my_rows
        out = self.r.alloc_target(self.width, rows, self.fmt if self.rank == 0 else _lib.GREY_OF[self.fmt])
        _lib.shard_call("vr_shard_copy_frame", self._h, ctypes.c_void_p(out.data_ptr()), 0, _stream_handle(stream))
        return out

    def close(self):
        if getattr(self, "_h", None):
            _lib.shard_call("vr_shard_destroy", self._h)
            self._h = None
