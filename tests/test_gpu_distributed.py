"""Multi-rank frame path on a real GPU: 2 ranks share the one GPU of the test
box and gather over gloo.  The 8-GPU RCCL run is the driver's.  The rank-0
frame, assembled by vr_assemble_bands, must equal a one-rank render."""
import os
import socket

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q, share=False):
    import sys
    sys.path.insert(0, ROOT)
    import torch.distributed as dist

    import volumetricrenderer_amd as vr
    from volumetricrenderer_amd.distributed import BandSharder, share_volume
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        torch.cuda.set_device(0)
        W, H = 640, 360
        with vr.Renderer(0) as r:
            if share:   # only rank 0 makes the volume; the others receive it (SURVEY.md 8e collective 1)
                vol = None
                if rank == 0:
                    r.generate_volume(vr.volume_recipe_defaults(size=64))
                    vol = r.get_volume()
                share_volume(r, vol, rank=rank)
            else:
                r.generate_volume(vr.volume_recipe_defaults(size=64))
            osd, gsd = vr.reference_shader_data(W / H, 10.0, 20.0)
            r.set_shader_data(osd, gsd)
            r.set_march(vr.march_defaults())
            sh = BandSharder(r, W, H, vr.FMT_RGBA32F, band_rows=16, world=world, rank=rank)
            frame = sh.frame()
            torch.cuda.synchronize()
            if rank == 0:
                full = r.render(W, H, vr.FMT_RGBA32F).cpu().numpy()
                q.put(("ok", bool(np.array_equal(frame.cpu().numpy(), full))))
            else:
                q.put(("ok", True))
            sh.close()
    except Exception as e:  # pragma: no cover
        q.put(("err", repr(e)))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,share", [(2, False), (3, False), (3, True)])
def test_gloo_ranks_on_one_gpu_assemble_the_frame(world, share):
    """share=True: the volume exists only on rank 0 and reaches the others
    through distributed.share_volume before the frame."""
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(rk, world, port, q, share)) for rk in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=300) for _ in procs]
    for p in procs:
        p.join(timeout=60)
    assert all(r == ("ok", True) for r in res), res


@pytest.mark.parametrize("fmt,band_rows,on_render,streams", [(1, 16, False, 2), (0, 8, False, 2), (1, 16, True, 2),
                                                             (1, 16, True, 4)])
def test_rccl_pipeline_one_rank(fmt, band_rows, on_render, streams):
    """The native frame loop (libvr_shard.so) with a one-rank RCCL
    communicator: render into the gather slot, (no peers), assemble, 2 frames
    in flight.  The frame equals a plain render; the kernel-time sample is
    positive; the RCCL barrier returns.  Multi-rank RCCL needs one GPU per rank (the driver's run)."""
    import sys
    sys.path.insert(0, ROOT)
    import volumetricrenderer_amd as vr
    from volumetricrenderer_amd.distributed import RcclBandPipeline
    W, H = 640, 360
    with vr.Renderer(0) as r:
        r.generate_volume(vr.volume_recipe_defaults(size=64))
        osd, gsd = vr.reference_shader_data(W / H, 10.0, 20.0)
        r.set_shader_data(osd, gsd)
        r.set_march(vr.march_defaults())
        pl = RcclBandPipeline(r, W, H, fmt, band_rows=band_rows, world=1, rank=0, exchange_on_render=on_render,
                              render_streams=streams)
        try:
            assert pl.my_rows == pl.rows_per_rank == vr.band_rows_packed(H, band_rows, 1, 0) >= H
            ms = pl.run_frames(5, sample_every=2)
            assert ms > 0
            pl.barrier()   # one-rank RCCL all-reduce + host wait (the bench's bracket)
            got = pl.frame()
            full = r.render(W, H, fmt)
            torch.cuda.synchronize()
            assert np.array_equal(got.cpu().numpy(), full.cpu().numpy())
            pl.run_frames(4)
            got2 = pl.frame()
            torch.cuda.synchronize()
            assert np.array_equal(got2.cpu().numpy(), full.cpu().numpy())
        finally:
            pl.close()


def test_rccl_pipeline_deadline_aborts():
    """The failure path of the native frame loop (verdict r02 #6): with a
    deadline far shorter than the queued work, the barrier's host wait gives
    up, aborts the (one-rank, non-blocking) communicator and raises
    VR_ERR_TIMEOUT instead of waiting; every later collective on the shard
    fails at once with VR_ERR_COMM, and the shard can still be closed."""
    import sys
    sys.path.insert(0, ROOT)
    import volumetricrenderer_amd as vr
    from volumetricrenderer_amd.distributed import RcclBandPipeline
    W, H = 3840, 2160
    with vr.Renderer(0) as r:
        r.generate_volume(vr.volume_recipe_defaults(size=128))
        osd, gsd = vr.reference_shader_data(W / H)
        r.set_shader_data(osd, gsd)
        r.set_march(vr.march_defaults(max_steps=256))
        pl = RcclBandPipeline(r, W, H, vr.FMT_RGBA32F, band_rows=16, world=1, rank=0, timeout_s=30.0)
        try:
            pl.run_frames(2)
            pl.barrier()            # within the deadline: fine
            assert not pl.aborted
            pl.set_timeout(1e-6)    # ~20 frames of 4K x 256 take milliseconds
            pl.run_frames(20)
            with pytest.raises(vr.VRError) as e:
                pl.barrier()
            assert e.value.status == 7, e.value   # VR_ERR_TIMEOUT
            assert pl.aborted
            with pytest.raises(vr.VRError) as e2:
                pl.run_frames(1)
            assert e2.value.status == 8, e2.value  # VR_ERR_COMM
            torch.cuda.synchronize()
        finally:
            pl.close()


def test_rccl_init_deadline_when_a_peer_never_joins():
    """A 2-rank communicator whose rank 1 never joins (it died before the
    collective init): rank 0's non-blocking ncclCommInitRankConfig gives up at
    the deadline with VR_ERR_TIMEOUT and the communicator aborted, instead of
    waiting forever (the init deadline, untested until now)."""
    import ctypes
    import sys
    import time
    sys.path.insert(0, ROOT)
    import volumetricrenderer_amd as vr
    from volumetricrenderer_amd import _lib
    with vr.Renderer(0) as r:
        h = ctypes.c_void_p()
        _lib.shard_call("vr_shard_alloc", r._ctx, 2, 0, 64, 64, 1, 16, ctypes.byref(h))
        try:
            _lib.shard_call("vr_shard_set_timeout", h, 3.0)
            uid = (ctypes.c_uint8 * _lib.SHARD_ID_BYTES)()
            _lib.shard_call("vr_shard_unique_id", uid)
            t0 = time.perf_counter()
            with pytest.raises(vr.VRError) as e:
                _lib.shard_call("vr_shard_connect", h, uid)
            el = time.perf_counter() - t0
            assert e.value.status == 7, e.value   # VR_ERR_TIMEOUT
            assert 2.5 < el < 30.0, el
            assert _lib.shard_call("vr_shard_aborted", h) == 1
            with pytest.raises(vr.VRError) as e2:   # every later collective fails at once
                _lib.shard_call("vr_shard_barrier", h, None)
            assert e2.value.status in (2, 8), e2.value
        finally:
            _lib.shard_call("vr_shard_destroy", h)


def slot_rows(vr, H, band_rows, renderers, first0=0, serpentine=True):
    """Rows of a gather slot: the largest renderer's band set (serpentine:
    renderer k's odd bands shifted by R-1-2k, vr_shard_set_serpentine)."""
    R = renderers
    return max(vr.band_rows_packed(H, band_rows, R, first0 + k, (R - 1 - 2 * k) if serpentine and R > 1 else 0)
               for k in range(R))


@pytest.mark.parametrize("render_streams", [1, 2, 3, 4])
@pytest.mark.parametrize("world,band_rows,fmt,W,serp", [(2, 16, 1, 500, None), (3, 16, 0, 500, None),
                                                        (8, 16, 1, 500, None), (5, 7, 1, 500, None),
                                                        (3, 16, 2, 499, None), (4, 16, 0, 499, None),
                                                        (8, 16, 1, 500, False), (3, 16, 0, 499, False)])
def test_native_pipeline_loopback_ranks(world, band_rows, fmt, W, render_streams, serp):
    """The native frame loop's N-rank data layout (grey band sets in gather
    slots of rank 0's row count, expanded by vr_assemble_frame) with every
    rank's bands rendered by this one process: the frame equals a plain
    render.  Width 499 takes the per-pixel expansion, 500 the 4-pixel one.
    With 1 render stream and with 2 (consecutive frames overlap).  Band sets
    serpentine (the default) and plain (serp False)."""
    import sys
    sys.path.insert(0, ROOT)
    import volumetricrenderer_amd as vr
    from volumetricrenderer_amd.distributed import RcclBandPipeline
    H = 283
    with vr.Renderer(0) as r:
        r.generate_volume(vr.volume_recipe_defaults(size=64))
        osd, gsd = vr.reference_shader_data(W / H, -30.0, 40.0)
        r.set_shader_data(osd, gsd)
        r.set_march(vr.march_defaults())
        pl = RcclBandPipeline(r, W, H, fmt, band_rows=band_rows, world=world, rank=0, loopback=True,
                              render_streams=render_streams, serpentine=serp)
        try:
            assert pl.render_streams == render_streams
            assert pl.serpentine == (serp is not False)
            R = world - 1 if pl.compositor else world
            assert pl.rows_per_rank == slot_rows(vr, H, band_rows, R, 0, pl.serpentine)
            pl.run_frames(3)
            pl.barrier()   # loopback: a stream synchronisation
            got = pl.frame()
            full = r.render(W, H, fmt)
            torch.cuda.synchronize()
            assert np.array_equal(got.cpu().numpy(), full.cpu().numpy())
        finally:
            pl.close()


@pytest.mark.parametrize("world,fmt,W,render_streams,lead", [(2, 1, 500, 2, 16), (3, 0, 499, 1, 112),
                                                              (8, 1, 500, 2, "pct80"), (8, 2, 500, 3, 48),
                                                              (8, 1, 499, 2, 272), (4, 1, 500, 4, "pct50"),
                                                              (8, 0, 500, 2, 0)])
def test_native_pipeline_loopback_lead_rows(world, fmt, W, render_streams, lead):
    """Rank 0 as a compositor that also renders the frame's lead rows in place
    (vr_shard_set_lead_rows / vr_shard_balance_lead; verdict r05 #5): the
    renderers' band sets start below the lead rows (vr_shard_bands reports
    the offset sets), the assembly expands the frame below them, and the frame
    equals a plain render -- explicit lead rows (0, one band, up to a quarter
    of the frame) and a lead sized from the camera (pct of a mean share), on
    1-4 render streams.  Bad lead rows are refused."""
    import sys
    sys.path.insert(0, ROOT)
    import volumetricrenderer_amd as vr
    from volumetricrenderer_amd import _lib
    from volumetricrenderer_amd.distributed import RcclBandPipeline
    H = 283
    with vr.Renderer(0) as r:
        r.generate_volume(vr.volume_recipe_defaults(size=64))
        osd, gsd = vr.reference_shader_data(W / H, -30.0, 40.0)
        r.set_shader_data(osd, gsd)
        r.set_march(vr.march_defaults())
        kw = dict(lead_pct=int(lead[3:])) if isinstance(lead, str) else dict(lead_rows=lead)
        pl = RcclBandPipeline(r, W, H, fmt, band_rows=16, world=world, rank=0, loopback=True,
                              render_streams=render_streams, compositor=True, **kw)
        try:
            for bad in (8, -16, 288):   # not whole bands / negative / past the frame
                with pytest.raises(vr.VRError):
                    _lib.shard_call("vr_shard_set_lead_rows", pl._h, bad)
            pl.run_frames(3)
            pl.barrier()
            lr = pl.lead_rows
            if isinstance(lead, str):   # (the balance may choose no lead rows on a small frame)
                assert lr >= 0 and lr % 16 == 0, lr
            else:
                assert lr == lead
            assert pl.my_rows == lr and pl.band_first == -1
            assert pl.rows_per_rank == slot_rows(vr, H, 16, world - 1, lr // 16)
            got = pl.frame()
            full = r.render(W, H, fmt)
            torch.cuda.synchronize()
            assert np.array_equal(got.cpu().numpy(), full.cpu().numpy())
            with pytest.raises(vr.VRError):   # the geometry is fixed once frames are queued
                _lib.shard_call("vr_shard_set_lead_rows", pl._h, lr + 16)
        finally:
            pl.close()
    with vr.Renderer(0) as r:   # lead rows need the compositor over band sets
        r.generate_volume(vr.volume_recipe_defaults(size=32))
        r.set_shader_data(osd, gsd)
        with pytest.raises(ValueError):
            RcclBandPipeline(r, W, H, fmt, band_rows=16, world=world, rank=0, loopback=True, compositor=False,
                             lead_rows=16)


@pytest.mark.parametrize("world,compositor,fmt,W,render_streams", [(2, False, 1, 500, 2), (5, False, 0, 499, 1),
                                                                   (8, True, 1, 500, 2), (8, False, 2, 500, 4),
                                                                   (3, True, 1, 499, 3)])
def test_native_pipeline_loopback_row_ranges(world, compositor, fmt, W, render_streams):
    """The loop's contiguous row ranges (vr_shard_balance_rows): every
    renderer's range rendered by this process into a grey frame, rank 0's
    own range in place (or none, as a compositor), the rows below rank 0's
    expanded in one launch.  The frame equals a plain render; the ranges tile
    the frame in rank order."""
    import ctypes
    import sys
    sys.path.insert(0, ROOT)
    import volumetricrenderer_amd as vr
    from volumetricrenderer_amd import _lib
    from volumetricrenderer_amd.distributed import RcclBandPipeline
    H = 283
    with vr.Renderer(0) as r:
        r.generate_volume(vr.volume_recipe_defaults(size=64))
        osd, gsd = vr.reference_shader_data(W / H, -30.0, 40.0)
        r.set_shader_data(osd, gsd)
        r.set_march(vr.march_defaults())
        pl = RcclBandPipeline(r, W, H, fmt, band_rows=16, world=world, rank=0, loopback=True,
                              render_streams=render_streams, compositor=compositor, partition="rows")
        try:
            assert pl.row_range is None   # balanced at the first frames
            pl.run_frames(3)
            assert _lib.shard_call("vr_shard_partition", pl._h) == 1
            nxt = 0
            for k in range(world):
                r0, n = ctypes.c_int(), ctypes.c_int()
                _lib.shard_call("vr_shard_row_range", pl._h, k, ctypes.byref(r0), ctypes.byref(n))
                if compositor and k == 0:
                    assert n.value == 0
                    continue
                assert r0.value == nxt and (r0.value % 8 == 0)
                nxt = r0.value + n.value
            assert nxt == H
            assert pl.row_range == ((0, 0) if compositor else pl.row_range) and pl.my_rows == pl.row_range[1]
            pl.barrier()
            got = pl.frame()
            full = r.render(W, H, fmt)
            torch.cuda.synchronize()
            assert np.array_equal(got.cpu().numpy(), full.cpu().numpy())
            with pytest.raises(vr.VRError):   # fixed once frames are queued
                _lib.shard_call("vr_shard_set_rows", pl._h, None)
        finally:
            pl.close()


@pytest.mark.parametrize("world,loopback", [(1, False), (4, True)])
def test_native_share_volume(world, loopback):
    """vr_shard_share_volume: rank 0's device volume installed through the
    native pipeline -- over a one-rank RCCL communicator (the agreement
    all-reduce and the in-place broadcast run for real) or in loopback.  The
    renderer started without a volume; afterwards it holds exactly those
    bytes and the pipeline's frame equals a plain render of them by a second
    renderer."""
    import sys
    sys.path.insert(0, ROOT)
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import vr_oracle as oracle

    import volumetricrenderer_amd as vr
    from volumetricrenderer_amd.distributed import RcclBandPipeline
    W, H = 400, 240
    vol = oracle.build_volume(40)
    osd, gsd = vr.reference_shader_data(W / H, 15.0, -25.0)
    with vr.Renderer(0) as r, vr.Renderer(0) as ref:
        r.set_shader_data(osd, gsd)
        r.set_march(vr.march_defaults())
        pl = RcclBandPipeline(r, W, H, vr.FMT_RGBA32F, band_rows=16, world=world, rank=0, loopback=loopback)
        try:
            pl.share_volume(torch.from_numpy(vol).cuda())
            assert np.array_equal(r.get_volume(), vol)
            pl.run_frames(2)
            pl.barrier()
            got = pl.frame()
            ref.set_volume(vol)
            ref.set_shader_data(osd, gsd)
            ref.set_march(vr.march_defaults())
            full = ref.render(W, H, vr.FMT_RGBA32F)
            torch.cuda.synchronize()
            assert np.array_equal(got.cpu().numpy(), full.cpu().numpy())
            with pytest.raises(ValueError):   # not RGBA8
                pl.share_volume(torch.zeros((4, 4, 4, 3), dtype=torch.uint8, device="cuda"))
        finally:
            pl.close()


SPIN_DEG = 1.6   # TestMain.cpp:171-184, :222-224: the held A/D key, 100 deg/s x 0.016 s


@pytest.mark.parametrize("fmt,render_streams,threads,on_render,compositor",
                         [(0, 2, 1, False, None), (1, 2, 1, False, None), (1, 1, 1, False, None),
                          (1, 2, 2, False, None), (0, 2, 1, True, None), (1, 2, 1, True, False),
                          (1, 1, 1, True, True), (1, 3, 1, True, None), (0, 4, 1, True, False),
                          (1, 2, 1, True, "lead")])
def test_native_loopback_spinning_8_ranks(oracle, fmt, render_streams, threads, on_render, compositor):
    """A moving camera through the native 8-rank frame loop (loopback: this
    process renders every rank's interleaved band set): 40 frames, frame i
    with its own shader data (vr_shard_run_frames, phi += 1.6 deg), 2 in
    flight, on two alternating render streams (the default) or one.  Frames
    1, 33 and 40, assembled on rank 0, equal the oracle's whole frame bit for
    bit (RGBA32F and RGBA8).  At 8 ranks rank 0 is a compositor by default
    (renders no bands); compositor=False keeps it rendering in place;
    "lead": the compositor also renders 48 lead rows in place, and the band
    sets start below them, for the moving camera."""
    import sys
    sys.path.insert(0, ROOT)
    import volumetricrenderer_amd as vr
    from volumetricrenderer_amd.distributed import RcclBandPipeline
    W, H = 320, 180
    vol = oracle.build_volume(128)
    with vr.Renderer(0) as r:
        r.set_volume(vol)
        cams = [vr.reference_shader_data(W / H, SPIN_DEG * i, 0.0) for i in range(1, 41)]
        r.set_shader_data(*cams[0])
        r.set_march(vr.march_defaults())
        pl = RcclBandPipeline(r, W, H, fmt, band_rows=16, world=8, rank=0, loopback=True,
                              render_streams=render_streams, host_threads=threads, exchange_on_render=on_render,
                              compositor=True if compositor == "lead" else compositor,
                              lead_rows=48 if compositor == "lead" else None)
        assert pl.compositor == (compositor is not False)
        # (rank 0 rendering its own serpentine set 0: flip 7; the slot holds the largest set)
        assert pl.my_rows == (pl.lead_rows if pl.compositor else vr.band_rows_packed(H, 16, 8, 0, 7))
        assert pl.rows_per_rank == slot_rows(vr, H, 16, 7 if pl.compositor else 8, pl.lead_rows // 16)
        got, done = {}, 0
        try:
            for stop in (1, 33, 40):
                pl.run_frames(stop - done, cameras=cams[done:stop])
                if stop == 1:   # the band geometry is fixed once frames are queued
                    from volumetricrenderer_amd import _lib
                    with pytest.raises(vr.VRError):
                        _lib.shard_call("vr_shard_set_compositor", pl._h, 0 if pl.compositor else 1)
                    if compositor == "lead":
                        assert pl.lead_rows == 48 and pl.my_rows == pl.lead_rows
                assert pl.host_ms >= 0.0
                done = stop
                got[stop] = pl.frame()
            torch.cuda.synchronize()
        finally:
            pl.close()
    for i, img in got.items():
        obj, glob = vr.shader_data_arrays(*cams[i - 1])
        ref, _ = oracle.render(vol, obj, glob, oracle.from_params(vr.march_defaults()), W, H, fmt)
        assert np.array_equal(img.cpu().numpy(), ref), i


def band_set_of(frame, rank, world, band_rows, flip=0):
    """The packed rows of `rank`'s interleaved bands in a whole frame (vr.h;
    flip: the set's odd bands shifted, vr_target.band_flip)."""
    H = frame.shape[0]
    nb = (H + band_rows - 1) // band_rows
    bands = [b for k in range(nb + 1) for b in [rank + k * world + (flip if k % 2 else 0)] if b < nb]
    rows = [y for b in bands for y in range(b * band_rows, min(H, (b + 1) * band_rows))]
    return frame[rows]


@pytest.mark.parametrize("render_streams,interval,threads,on_render,compositor,partition",
                         [(2, 3, 1, False, None, "bands"), (2, 32, 1, False, None, "bands"),
                          (1, 3, 1, False, None, "bands"), (2, 3, 2, False, None, "bands"),
                          (2, 3, 1, True, None, "bands"), (2, 3, 1, True, True, "bands"),
                          (2, 3, 1, True, None, "rows"), (2, 3, 1, True, True, "rows"),
                          (2, 3, 1, True, True, "lead")])
def test_native_solo_rank_spinning(oracle, render_streams, interval, threads, on_render, compositor, partition):
    """One rank of a 4-rank frame loop rehearsed alone (vr_shard_set_solo:
    its band set only, no exchange) with a moving camera: 24 frames with their
    own shader data on two alternating render streams, the region lists
    rebuilt on the GPU every `interval` renders while the previous frame is
    still in flight on the other stream (per-stream retire events).  The band
    set of frames 1, 7, 20 and 24 equals the rows of the oracle's frame.
    partition="rows": the rank's contiguous row range instead, balanced for
    the first frame's camera and kept for the others.  "lead": band sets
    below rank 0's lead rows (vr_shard_balance_lead at the first frame; on
    this small frame the balance may choose no lead)."""
    import sys
    sys.path.insert(0, ROOT)
    import volumetricrenderer_amd as vr
    from volumetricrenderer_amd.distributed import RcclBandPipeline
    W, H, world, rank = 320, 180, 4, 2
    vol = oracle.build_volume(128)
    with vr.Renderer(0) as r:
        r.set_volume(vol)
        r.set_option("region_interval", interval)
        cams = [vr.reference_shader_data(W / H, SPIN_DEG * i, 0.5 * i) for i in range(1, 25)]
        r.set_shader_data(*cams[0])
        r.set_march(vr.march_defaults())
        pl = RcclBandPipeline(r, W, H, 1, band_rows=16, world=world, rank=rank, loopback=True, solo=True,
                              render_streams=render_streams, host_threads=threads, exchange_on_render=on_render,
                              compositor=compositor, partition="bands" if partition == "lead" else partition,
                              lead_pct=60 if partition == "lead" else None)
        if partition == "lead":
            pl.run_frames(1, cameras=cams[:1])   # sizes the lead rows for the first camera
            assert pl.lead_rows >= 0 and pl.lead_rows % 16 == 0
        stride, first, flip = pl.band_stride, pl.band_first, pl.band_flip
        lead_band = pl.lead_rows // 16
        assert (stride, first) == ((world - 1, rank - 1 + lead_band) if compositor else (world, rank))
        k = rank - 1 if compositor else rank   # the renderer index: serpentine by default
        assert pl.serpentine
        if partition != "rows":   # (the row ranges are set at the first run)
            assert flip == stride - 1 - 2 * k
        got, done = {}, (1 if partition == "lead" else 0)
        try:
            for stop in (1, 7, 20, 24):
                if stop <= done:
                    got[stop] = pl.frame()
                    continue
                pl.run_frames(stop - done, cameras=cams[done:stop])
                done = stop
                got[stop] = pl.frame()
            torch.cuda.synchronize()
            builds = r.get_option("region_gpu_builds")
        finally:
            pl.close()
    assert builds >= (24 // interval) - 1, builds
    for i, img in got.items():
        obj, glob = vr.shader_data_arrays(*cams[i - 1])
        ref, _ = oracle.render(vol, obj, glob, oracle.from_params(vr.march_defaults()), W, H, 1)
        if partition == "rows":
            want = ref[pl.row_range[0]:pl.row_range[0] + pl.row_range[1], :, 0]
        else:
            want = band_set_of(ref, first, stride, 16, flip)[..., 0]
            # (a set holding the frame's last, partial band has that band's
            # rows past the frame packed too: vr_band_rows_packed counts whole bands)
            assert img.shape[0] == vr.band_rows_packed(H, 16, stride, first, flip)
            img = img[:want.shape[0]]
        assert img.shape == want.shape and np.array_equal(img.cpu().numpy(), want), i


def test_render_sequence_spinning(oracle):
    """vr_render_sequence, the one-GPU frame loop with a moving camera: 33
    frames queued in one native call (with GPU-rebuilt region lists every 8
    renders); the target holds frame 33, equal to the oracle's."""
    import sys
    sys.path.insert(0, ROOT)
    import volumetricrenderer_amd as vr
    W, H = 320, 180
    vol = oracle.build_volume(128)
    with vr.Renderer(0) as r:
        r.set_volume(vol)
        r.set_march(vr.march_defaults())
        r.set_option("region_interval", 8)
        cams = [vr.reference_shader_data(W / H, SPIN_DEG * i, 0.0) for i in range(1, 34)]
        r.set_shader_data(*cams[0])
        out = r.alloc_target(W, H, 0)
        r.render(W, H, 0, out=out)   # the first lists: a host build
        r.render_sequence(W, H, 0, out, cams)
        torch.cuda.synchronize()
        assert r.get_option("region_gpu_builds") >= 3
        obj, glob = vr.shader_data_arrays(*cams[-1])
        ref, _ = oracle.render(vol, obj, glob, oracle.from_params(vr.march_defaults()), W, H, 0)
        assert np.array_equal(out.cpu().numpy(), ref)


def test_one_rank_frames_in_flight(oracle):
    """BandSharder at world 1 with inflight=2 (bench.py --inflight 2): grid
    frames alternate two streams and two targets (two frames in flight);
    each target's frame equals the oracle's, and the caller's stream waits
    for both.  The procedural medium with deferred shadow rays runs two in
    flight too since round 6 (per-stream deferred scratch): exact as well."""
    import sys
    sys.path.insert(0, ROOT)
    import volumetricrenderer_amd as vr
    from volumetricrenderer_amd.distributed import BandSharder
    W, H = 320, 180
    vol = oracle.build_volume(128)
    with vr.Renderer(0) as r:
        r.set_volume(vol)
        osd, gsd = vr.reference_shader_data(W / H, 10.0, 5.0)
        r.set_shader_data(osd, gsd)
        r.set_march(vr.march_defaults())
        sh = BandSharder(r, W, H, 0, inflight=2)
        obj, glob = vr.shader_data_arrays(osd, gsd)
        ref, _ = oracle.render(vol, obj, glob, oracle.from_params(vr.march_defaults()), W, H, 0)
        for k in (1, 4, 5):
            frame = sh.run_frames(k)
            torch.cuda.current_stream().synchronize()   # the caller's stream joined both
            assert np.array_equal(frame.cpu().numpy(), ref), k
        assert len(sh._targets2) == 2 and all(np.array_equal(t.cpu().numpy(), ref) for t in sh._targets2)
        m = vr.march_defaults(max_steps=32)
        r.set_march(m)
        r.set_procedural(shadow_steps=4)
        p = oracle.procedural_from(r.procedural)
        sh2 = BandSharder(r, W, H, 0, inflight=2)
        frame = sh2.run_frames(3)
        torch.cuda.synchronize()
        ref2, _ = oracle.render_procedural(p, obj, glob, oracle.from_params(m), W, H, 0)
        assert np.array_equal(frame.cpu().numpy(), ref2)
        assert getattr(sh2, "_launch2", None) is not None
        assert all(np.array_equal(t.cpu().numpy(), ref2) for t in sh2._targets2)


def test_frames_in_flight_then_one_stream_paths(oracle):
    """after an inflight=2 run of an even number of frames, the
    one-stream paths of the SAME sharder -- frame() and a procedural
    run_frames -- must return what they just rendered, not the other
    in-flight target.  Each path's frame is checked against the oracle after
    the camera changed, so a stale buffer shows."""
    import sys
    sys.path.insert(0, ROOT)
    import volumetricrenderer_amd as vr
    from volumetricrenderer_amd.distributed import BandSharder
    W, H = 320, 180
    vol = oracle.build_volume(96)
    cams = [vr.reference_shader_data(W / H, a, 5.0) for a in (10.0, 40.0, 70.0)]
    with vr.Renderer(0) as r:
        r.set_volume(vol)
        r.set_march(vr.march_defaults())
        sh = BandSharder(r, W, H, 0, inflight=2)

        def ref(c):
            obj, glob = vr.shader_data_arrays(*c)
            return oracle.render(vol, obj, glob, oracle.from_params(vr.march_defaults()), W, H, 0)[0]
        r.set_shader_data(*cams[0])
        f = sh.run_frames(4)
        torch.cuda.current_stream().synchronize()
        assert np.array_equal(f.cpu().numpy(), ref(cams[0]))
        r.set_shader_data(*cams[1])
        f = sh.frame()
        torch.cuda.synchronize()
        assert np.array_equal(f.cpu().numpy(), ref(cams[1]))
        m = vr.march_defaults(max_steps=32)
        r.set_march(m)
        r.set_procedural(shadow_steps=0)
        r.set_shader_data(*cams[2])
        f = sh.run_frames(2)
        torch.cuda.synchronize()
        obj, glob = vr.shader_data_arrays(*cams[2])
        want, _ = oracle.render_procedural(oracle.procedural_from(r.procedural), obj, glob, oracle.from_params(m),
                                           W, H, 0)
        assert np.array_equal(f.cpu().numpy(), want)


def test_procedural_frames_in_flight_readers_and_writers(oracle):
    """A procedural medium without shadow rays, two frames in flight
    (BandSharder inflight=2): frames that reuse the camera's cost order only
    read the ctx's scratch and overlap on two streams; a frame with a new
    camera rebuilds the order (writes) and must wait for the reader still in
    flight on the other stream, and the next readers for it.  Every frame of
    both cameras equals the oracle's; then the same with deferred shadow rays,
    two in flight as well (round 6: a reusing frame writes only its stream's
    deferred scratch set)."""
    import sys
    sys.path.insert(0, ROOT)
    import volumetricrenderer_amd as vr
    from volumetricrenderer_amd.distributed import BandSharder
    W, H = 320, 180
    m = vr.march_defaults(max_steps=32)
    cams = [vr.reference_shader_data(W / H, a, 5.0) for a in (15.0, 55.0)]
    with vr.Renderer(0) as r:
        r.set_march(m)
        r.set_procedural(shadow_steps=0)
        assert r.get_option("procedural") == 1
        p = oracle.procedural_from(r.procedural)
        sh = BandSharder(r, W, H, 0, inflight=2)
        want = []
        for c in cams:
            obj, glob = vr.shader_data_arrays(*c)
            want.append(oracle.render_procedural(p, obj, glob, oracle.from_params(m), W, H, 0)[0])
        for k, c in ((5, 0), (4, 1), (3, 0)):
            r.set_shader_data(*cams[c])
            f = sh.run_frames(k)
            torch.cuda.current_stream().synchronize()
            assert sh._launch2 is not None
            assert np.array_equal(f.cpu().numpy(), want[c]), (k, c)
            assert all(np.array_equal(t.cpu().numpy(), want[c]) for t in sh._targets2), (k, c)
        # deferred shadow rays (round 6): a frame that reuses the order writes
        # only its stream's scratch set, so these overlap on two streams too
        r.set_procedural(shadow_steps=4)
        assert r.get_option("procedural") == 2
        p = oracle.procedural_from(r.procedural)
        want = []
        for c in cams:
            obj, glob = vr.shader_data_arrays(*c)
            want.append(oracle.render_procedural(p, obj, glob, oracle.from_params(m), W, H, 0)[0])
        sh2 = BandSharder(r, W, H, 0, inflight=2)
        for k, c in ((5, 0), (4, 1), (3, 0), (6, 1)):
            r.set_shader_data(*cams[c])
            f = sh2.run_frames(k)
            torch.cuda.current_stream().synchronize()
            assert sh2._launch2 is not None and r.get_option("shadow_defer_last") == 1
            assert np.array_equal(f.cpu().numpy(), want[c]), (k, c)
            assert all(np.array_equal(t.cpu().numpy(), want[c]) for t in sh2._targets2), (k, c)
        assert r.get_option("shadow_defer_kib") > 0


def test_row_partition_measured_and_one_rank_rebalance():
    """vr_row_partition_measured: with the model's own split and times equal
    to its estimate the split stays (to a strip); a range measured twice as
    slow shrinks and the others grow.  vr_shard_rebalance_rows over a one-rank
    RCCL communicator (the all-reduce of the times and the broadcast run for
    real) keeps the whole frame and the frames stay exact."""
    import sys
    sys.path.insert(0, ROOT)
    import volumetricrenderer_amd as vr
    from volumetricrenderer_amd.distributed import RcclBandPipeline
    W, H = 640, 360
    with vr.Renderer(0) as r:
        r.generate_volume(vr.volume_recipe_defaults(size=64))
        r.set_shader_data(*vr.reference_shader_data(W / H, 10.0, 20.0))
        r.set_march(vr.march_defaults())
        rb = r.row_partition(W, H, 4)
        same = r.row_partition_measured(W, H, rb, [1.0, 1.0, 1.0, 1.0])
        assert all(abs(a - b) <= 8 for a, b in zip(rb, same)), (rb, same)
        slow0 = r.row_partition_measured(W, H, rb, [2.0, 1.0, 1.0, 1.0])
        assert slow0[1] < rb[1] and slow0[0] == 0 and slow0[-1] == H, (rb, slow0)
        with pytest.raises(vr.VRError):
            r.row_partition_measured(W, H, [0, 7, H], [1.0, 1.0])   # not a multiple of 8
        pl = RcclBandPipeline(r, W, H, 1, band_rows=16, world=1, rank=0, partition="rows")
        try:
            pl.run_frames(3)
            assert pl.row_range == (0, H)
            assert pl.rebalance_rows(frames=4) == (0, H)
            pl.run_frames(3)
            pl.barrier()
            got = pl.frame()
            full = r.render(W, H, 1)
            torch.cuda.synchronize()
            assert np.array_equal(got.cpu().numpy(), full.cpu().numpy())
        finally:
            pl.close()


def test_timed_path_config5_native_loop_512(oracle):
    """Verdict r05 #2: the exact path bench.py times at N = 1 -- the native
    frame loop (RcclBandPipeline, world 1, default 2 render streams with the
    exchange on the render streams, frames_overlap on, which moves the auto
    split threshold) at BASELINE config 5's size: 512^3 recipe volume,
    1920 x 1080 x 128, RGBA8 UNORM, reference camera.  The frames of both
    render streams (3 and 4 frames run) equal the oracle's whole frame bit for
    bit, and the executed-step count of a render under the loop's split rule
    equals the oracle's (1.674e7)."""
    import sys
    sys.path.insert(0, ROOT)
    import volumetricrenderer_amd as vr
    from volumetricrenderer_amd.distributed import RcclBandPipeline
    W, H, fmt = 1920, 1080, vr.FMT_RGBA8_UNORM
    with vr.Renderer(0) as r:
        r.generate_volume(vr.scaled_recipe(512))
        vol = r.get_volume()
        osd, gsd = vr.reference_shader_data(1280.0 / 720.0)
        r.set_shader_data(osd, gsd)
        march = vr.march_defaults(max_steps=128)
        r.set_march(march)
        obj, glob = vr.shader_data_arrays(osd, gsd)
        ref, ref_steps = oracle.render(vol, obj, glob, oracle.from_params(march), W, H, oracle.FMT_RGBA8_UNORM)
        pl = RcclBandPipeline(r, W, H, fmt, band_rows=16, world=1, rank=0)
        try:
            assert pl.render_streams == 2 and not pl.compositor and pl.partition == "bands"
            for k in (3, 4):   # the last frame on render stream 0, then on stream 1
                ms = pl.run_frames(k, sample_every=1)
                assert ms > 0
                assert r.get_option("frames_overlap") == 1   # the loop's split rule is in force
                busy, span = pl.sampled_busy()
                assert 0 < busy <= span + 1e-3
                got = pl.frame()
                torch.cuda.synchronize()
                assert np.array_equal(got.cpu().numpy(), ref), k
            assert "col48" in r.kernel_variant
            counter = torch.zeros(1, dtype=torch.int64, device="cuda")
            r.render(W, H, fmt, step_counter=counter)
            torch.cuda.synchronize()
            assert int(counter.item()) == ref_steps
        finally:
            pl.close()
        assert r.get_option("frames_overlap") == 0   # restored with the pipeline
