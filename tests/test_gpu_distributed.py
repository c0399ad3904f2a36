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


@pytest.mark.parametrize("fmt,band_rows", [(1, 16), (0, 8)])
def test_rccl_pipeline_one_rank(fmt, band_rows):
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
        pl = RcclBandPipeline(r, W, H, fmt, band_rows=band_rows, world=1, rank=0)
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


@pytest.mark.parametrize("world,band_rows,fmt,W", [(2, 16, 1, 500), (3, 16, 0, 500), (8, 16, 1, 500), (5, 7, 1, 500),
                                                   (3, 16, 2, 499), (4, 16, 0, 499)])
def test_native_pipeline_loopback_ranks(world, band_rows, fmt, W):
    """The native frame loop's N-rank data layout (grey band sets in gather
    slots of rank 0's row count, expanded by vr_assemble_frame) with every
    rank's bands rendered by this one process: the frame equals a plain
    render.  Width 499 takes the per-pixel expansion, 500 the 4-pixel one."""
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
        pl = RcclBandPipeline(r, W, H, fmt, band_rows=band_rows, world=world, rank=0, loopback=True)
        try:
            assert pl.rows_per_rank == vr.band_rows_packed(H, band_rows, world, 0)
            pl.run_frames(3)
            pl.barrier()   # loopback: a stream synchronisation
            got = pl.frame()
            full = r.render(W, H, fmt)
            torch.cuda.synchronize()
            assert np.array_equal(got.cpu().numpy(), full.cpu().numpy())
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
