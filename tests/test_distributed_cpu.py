"""Multi-rank frame sharding on CPU (gloo, world_size 2 and 3).

The band plan and the gather to rank 0 are the ones bench.py runs over RCCL.
Here a CPU stand-in renders each rank's bands: the oracle, which is allowed
in tests, wrapped in the Renderer interface that BandSharder expects.  The
frame that rank 0 assembles must equal one full-frame oracle render.  The
HIP assembly kernel itself is covered in tests/test_gpu_parity.py.
"""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


class OracleRenderer:
    """CPU stand-in for volumetricrenderer_amd.Renderer (test only).  Grey
    formats 3-5 are the R channel of the RGBA formats 1, 2, 0."""

    RGBA_OF = {3: 1, 4: 2, 5: 0}

    def __init__(self, oracle, vol, obj, glob, march):
        self.o, self.vol, self.obj, self.glob, self.m = oracle, vol, obj, glob, march

    def alloc_target(self, width, height, fmt, band_rows=0, band_stride=1, band_first=0):
        from volumetricrenderer_amd.distributed import rows_for_rank
        rows = rows_for_rank(height, band_rows, band_stride, band_first) if band_rows else height
        shape = (rows, width) if fmt in self.RGBA_OF else (rows, width, 4)
        return torch.zeros(shape, dtype=torch.float32 if fmt in (0, 5) else torch.uint8)

    def render(self, width, height, fmt, out=None, band_rows=0, band_stride=1, band_first=0, step_counter=None):
        img, _ = self.o.render(self.vol, self.obj, self.glob, self.m, width, height, self.RGBA_OF.get(fmt, fmt),
                               band_rows=band_rows, band_stride=band_stride, band_first=band_first)
        if fmt in self.RGBA_OF:
            img = np.ascontiguousarray(img[..., 0])
        out[: img.shape[0]].copy_(torch.from_numpy(img))
        return out

    def set_volume(self, vol):
        self.vol = np.ascontiguousarray(vol, dtype=np.uint8)

    def assemble_frame(self, gathered, gfmt, nranks, width, height, band_rows, ffmt, frame=None):
        for y in range(height):
            b, r = divmod(y, band_rows)
            row = gathered[b % nranks, (b // nranks) * band_rows + r]
            if gfmt != ffmt:   # grey -> RGBA: G = B = R, A = 1 / 255
                alpha = 1.0 if ffmt == 0 else 255
                row = torch.stack([row, row, row, torch.full_like(row, alpha)], dim=-1)
            frame[y] = row
        return frame


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _share_worker(rank, world, port, W, H, q):
    """share_volume: only rank 0 holds the volume; after the broadcast every
    rank renders its bands from what it received."""
    import sys
    sys.path.insert(0, ROOT)
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import vr_oracle as oracle

    from volumetricrenderer_amd.distributed import BandSharder, share_volume
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        vol = np.random.default_rng(11).integers(0, 256, size=(18, 26, 22, 4), dtype=np.uint8)
        obj, glob = oracle.reference_shader_data(W / H, -30.0, 15.0)
        r = OracleRenderer(oracle, None, obj, glob, oracle.march(48))
        got = share_volume(r, vol if rank == 0 else None, rank=rank)
        same = bool(np.array_equal(got.numpy(), vol)) and bool(np.array_equal(r.vol, vol))
        frame = BandSharder(r, W, H, 0, band_rows=16, world=world, rank=rank).run_frames(1)
        if rank == 0:
            ref, _ = oracle.render(vol, obj, glob, oracle.march(48), W, H, 0)
            same = same and bool(np.array_equal(frame.numpy(), ref))
        q.put(("ok", same, rank))
    except Exception as e:  # pragma: no cover - surfaced by the assertion below
        q.put(("err", repr(e), rank))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_share_volume_from_rank0(world):
    """SURVEY.md sec. 8e collective (1) on the torch path: rank 0's volume
    reaches every rank (shape first, then the bytes) and the sharded frame
    equals a full-frame oracle render of it."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_share_worker, args=(rk, world, port, 80, 48, q)) for rk in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in procs]
    for p in procs:
        p.join(timeout=60)
    assert all(r[0] == "ok" and r[1] for r in res), res


def _bad_share_worker(rank, world, port, which, q):
    """Rank 0 passes a bad volume: every rank must raise, none may hang in
    the broadcast (the check used to come before it)."""
    import sys
    sys.path.insert(0, ROOT)
    from volumetricrenderer_amd.distributed import RcclBandPipeline, share_volume
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world, timeout=__import__("datetime").timedelta(seconds=60))
    try:
        bad = np.zeros((4, 4, 4, 3), dtype=np.uint8)   # three channels: not RGBA8
        try:
            if which == "torch":
                share_volume(None, bad if rank == 0 else None)   # rank from the group
            else:
                # the pipeline's Python side only; the bad volume is caught before any library call
                p = RcclBandPipeline.__new__(RcclBandPipeline)
                p.world, p.rank, p.group, p.loopback, p._h = world, rank, None, False, None
                p.share_volume(torch.from_numpy(bad) if rank == 0 else None)
            q.put(("no-raise", rank))
        except ValueError as e:
            q.put(("raised", rank, str(e)))
    except Exception as e:  # pragma: no cover - surfaced by the assertion below
        q.put(("err", rank, repr(e)))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("which", ["torch", "pipeline"])
def test_share_volume_bad_input_raises_on_every_rank(which):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_bad_share_worker, args=(rk, 2, port, which, q)) for rk in range(2)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in procs]
    for p in procs:
        p.join(timeout=60)
    assert sorted(r[1] for r in res) == [0, 1], res
    assert all(r[0] == "raised" for r in res), res


def _worker(rank, world, port, W, H, fmt, q):
    import sys
    sys.path.insert(0, ROOT)
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import vr_oracle as oracle

    from volumetricrenderer_amd.distributed import BandSharder
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        vol = np.random.default_rng(7).integers(0, 256, size=(24, 20, 28, 4), dtype=np.uint8)
        obj, glob = oracle.reference_shader_data(W / H, 25.0, -10.0)
        r = OracleRenderer(oracle, vol, obj, glob, oracle.march(64))
        sh = BandSharder(r, W, H, fmt, band_rows=16, world=world, rank=rank)
        assert sh.gfmt == {0: 5, 1: 3, 2: 4}[fmt]   # grey band sets travel
        frame = sh.run_frames(3)
        if rank == 0:
            ref, _ = oracle.render(vol, obj, glob, oracle.march(64), W, H, fmt)
            q.put(("ok", bool(np.array_equal(frame.numpy(), ref)), int(sh.my_rows)))
        else:
            q.put(("ok", True, int(sh.my_rows)))
    except Exception as e:  # pragma: no cover - surfaced by the assertion below
        q.put(("err", repr(e), 0))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,W,H,fmt", [(2, 96, 72, 0), (3, 64, 100, 0), (2, 80, 48, 1)])
def test_band_shard_gather_matches_full_frame(world, W, H, fmt):
    """Grey band sets (one value per pixel) gathered over gloo and expanded
    on rank 0 equal one full-frame oracle render, RGBA32F and RGBA8."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(rk, world, port, W, H, fmt, q)) for rk in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in procs]
    for p in procs:
        p.join(timeout=60)
    assert all(r[0] == "ok" for r in res), res
    assert all(r[1] for r in res), res
    rows = sorted(r[2] for r in res)
    assert sum(rows) >= H  # every frame row is rendered by some rank
