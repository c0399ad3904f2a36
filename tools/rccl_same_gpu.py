"""The native frame loop's connected path (libvr_shard over RCCL) with N real
ranks -- N processes that all render on GPU 0.  The driver's 8-GPU run is the
first place RCCL point-to-point runs across devices; this rehearses the same
code (communicator init and split, grouped send/receive on the render
streams, rank 0 rendering in place beside the receives, the compositor's slot
offsets, lead rows, row ranges) on the one GPU a gpurun box has, if RCCL
accepts two ranks on one device.  Rank 0 compares every case's assembled
frame with a plain one-GPU render of the same camera, bit for bit.

    python tools/rccl_same_gpu.py [--ranks 2] [--cases all]
"""
import argparse
import os
import socket
import sys
import time

import torch
import torch.distributed as dist
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

CASES = {
    # name: RcclBandPipeline keyword arguments
    "bands": dict(render_streams=2),
    "bands_plain": dict(render_streams=2, serpentine=False),
    "bands_1stream": dict(render_streams=1),
    "bands_commstream": dict(render_streams=2, exchange_on_render=False),
    "compositor": dict(render_streams=2, compositor=True, lead_pct=None),
    "compositor_lead": dict(render_streams=2, compositor=True, lead_rows=48),
    "rows": dict(render_streams=3, partition="rows"),
    "rows_compositor": dict(render_streams=3, partition="rows", compositor=True),
}


def worker(rank, world, port, cases, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    sys.path.insert(0, ROOT)
    import volumetricrenderer_amd as vr
    from volumetricrenderer_amd.distributed import RcclBandPipeline
    dist.init_process_group("gloo", rank=rank, world_size=world)
    out = []
    try:
        W, H = 640, 360
        with vr.Renderer(0) as r:
            r.generate_volume(vr.volume_recipe_defaults(size=128))
            r.set_march(vr.march_defaults())
            cams = [vr.reference_shader_data(W / H, 7.0 * i, 0.5 * i) for i in range(12)]
            r.set_shader_data(*cams[0])
            for name in cases:
                kw = CASES[name]
                t0 = time.time()
                pl = RcclBandPipeline(r, W, H, vr.FMT_RGBA8_UNORM, band_rows=16, world=world, rank=rank,
                                      timeout_s=60, **kw)
                try:
                    pl.run_frames(6, cameras=cams[:6])
                    pl.run_frames(6, cameras=cams[6:])
                    pl.barrier()
                    if rank == 0:
                        got = pl.frame().clone()
                        r.set_shader_data(*cams[11])
                        want = r.render(W, H, vr.FMT_RGBA8_UNORM)
                        torch.cuda.synchronize()
                        ok = torch.equal(got, want)
                        out.append(f"{name}: {'exact' if ok else 'MISMATCH'} (serpentine {pl.serpentine}, "
                                   f"compositor {pl.compositor}, lead rows {pl.lead_rows}, partition {pl.partition}, "
                                   f"{time.time() - t0:.1f} s)")
                finally:
                    pl.close()
                dist.barrier()
    except Exception as e:   # report, so the parent does not wait for a message that never comes
        out.append(f"rank {rank}: {type(e).__name__}: {e}")
    q.put((rank, out))
    dist.destroy_process_group()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--ranks", type=int, default=2)
    ap.add_argument("--cases", default="all")
    a = ap.parse_args()
    cases = list(CASES) if a.cases == "all" else a.cases.split(",")
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    ps = [ctx.Process(target=worker, args=(k, a.ranks, port, cases, q)) for k in range(a.ranks)]
    for p in ps:
        p.start()
    res = {}
    for _ in ps:
        k, out = q.get(timeout=600)
        res[k] = out
    for p in ps:
        p.join(timeout=60)
    bad = False
    for k in sorted(res):
        for line in res[k]:
            print(f"[rank {k}] {line}", flush=True)
            bad |= "MISMATCH" in line or "Error" in line
    print("all exact" if not bad else "FAILED", flush=True)
    sys.exit(1 if bad else 0)


if __name__ == "__main__":
    main()
