"""Host cost per frame of the native frame loop (libvr_shard, vr_shard_run):
a one-rank RCCL communicator on a tiny frame, so the GPU work is negligible
and the wall time per frame is the host's (render launch, RCCL group,
assembly launch, events).  Also a plain vr_render loop for comparison.

    python tools/shard_overhead.py [--frames 2000] [--size 64]
"""
import argparse
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import volumetricrenderer_amd as vr  # noqa: E402
from volumetricrenderer_amd.distributed import RcclBandPipeline  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--frames", type=int, default=2000)
    ap.add_argument("--size", type=int, default=64)
    a = ap.parse_args()
    W = H = a.size
    with vr.Renderer(0) as r:
        r.generate_volume(vr.volume_recipe_defaults(size=32))
        osd, gsd = vr.reference_shader_data(1.0)
        r.set_shader_data(osd, gsd)
        r.set_march(vr.march_defaults(max_steps=8))
        out = r.render(W, H, 1)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(a.frames):
            r.render(W, H, 1, out=out)
        torch.cuda.synchronize()
        t_render = (time.perf_counter() - t0) / a.frames * 1e6
        pl = RcclBandPipeline(r, W, H, 1, band_rows=16, world=1, rank=0)
        try:
            pl.run_frames(10)
            pl.barrier()
            t0 = time.perf_counter()
            pl.run_frames(a.frames)
            t_enq = (time.perf_counter() - t0) / a.frames * 1e6
            pl.barrier()
            t_all = (time.perf_counter() - t0) / a.frames * 1e6
            t0 = time.perf_counter()
            for _ in range(200):
                pl.barrier()
            t_bar = (time.perf_counter() - t0) / 200 * 1e6
        finally:
            pl.close()
    print(f"{W}x{H}: vr_render from Python {t_render:.1f} us/frame; native loop enqueue {t_enq:.1f} us/frame, "
          f"to completion {t_all:.1f} us/frame; vr_shard_barrier {t_bar:.1f} us (one rank)")


if __name__ == "__main__":
    main()
