"""Host (CPU) cost per call of the per-frame entry points, on a tiny frame
whose GPU time is negligible: the floor that multi-GPU strong scaling of a
0.2 ms frame runs into."""
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import volumetricrenderer_amd as vr  # noqa: E402


def per_call(fn, n=3000):
    for _ in range(50):
        fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(n):
        fn()
    t1 = time.perf_counter()
    torch.cuda.synchronize()
    return (t1 - t0) / n * 1e6, (time.perf_counter() - t0) / n * 1e6


def main():
    with vr.Renderer(0) as r:
        r.set_volume(np.full((8, 8, 8, 4), 100, np.uint8))
        osd, gsd = vr.reference_shader_data(1.0)
        r.set_shader_data(osd, gsd)
        r.set_march(vr.march_defaults(max_steps=4))
        out = r.alloc_target(64, 64, vr.FMT_RGBA8_UNORM)
        print("render      host %.1f us/call, wall %.1f us/call" % per_call(lambda: r.render(64, 64, 1, out=out)))
        g = torch.zeros((4, 16, 64, 4), dtype=torch.uint8, device="cuda")
        fr = torch.zeros((64, 64, 4), dtype=torch.uint8, device="cuda")
        print("assemble    host %.1f us/call, wall %.1f us/call" % per_call(lambda: r.assemble_bands(g, 4, 64, 64, 16, frame=fr)))
        ev = torch.cuda.Event()
        print("event rec   host %.1f us/call, wall %.1f us/call" % per_call(lambda: ev.record()))
        x = torch.zeros(16, device="cuda")
        print("torch add_  host %.1f us/call, wall %.1f us/call" % per_call(lambda: x.add_(1)))


if __name__ == "__main__" and len(sys.argv) == 1:
    main()


def gather_overhead():
    """Host cost of one async torch.distributed gather on the RCCL backend
    (world 1: the collective's host path, no peers)."""
    import torch.distributed as dist
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ.setdefault("MASTER_PORT", "29533")
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda", 0))
    x = torch.zeros(1 << 20, dtype=torch.uint8, device="cuda")
    g = [torch.empty_like(x)]

    def one():
        w = dist.gather(x, gather_list=g, dst=0, async_op=True)
        w.wait()
    print("gather+wait host %.1f us/call, wall %.1f us/call" % per_call(one, 1000))
    dist.destroy_process_group()


if __name__ == "__main__" and len(sys.argv) > 1 and sys.argv[1] == "gather":
    gather_overhead()
