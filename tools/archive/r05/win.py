"""Where the N = 1 bench window loses time against the rehearsal: the native
loop's frames timed with/without sampled events, with/without the RCCL barrier."""
import os, sys, time
import numpy as np, torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))))
import volumetricrenderer_amd as vr
from volumetricrenderer_amd.distributed import RcclBandPipeline
W, H = 1920, 1080
with vr.Renderer(0) as r:
    r.generate_volume(vr.scaled_recipe(512))
    r.set_shader_data(*vr.reference_shader_data(1280 / 720))
    r.set_march(vr.march_defaults(max_steps=128))
    st = torch.cuda.current_stream()
    p = RcclBandPipeline(r, W, H, vr.FMT_RGBA8_UNORM, band_rows=16, world=1, rank=0)
    p.run_frames(8); p.barrier(st)
    res = {}
    for rnd in range(3):
        for name, frames, samp, bar in (("bench50", 50, 4, True), ("nosamp50", 50, 0, True), ("nobar50", 50, 0, False),
                                         ("events100", 100, 0, False), ("bench100", 100, 4, True)):
            p.run_frames(3); p.barrier(st)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            t0 = time.perf_counter(); e0.record()
            p.run_frames(frames, stream=st, sample_every=samp)
            e1.record()
            if bar:
                p.barrier(st)
            torch.cuda.synchronize()
            el = time.perf_counter() - t0
            res.setdefault(name, []).append((el / frames * 1e3, e0.elapsed_time(e1) / frames))
    for k, v in res.items():
        print(k, "wall ms/frame", " ".join(f"{a:.4f}" for a, _ in v), " events", " ".join(f"{b:.4f}" for _, b in v), flush=True)
    p.close()
