"""Where config 2's time goes: the sorted procedural march at 1080p x 128 with
1-4 fBm octaves (each octave one Perlin evaluation per density sample), and
with the Worley term's frequency pushed so the pruned cube always decides
(worley_freq tiny: every sample in one cell)."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import volumetricrenderer_amd as vr  # noqa: E402

W, H = 1920, 1080
with vr.Renderer(0) as r:
    osd, gsd = vr.reference_shader_data(1280 / 720)
    r.set_shader_data(osd, gsd)
    r.set_march(vr.march_defaults(max_steps=128))
    out = r.alloc_target(W, H, 1)

    def timeit(tag, frames=30, **kw):
        r.set_procedural(**kw)
        for _ in range(5):
            r.render(W, H, 1, out=out)
        ev = [torch.cuda.Event(enable_timing=True) for _ in range(2 * frames)]
        for i in range(frames):
            ev[2 * i].record()
            r.render(W, H, 1, out=out)
            ev[2 * i + 1].record()
        torch.cuda.synchronize()
        t = float(np.median([ev[2 * i].elapsed_time(ev[2 * i + 1]) for i in range(frames)]))
        print(f"{tag}: {t:.4f} ms", flush=True)

    for rep in range(2):
        for o in (0, 1, 2, 3, 4):
            timeit(f"octaves {o}", octaves=o)
        timeit("octaves 4, shadow 8", octaves=4, shadow_steps=8)
        timeit("octaves 0, shadow 8", octaves=0, shadow_steps=8)
