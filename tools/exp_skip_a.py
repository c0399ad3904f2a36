"""Timing experiment: the config-5 frame with the A channel also made uniform
(its taps then cost no loads), to bound what a cheaper A-channel layout could
save.  Needs a libvr built with -DVR_UM_EXPERIMENT (VR_LIB)."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import volumetricrenderer_amd as vr  # noqa: E402

W, H = 1920, 1080
with vr.Renderer(0) as r:
    r.generate_volume(vr.scaled_recipe(512))
    osd, gsd = vr.reference_shader_data(1280 / 720)
    r.set_shader_data(osd, gsd)
    r.set_march(vr.march_defaults(max_steps=128))
    out = r.alloc_target(W, H, 1)

    def timeit(tag, frames=40):
        for _ in range(5):
            r.render(W, H, 1, out=out)
        ev = [torch.cuda.Event(enable_timing=True) for _ in range(2 * frames)]
        for i in range(frames):
            ev[2 * i].record()
            r.render(W, H, 1, out=out)
            ev[2 * i + 1].record()
        torch.cuda.synchronize()
        t = float(np.median([ev[2 * i].elapsed_time(ev[2 * i + 1]) for i in range(frames)]))
        print(f"{tag}: {r.kernel_variant} mask {r.get_option('uniform_mask')} {t:.4f} ms", flush=True)

    for rep in range(3):
        timeit("recipe")
    vol = r.get_volume()
    vol[..., 3] = 128
    r.set_volume(vol)
    for rep in range(3):
        timeit("A uniform too")
