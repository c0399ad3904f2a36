"""Debug: deferred shadow passes vs the in-wave compaction on single frames:
repeat renders of one frame, several sizes / cameras / step counts."""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))
import volumetricrenderer_amd as vr  # noqa: E402

r = vr.Renderer()
r.set_procedural(shadow_steps=8)
for W, H, ms, phi, th in [(160, 96, 64, 1.6, 0.0), (160, 96, 64, 20.0, 15.0), (128, 72, 128, 20.0, 15.0),
                          (128, 72, 128, 1.6, 0.0), (160, 96, 128, 1.6, 0.0), (64, 64, 64, 1.6, 0.0),
                          (200, 150, 64, 1.6, 0.0)]:
    r.set_march(vr.march_defaults(max_steps=ms))
    osd, gsd = vr.reference_shader_data(W / H, phi, th)
    r.set_shader_data(osd, gsd)
    outs = {}
    for defer in (0, 1, 1, 1):
        r.set_option("shadow_defer", defer)
        img = r.render(W, H, 0)
        torch.cuda.synchronize()
        outs.setdefault(defer, []).append(img[..., 0].cpu().numpy())
    ref = outs[0][0]
    line = []
    for k, img in enumerate(outs[1]):
        bad = np.argwhere(img != ref)
        line.append(len(bad))
        if k == 0 and len(bad):
            ys, xs = bad[:, 0], bad[:, 1]
            rat = img[img != ref] / np.maximum(ref[img != ref], 1e-30)
            print(f"   rows {ys.min()}-{ys.max()} cols {xs.min()}-{xs.max()} ratio min {rat.min():.3f} "
                  f"med {np.median(rat):.3f} max {rat.max():.3f} first {bad[:6].tolist()}")
    print(f"W={W} H={H} ms={ms} phi={phi} th={th}: bad per repeat {line}", flush=True)
