"""Frame period of one rank's share rendered on 1-4 alternating streams
(prepare_render launchers, no exchange): does a third frame in flight help?"""
import os, sys
import numpy as np, torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))))
import volumetricrenderer_amd as vr
for size, W, H, S, stride, first in ((512, 1920, 1080, 128, 7, 0), (128, 3840, 2160, 256, 8, 1), (512, 1920, 1080, 128, 1, 0)):
    with vr.Renderer(0) as r:
        r.generate_volume(vr.scaled_recipe(size))
        r.set_shader_data(*vr.reference_shader_data(1280 / 720))
        r.set_march(vr.march_defaults(max_steps=S))
        r.set_option("frames_overlap", 1)
        fmt = vr.FMT_R8_UNORM if hasattr(vr, "FMT_R8_UNORM") else 3
        for ns in (1, 2, 3, 4):
            streams = [torch.cuda.Stream() for _ in range(ns)]
            outs = [r.alloc_target(W, H, 3, 16, stride, first) for _ in range(ns)]
            ls = [r.prepare_render(W, H, 3, outs[k], 16, stride, first, stream=streams[k]) for k in range(ns)]
            for i in range(300):
                ls[i % ns]()
            torch.cuda.synchronize()
            res = []
            for rnd in range(3):
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                cur = torch.cuda.current_stream()
                e0.record()
                for st in streams:
                    st.wait_stream(cur)
                for i in range(200):
                    ls[i % ns]()
                for st in streams:
                    cur.wait_stream(st)
                e1.record()
                torch.cuda.synchronize()
                res.append(e0.elapsed_time(e1) / 200)
            print(f"{size}^3 {W}x{H}x{S} bands16 stride {stride} first {first}: {ns} streams {np.median(res):.4f} ms/frame", flush=True)
