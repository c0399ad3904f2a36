"""Frames in flight on one GPU (verdict-free experiment, round 4): config 5
frames rendered back to back on one stream into one target, against two
streams alternating two targets (frame i+1's waves fill the SIMDs during
frame i's tail, as the reference's 2 frames in flight, VulkanRenderer.cpp:13,
allow).  Prints ms per frame of each, interleaved rounds."""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import volumetricrenderer_amd as vr  # noqa: E402


def main():
    W, H, K = 1920, 1080, 40
    with vr.Renderer(0) as r:
        r.generate_volume(vr.scaled_recipe(int(sys.argv[1]) if len(sys.argv) > 1 else 512))
        osd, gsd = vr.reference_shader_data(1280 / 720)
        r.set_shader_data(osd, gsd)
        r.set_march(vr.march_defaults(max_steps=128))
        s0, s1 = torch.cuda.Stream(), torch.cuda.Stream()
        t0, t1 = r.alloc_target(W, H, 1), r.alloc_target(W, H, 1)
        l0 = r.prepare_render(W, H, 1, t0, stream=s0)
        l1 = r.prepare_render(W, H, 1, t1, stream=s1)
        for _ in range(5):
            with torch.cuda.stream(s0):
                l0()
            with torch.cuda.stream(s1):
                l1()
        torch.cuda.synchronize()
        for rnd in range(4):
            for mode in ("one", "two", "two_s1only"):
                torch.cuda.synchronize()
                t = time.perf_counter()
                for i in range(K):
                    if mode == "one":
                        with torch.cuda.stream(s0):
                            l0()
                    elif mode == "two":
                        with torch.cuda.stream(s0 if i % 2 == 0 else s1):
                            (l0 if i % 2 == 0 else l1)()
                    else:
                        with torch.cuda.stream(s1):
                            l1()
                torch.cuda.synchronize()
                el = (time.perf_counter() - t) / K * 1e3
                print(f"round {rnd} {mode}: {el:.4f} ms/frame", flush=True)


if __name__ == "__main__":
    main()
