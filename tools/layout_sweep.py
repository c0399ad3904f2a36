"""Time the march kernel for each volume layout, interleaved in one process.

    python tools/layout_sweep.py [--sizes 128,512] [--rounds 5] [--frames 10]

Prints median ms per frame and nominal Mray/s, and checks that every layout
produces the same image as the first one.
"""
import argparse
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import volumetricrenderer_amd as vr  # noqa: E402

NAMES = {1: "planar", 2: "brick5", 3: "brick8", 4: "brick16", 5: "corner8", 6: "brick4", 7: "zpair", 8: "brick448", 9: "brick488", 10: "brick4816", 11: "brick41616", 12: "brick4832", 13: "brick4864", 14: "cornerh", 15: "col48", 16: "col48z"}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--sizes", default="128,512")
    ap.add_argument("--layouts", default="2,3,4,5,1")
    ap.add_argument("--variants", default="",
                    help="comma list of layout:schedule:waves_per_simd|tiles_per_wave[:wedges], overrides --layouts")
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--frames", type=int, default=10)
    ap.add_argument("--width", type=int, default=1920)
    ap.add_argument("--height", type=int, default=1080)
    ap.add_argument("--steps", type=int, default=128)
    ap.add_argument("--phi", type=float, default=0.0, help="camera orbit angles (deg), to check view dependence")
    ap.add_argument("--theta", type=float, default=0.0)
    ap.add_argument("--no-check", action="store_true", help="skip the cross-layout image check (timing builds)")
    args = ap.parse_args()
    W, H, S = args.width, args.height, args.steps
    if args.variants:
        layouts = [tuple(int(v) for v in x.split(":")) for x in args.variants.split(",")]
    else:
        layouts = [(int(x), 1, 4) for x in args.layouts.split(",")]

    def apply(r, lay):
        r.set_layout_preference(lay[0])
        r.set_option("schedule", lay[1])
        if lay[1] == 1 and lay[2] > 0:
            r.set_option("waves_per_simd", lay[2])
        r.set_option("tiles_per_wave", lay[2] if lay[1] in (2, 4, 5) else 0)
        if lay[1] == 5:
            r.set_option("wedges", lay[3] if len(lay) > 3 else 1)

    def name(lay):
        return f"{NAMES[lay[0]]}/{['static', 'queue', 'strided', 'xcdrows', 'rings', 'regions'][lay[1]]}{lay[2] if lay[1] else ''}{'w%d' % lay[3] if len(lay) > 3 else ''}"
    res = {}
    with vr.Renderer(0) as r:
        osd, gsd = vr.reference_shader_data(W / H, args.phi, args.theta)
        r.set_shader_data(osd, gsd)
        r.set_march(vr.march_defaults(max_steps=S))
        for n in [int(x) for x in args.sizes.split(",")]:
            if n <= 2:
                r.set_volume(np.full((n, n, n, 4), 200, np.uint8))
            else:
                r.generate_volume(vr.scaled_recipe(n))
            out = r.alloc_target(W, H, vr.FMT_RGBA8_UNORM)
            ref = None
            times = {lay: [] for lay in layouts}
            for lay in layouts:  # build + parity
                apply(r, lay)
                img = r.render(W, H, vr.FMT_RGBA8_UNORM, out=out).cpu().numpy()
                if ref is None:
                    ref = img
                assert args.no_check or np.array_equal(img, ref), f"layout {lay} differs at N={n}"
            for _ in range(args.rounds):
                for lay in layouts:
                    apply(r, lay)
                    r.render(W, H, vr.FMT_RGBA8_UNORM, out=out)
                    ev = [torch.cuda.Event(enable_timing=True) for _ in range(args.frames + 1)]
                    ev[0].record()
                    for k in range(args.frames):
                        r.render(W, H, vr.FMT_RGBA8_UNORM, out=out)
                        ev[k + 1].record()
                    torch.cuda.synchronize()
                    times[lay] += [ev[k].elapsed_time(ev[k + 1]) for k in range(args.frames)]
            for lay in layouts:
                t = float(np.median(times[lay]))
                key = f"N{n}_{name(lay)}"
                res[key] = {"ms": round(t, 4), "min_ms": round(float(np.min(times[lay])), 4),
                            "mray_s": round(W * H * S / (t * 1e-3) / 1e6, 1), "variant": None}
                print(f"{key:>24}: median {t:.4f} ms  min {np.min(times[lay]):.4f} ms  "
                      f"{W * H * S / (t * 1e-3) / 1e6:,.0f} Mray/s", flush=True)
            r.set_layout_preference(0)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
