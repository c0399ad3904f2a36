"""Render one configuration repeatedly (for rocprofv3 counter runs).

    python tools/prof_case.py --size 512 --layout 3 --schedule 2 --tpw 1 --frames 20
"""
import argparse
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import volumetricrenderer_amd as vr  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--size", type=int, default=512)
    ap.add_argument("--layout", type=int, default=0)
    ap.add_argument("--schedule", type=int, default=-1)
    ap.add_argument("--tpw", type=int, default=0)
    ap.add_argument("--frames", type=int, default=20)
    ap.add_argument("--wedges", type=int, default=0, help="regions schedule: wedges per XCD")
    ap.add_argument("--width", type=int, default=1920)
    ap.add_argument("--height", type=int, default=1080)
    ap.add_argument("--steps", type=int, default=128)
    ap.add_argument("--proc", action="store_true", help="procedural medium (config 2)")
    ap.add_argument("--shadow", type=int, default=0, help="procedural shadow steps (config 3: 8)")
    ap.add_argument("--slab", type=int, default=-1, help="LDS slab march (COL48): 1 on, 0 off")
    ap.add_argument("--proc-enum", type=int, default=-1, help="procedural sort: 1 region enumeration with shadows")
    ap.add_argument("--slab-cap", type=int, default=-1)
    ap.add_argument("--opt", action="append", default=[], help="vr option NAME=VALUE")
    a = ap.parse_args()
    with vr.Renderer(0) as r:
        if a.proc:
            r.set_procedural(shadow_steps=a.shadow)
        elif a.size <= 2:
            r.set_volume(np.full((a.size,) * 3 + (4,), 200, np.uint8))
        else:
            r.generate_volume(vr.scaled_recipe(a.size))
        if not a.proc:
            r.set_layout_preference(a.layout)
        if a.schedule >= 0:
            r.set_option("schedule", a.schedule)
        if a.slab >= 0:
            r.set_option("slab", a.slab)
        if a.proc_enum >= 0:
            r.set_option("proc_enum", a.proc_enum)
        if a.slab_cap >= 0:
            r.set_option("slab_cap", a.slab_cap)
        if a.wedges > 0:
            r.set_option("wedges", a.wedges)
        if a.tpw > 0:
            r.set_option("tiles_per_wave", a.tpw)
        for o in a.opt:
            k, v = o.split("=")
            r.set_option(k, int(v))
        osd, gsd = vr.reference_shader_data(a.width / a.height)
        r.set_shader_data(osd, gsd)
        r.set_march(vr.march_defaults(max_steps=a.steps))
        out = r.alloc_target(a.width, a.height, vr.FMT_RGBA8_UNORM)
        for _ in range(a.frames):
            r.render(a.width, a.height, vr.FMT_RGBA8_UNORM, out=out)
        torch.cuda.synchronize()
        print("variant", r.kernel_variant, "schedule", r.get_option("schedule"))


if __name__ == "__main__":
    main()
