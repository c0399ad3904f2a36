"""Per-wave timeline of one regions-schedule march launch (timing build).

    make -C volumetricrenderer_amd/csrc timeline
    VR_LIB=volumetricrenderer_amd/libvr_tl.so python tools/timeline.py [--size 512] [--layout 12]

Each wave of the launch records its start and end (s_memrealtime, 100 MHz),
its XCD and its executed lane-steps (vr_march_kernels.h VR_TIMELINE).  Prints
the launch span, the longest wave, the number of waves resident over time
and per-XCD spans: whether the frame is bound by throughput (many waves to
the end) or by the critical path of its longest rays (a tail of few waves).
"""
import argparse
import ctypes
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import volumetricrenderer_amd as vr  # noqa: E402
from volumetricrenderer_amd import _lib  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--size", type=int, default=512)
    ap.add_argument("--layout", type=int, default=0)
    ap.add_argument("--split", type=int, default=1)
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--json", default="")
    ap.add_argument("--opt", action="append", default=[], help="extra vr_set_option name=value")
    ap.add_argument("--width", type=int, default=1920)
    ap.add_argument("--height", type=int, default=1080)
    ap.add_argument("--steps", type=int, default=128)
    ap.add_argument("--bands", type=int, default=1, help="render rank 0's 16-row bands of N (a 1/N frame share)")
    a = ap.parse_args()
    lib = _lib.load()
    lib.vr_timeline_fetch.argtypes = [ctypes.c_void_p, ctypes.c_int]
    lib.vr_timeline_fetch_c8.argtypes = [ctypes.c_void_p, ctypes.c_int]   # the CORNER8 / CORNERH unit
    W, H = a.width, a.height
    band = dict(band_rows=16, band_stride=a.bands, band_first=0) if a.bands > 1 else {}
    out_all = {}
    with vr.Renderer(0) as r:
        r.generate_volume(vr.scaled_recipe(a.size))
        r.set_layout_preference(a.layout)
        r.set_option("split", a.split)
        for kv in a.opt:
            k, v = kv.split("=")
            r.set_option(k, int(v))
        osd, gsd = vr.reference_shader_data(1280 / 720)
        r.set_shader_data(osd, gsd)
        r.set_march(vr.march_defaults(max_steps=a.steps))
        out = r.alloc_target(W, H, vr.FMT_RGBA8_UNORM, **band)
        for _ in range(5):
            r.render(W, H, vr.FMT_RGBA8_UNORM, out=out, **band)
        torch.cuda.synchronize()
        ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
        ev[0].record()
        for _ in range(20):
            r.render(W, H, vr.FMT_RGBA8_UNORM, out=out, **band)
        ev[1].record()
        torch.cuda.synchronize()
        print(json.dumps({"opts": a.opt, "split": a.split, "ms_per_frame_20": round(ev[0].elapsed_time(ev[1]) / 20, 4)}))
        for rep in range(a.reps):
            assert lib.vr_timeline_clear() == 0 and lib.vr_timeline_clear_c8() == 0
            r.render(W, H, vr.FMT_RGBA8_UNORM, out=out, **band)
            torch.cuda.synchronize()
            buf = np.zeros((1 << 16, 3), np.uint64)
            assert lib.vr_timeline_fetch(buf.ctypes.data, 1 << 16) == 0
            if not (buf[:, 1] > 0).any():
                assert lib.vr_timeline_fetch_c8(buf.ctypes.data, 1 << 16) == 0
            rec = buf[buf[:, 1] > 0]
            t0 = rec[:, 0].min()
            s = (rec[:, 0] - t0).astype(np.float64) / 100.0   # us
            e = (rec[:, 1] - t0).astype(np.float64) / 100.0
            steps = (rec[:, 2] >> np.uint64(24)).astype(np.int64)
            xcd = (rec[:, 2] & np.uint64(255)).astype(np.int64)
            hw = ((rec[:, 2] >> np.uint64(8)) & np.uint64(0xfff)).astype(np.int64)   # HW_ID [15:4]
            simd = xcd * 4096 + hw   # one SIMD of one CU of one XCD
            span = e.max()
            dur = e - s
            grid = np.linspace(0, span, 41)
            resident = [int(((s <= t) & (e > t)).sum()) for t in grid[:-1]]
            work = steps > 0
            res = {
                "variant": r.kernel_variant, "waves": int(len(rec)), "waves_with_work": int(work.sum()),
                "span_us": round(span, 2),
                "longest_wave_us": round(dur.max(), 2),
                "longest_wave_steps_per_lane": round(steps[dur.argmax()] / 64, 1),
                "median_wave_us": round(float(np.median(dur[work])), 2),
                "last_start_us": round(s.max(), 2),
                "end_p50_p90_p99_us": [round(float(np.percentile(e, q)), 2) for q in (50, 90, 99)],
                "resident_waves_over_time": resident,
                "xcd_end_us": [round(float(e[xcd == x].max()), 2) for x in range(8)],
                "xcd_steps": [int(steps[xcd == x].sum()) for x in range(8)],
                "us_per_step_longest": round(dur.max() / max(1, steps[dur.argmax()] / 64), 3),
            }
            # per SIMD: waves, the busy span (first start to last end) and the
            # summed lane-steps; the SIMD of the longest wave and the busiest ones
            ids, inv = np.unique(simd, return_inverse=True)
            nw = np.bincount(inv)
            sstep = np.bincount(inv, weights=steps)
            send = np.zeros(len(ids)); np.maximum.at(send, inv, e)
            lw = int(dur.argmax())
            mates = (inv == inv[lw])
            res.update({
                "simds_used": int(len(ids)),
                "waves_per_simd_p50_max": [int(np.median(nw)), int(nw.max())],
                "simd_steps_p50_p99_max": [int(np.median(sstep)), int(np.percentile(sstep, 99)), int(sstep.max())],
                "simd_end_p50_p99_max_us": [round(float(np.median(send)), 2), round(float(np.percentile(send, 99)), 2),
                                            round(float(send.max()), 2)],
                "longest_wave_simd": {"waves": int(mates.sum()), "steps_per_lane": [round(float(v) / 64, 1) for v in steps[mates]],
                                      "start_end_us": [[round(float(a_), 2), round(float(b_), 2)] for a_, b_ in zip(s[mates], e[mates])]},
                "slowest_simd_steps_rank": int((sstep > sstep[inv[int(e.argmax())]]).sum()),
            })
            print(json.dumps(res))
            out_all[f"rep{rep}"] = res
    if a.json:
        with open(a.json, "w") as f:
            json.dump(out_all, f, indent=1)


if __name__ == "__main__":
    main()
