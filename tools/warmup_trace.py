"""Per-frame durations from a cold start, with the GPU's clock sampled beside
them (verdict r05 #1: attribute the driver's --warmup 5 line against the
builder's 300-frame one).

For each phase, frames are queued back to back on one stream with a HIP event
after every frame; the frame period is the distance between consecutive end
events.  A separate process samples the card's clock, power and DPM files (hwmon
freq1_input / power1_*, pp_dpm_sclk / fclk / mclk / socclk) every ~1 ms on the host clock, anchored to
the GPU timeline by a synchronize before each phase.  The phases follow
bench.py's order: config 5 from process start, then config 4's host set-up
(new renderer, volume, first render with its layout / region-list build),
its frames, an idle gap, and config 4 again.

    python tools/warmup_trace.py [--frames 400] [--idle 1.0] > trace.txt
"""
import argparse
import glob
import json
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import volumetricrenderer_amd as vr  # noqa: E402


def our_card():
    """The DRM device directory of cuda:0 (matched by PCI bus id), or None."""
    try:
        pr = torch.cuda.get_device_properties(0)
        bus = getattr(pr, "pci_bus_id", None)
        dom = getattr(pr, "pci_domain_id", 0)
        dev = getattr(pr, "pci_device_id", None)
        if bus is None:
            return None
        for d in sorted(glob.glob("/sys/class/drm/card*/device")):
            addr = os.path.basename(os.path.realpath(d))   # 0000:75:00.0
            parts = addr.replace(".", ":").split(":")
            if len(parts) == 4 and int(parts[0], 16) == dom and int(parts[1], 16) == bus and \
                    (dev is None or int(parts[2], 16) == dev):
                return d
    except Exception:   # pragma: no cover - best effort
        pass
    return None


def clock_files(card):
    """Clock / power files of one card (all cards when it is unknown)."""
    dirs = [card] if card else sorted(glob.glob("/sys/class/drm/card*/device"))
    files = []
    for d in dirs:
        cands = glob.glob(d + "/hwmon/hwmon*/freq1_input") + glob.glob(d + "/hwmon/hwmon*/power1_average") + \
            glob.glob(d + "/hwmon/hwmon*/power1_input") + \
            [d + "/pp_dpm_sclk", d + "/pp_dpm_fclk", d + "/pp_dpm_mclk", d + "/pp_dpm_socclk", d + "/pp_dpm_dcefclk",
             d + "/gpu_busy_percent"]
        for f in cands:
            try:
                with open(f) as fh:
                    fh.read()
                files.append(f)
            except OSError:
                pass
    return files


def read_clock(f):
    with open(f) as fh:
        s = fh.read()
    if f.endswith("freq1_input"):
        return int(s) / 1e6   # Hz -> MHz
    if "power1" in f:
        return int(s) / 1e6   # uW -> W
    if f.endswith("gpu_busy_percent"):
        return float(s)
    for ln in s.splitlines():   # "1: 2400Mhz *"
        if ln.rstrip().endswith("*"):
            return float(ln.split(":")[1].strip().split("M")[0])
    return float("nan")


def sampler_proc(files, path, stop_path):
    """A separate process (no GIL shared with the frame loop): samples every
    ~1 ms, one line per sample: host time (perf_counter, CLOCK_MONOTONIC) and
    the values."""
    with open(path, "w") as out:
        while not os.path.exists(stop_path):
            t = time.perf_counter()
            vals = []
            for f in files:
                try:
                    vals.append(read_clock(f))
                except (OSError, ValueError):
                    vals.append(float("nan"))
            out.write(json.dumps([t, vals]) + "\n")
            time.sleep(0.001)


class Sampler:
    def __init__(self, files, tmpdir):
        import multiprocessing as mp
        self.files = files
        self.keep = list(range(len(files)))   # the columns reported
        self.path = os.path.join(tmpdir, f"clk_{os.getpid()}.jsonl")
        self.stop_path = self.path + ".stop"
        self.p = mp.get_context("spawn").Process(target=sampler_proc, args=(files, self.path, self.stop_path),
                                                 daemon=True)
        self.p.start()

    @property
    def samples(self):
        out = []
        try:
            with open(self.path) as f:
                for ln in f:
                    try:
                        out.append(tuple(json.loads(ln)))
                    except ValueError:
                        pass
        except OSError:
            pass
        return out

    def close(self):
        open(self.stop_path, "w").close()
        self.p.join(timeout=5)


def phase(name, launch, frames, sampler, log):
    torch.cuda.synchronize()
    t_host0 = time.perf_counter()
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(frames + 1)]
    ev[0].record()
    for i in range(frames):
        launch()
        ev[i + 1].record()
    torch.cuda.synchronize()
    t_end = [ev[0].elapsed_time(e) for e in ev[1:]]   # ms from the phase start
    per = np.diff([0.0] + t_end)
    # clock samples inside the phase, on the GPU timeline (host time - anchor)
    cs = [(1e3 * (t - t_host0), v) for t, v in sampler.samples if t >= t_host0 and
          1e3 * (t - t_host0) <= t_end[-1] + 1.0] if sampler else []
    log.append({"phase": name, "frames": frames, "frame_ms": [round(float(x), 5) for x in per],
                "files": [sampler.files[j] for j in sampler.keep] if sampler else [],
                "clock": [(round(t, 3), [v[j] for j in sampler.keep]) for t, v in cs]})
    print(f"== {name}: {frames} frames, {t_end[-1]:.2f} ms", flush=True)
    edges = [0, 1, 2, 3, 5, 10, 20, 40, 80, 160, 320, frames]
    for a, b in zip(edges[:-1], edges[1:]):
        if a >= frames:
            break
        b = min(b, frames)
        seg = per[a:b]
        t_a, t_b = (t_end[a - 1] if a else 0.0), t_end[b - 1]
        clk = [v for t, v in cs if t_a <= t <= t_b]
        clk_s = ""
        if clk:
            arr = np.array(clk, dtype=float)
            clk_s = "  " + " ".join(f"{os.path.basename(sampler.files[j])}={np.nanmean(arr[:, j]):.0f}"
                                    f"[{np.nanmin(arr[:, j]):.0f},{np.nanmax(arr[:, j]):.0f}]"
                                    for j in sampler.keep)
        print(f"  frames {a:4d}-{b - 1:4d}  t {t_a:8.2f}-{t_b:8.2f} ms  mean {seg.mean():.4f}  "
              f"min {seg.min():.4f}  max {seg.max():.4f}{clk_s}", flush=True)
    return per


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--frames", type=int, default=400)
    ap.add_argument("--idle", type=float, default=1.0, help="seconds of idle GPU before the last phase")
    ap.add_argument("--json", default="", help="write every frame's period and the clock samples here")
    a = ap.parse_args()
    # the sampler starts before this process touches the GPU; it samples
    # every card's files, and the report keeps cuda:0's (matched by bus id)
    files = clock_files(None)
    sampler = Sampler(files, os.environ.get("TMPDIR", "/tmp")) if files else None
    while sampler and not sampler.samples and sampler.p.is_alive():
        time.sleep(0.05)
    card = our_card()
    if sampler and card:
        sampler.keep = [j for j, f in enumerate(files) if f.startswith(card + "/")]
    print("card:", card, "sampled files:", [files[j] for j in sampler.keep] if sampler else [], flush=True)
    log = []
    t0 = time.perf_counter()
    fmt = vr.FMT_RGBA8_UNORM
    osd, gsd = vr.reference_shader_data(1280.0 / 720.0)
    r5 = vr.Renderer(0)
    r5.generate_volume(vr.scaled_recipe(512))
    r5.set_shader_data(osd, gsd)
    r5.set_march(vr.march_defaults(max_steps=128))
    out5 = r5.alloc_target(1920, 1080, fmt)
    r5.render(1920, 1080, fmt, out=out5)
    print(f"config 5 set-up {1e3 * (time.perf_counter() - t0):.1f} ms ({r5.kernel_variant})", flush=True)
    phase("config 5 (512^3, 1080p x 128), cold process", r5.prepare_render(1920, 1080, fmt, out5), a.frames,
          sampler, log)

    def setup4():
        t1 = time.perf_counter()
        r4 = vr.Renderer(0)
        r4.generate_volume(vr.scaled_recipe(128))
        t2 = time.perf_counter()
        r4.set_shader_data(osd, gsd)
        r4.set_march(vr.march_defaults(max_steps=256))
        out4 = r4.alloc_target(3840, 2160, fmt)
        r4.render(3840, 2160, fmt, out=out4)
        torch.cuda.synchronize()
        t3 = time.perf_counter()
        print(f"config 4 set-up: renderer + volume {1e3 * (t2 - t1):.1f} ms, first render (layout, regions) "
              f"{1e3 * (t3 - t2):.1f} ms ({r4.kernel_variant})", flush=True)
        return r4, out4

    r4, out4 = setup4()
    phase("config 4 (128^3, 4K x 256) right after its set-up", r4.prepare_render(3840, 2160, fmt, out4), a.frames,
          sampler, log)
    time.sleep(a.idle)
    phase(f"config 4 after {a.idle:.1f} s idle", r4.prepare_render(3840, 2160, fmt, out4), a.frames, sampler, log)
    phase("config 5 after config 4 (hot GPU)", r5.prepare_render(1920, 1080, fmt, out5), a.frames, sampler, log)
    if sampler:
        sampler.close()
    if a.json:
        with open(a.json, "w") as f:
            json.dump(log, f)
    r4.close()
    r5.close()


if __name__ == "__main__":
    main()
