"""Per-frame figures of a `rocprofv3 --kernel-trace` run of bench.py, read from
its kernel_trace.csv (verdict r05 #1: the line's roofline must recompute from
the committed trace).

For each config of the default line, the march launches are found by kernel
name in dispatch order: the untimed counting passes, `--warmup` frames, then
the `--steps` timed frames.  Printed per config:

- wall per frame: the span from the first timed frame's first kernel start to
  the last timed frame's last kernel end, / steps (bench.py's ms_per_step also
  holds the barrier bracket, a few us);
- busy per frame: the union of the timed frames' kernel intervals / steps
  (the GPU time a frame holds the machine, overlapping launches counted once);
- mean launch duration (what rocprof's --stats average reports);
- per-frame periods across warm-up and window (end of frame i - end of frame i-1);
- with --line, the bench JSON: the roofline recomputed from the trace's busy
  time and wall time, against the line's.

    python tools/trace_frames.py TRACE.csv [--line bench.json] [--steps 20] [--warmup 5]
"""
import argparse
import csv
import json
import re

# the per-frame kernels of each config of the default line, and the untimed
# launches before its warm-up (bench.py: the step-counting passes)
CONFIGS = [
    # name, frame kernels (regex on the kernel name), counting passes, main kernel regex
    ("grid512", [r"march_regions_u<15,"], 1, r"march_regions_u<15,"),
    ("grid512_all_channels", [r"march_regions<15,"], 0, r"march_regions<15,"),
    ("grid4k", [r"march_regions_u<14,"], 1, r"march_regions_u<14,"),
    ("cloud", [r"march_proc_sorted<"], 3, r"march_proc_sorted<"),
    ("cloud_shadow", [r"march_proc_defer<", r"proc_shadow_scan", r"proc_shadow_map", r"proc_shadow_eval",
                      r"proc_shadow_resolve"], 3, r"march_proc_defer<"),
]


def load(path):
    rows = []
    with open(path) as f:
        for r in csv.DictReader(f):
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]))
    rows.sort()
    return rows


def union(iv):
    tot, cur_s, cur_e = 0, None, None
    for s, e in sorted(iv):
        if cur_e is None or s > cur_e:
            if cur_e is not None:
                tot += cur_e - cur_s
            cur_s, cur_e = s, e
        else:
            cur_e = max(cur_e, e)
    if cur_e is not None:
        tot += cur_e - cur_s
    return tot


def frames_of(rows, pats, main, skip):
    """Group the config's kernels into frames: frame i = main launch i and the
    other frame kernels dispatched after it, before main launch i+1."""
    mains = [k for k, r in enumerate(rows) if re.search(main, r[2])]
    frames = []
    for n, k in enumerate(mains):
        end = mains[n + 1] if n + 1 < len(mains) else len(rows)
        ks = [rows[k]] + [r for r in rows[k + 1:end] if any(re.search(p, r[2]) for p in pats) and not re.search(main, r[2])]
        frames.append(ks)
    return frames[skip:]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--line", default="")
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--periods", action="store_true", help="print every frame's period")
    a = ap.parse_args()
    rows = load(a.trace)
    line = None
    if a.line:
        with open(a.line) as f:
            line = json.loads(f.read().strip().splitlines()[-1])
    for name, pats, skip, main_re in CONFIGS:
        fr = frames_of(rows, pats, main_re, skip)
        if len(fr) < a.warmup + a.steps:
            print(f"{name}: {len(fr)} frames in the trace, fewer than warm-up + steps; skipped")
            continue
        # frame order per config (bench.py): [clock_warm frames] [--warmup] [timed window] ...
        # grid512: then the busy pass (K frames); grid4k: then the two-in-flight probe
        cw = 0
        if line is not None:
            obj = line if name == "grid512" else line.get("other_configs", {}).get(name)
            if obj and obj.get("clock_warm"):
                cw = obj["clock_warm"]["frames"]
        if name == "grid512_all_channels":
            first = a.warmup
        elif obj and obj.get("frames_in_flight") == 2:
            # config 2: the one-stream window and its warm-up come first, then the
            # two-in-flight window the line reports (bench.py other_config)
            first = cw + 2 * a.warmup + a.steps
        else:
            first = cw + a.warmup
        gated = None
        if name == "grid512" and obj and "gpu_ms_per_frame_gated" in obj.get("roofline", {}):
            # bench.py: the same K frames again, gated, after the window (the roofline's time)
            gf = obj["roofline"].get("gate_frames", 0)   # frames of the loop before the gated ones
            g = fr[first + a.steps + gf:first + 2 * a.steps + gf]   # (the frame check's render comes after the passes)
            giv = [(s_, e_) for f in g for (s_, e_, _) in f]
            gated = (max(e_ for _, e_ in giv) - min(s_ for s_, _ in giv)) / a.steps / 1e6
        timed = fr[first:first + a.steps]
        iv = [(s, e) for f in timed for (s, e, _) in f]
        t_first, t_last = min(s for s, _ in iv), max(e for _, e in iv)
        wall = (t_last - t_first) / a.steps / 1e6
        busy = union(iv) / a.steps / 1e6
        launch = sum(e - s for f in timed for (s, e, n) in f if re.search(main_re, n)) / a.steps / 1e6
        ends = [max(e for _, e, _ in f) for f in fr]
        periods = [(ends[i] - ends[i - 1]) / 1e6 for i in range(1, len(ends))]
        print(f"{name}: {len(fr)} frames after {skip} counting passes; timed window: wall {wall:.4f} ms/frame, "
              f"busy (union) {busy:.4f} ms/frame, main launch mean {launch:.4f} ms")
        if a.periods:
            print("  periods (ms): " + " ".join(f"{p:.4f}" for p in periods))
        if line is not None:
            obj = line if name == "grid512" else line.get("other_configs", {}).get(name)
            if name == "grid512_all_channels":
                obj = None
                al = line.get("all_channels_loaded")
                if al:
                    print(f"  line: ms_per_step {al['ms_per_step']}, trace wall {wall:.4f} "
                          f"({wall / al['ms_per_step'] - 1:+.1%})")
            if obj:
                ro = obj["roofline"]
                ms_line = obj["ms_per_step"]
                # the line's achieved x its time = the algorithmic units per frame
                if "gpu_window_ms" in ro.get("achieved_def", ""):
                    t_used = (obj.get("window", {}).get("gpu_window_ms") or obj.get("gpu_window_ms")) / a.steps
                elif "window" in ro.get("achieved_def", ""):
                    t_used = ms_line
                else:
                    t_used = obj["kernel_ms_mean"]
                units = ro["achieved"] * t_used
                if "gpu_ms_per_frame_gated" in ro:
                    t_used = ro["gpu_ms_per_frame_gated"]
                    units = ro["achieved"] * t_used
                checks = [("trace wall", wall), ("trace busy", busy)]
                if gated is not None:
                    checks.append(("trace wall of the gated pass", gated))
                for label, t in checks:
                    frac = units / t / ro["peak"]
                    print(f"  roofline: line frac {ro['frac']:.4f} (time {t_used:.4f} ms); {label} {t:.4f} ms -> "
                          f"frac {frac:.4f} ({frac / ro['frac'] - 1:+.1%})")


if __name__ == "__main__":
    main()
