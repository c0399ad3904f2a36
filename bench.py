#!/usr/bin/env python3
"""bench.py -- Mray/s of the ray-march hot path on 1..N MI355X GPUs.

Workload (BASELINE.json configs[4], the reference algorithm at the metric's
1920x1080x128 point): 512^3 RGBA8 density grid built by the reference recipe
(TestMain.cpp:43-92, frequencies scaled by 128/512), reference camera
(TestMain.cpp:219-245, aspect 16:9), 128 steps (frag.glsl:30), RGBA8 output.
One "step" of this bench = one frame.  The frame is sharded over the ranks as
interleaved 16-row bands.  With N > 1, each frame's bands are gathered to rank 0
over RCCL and assembled there.  The volume is resident in HBM before timing.

value = W*H*max_steps*frames / wall time (nominal Mray/s, the BASELINE
metric), max over ranks.  roofline: algorithmic gather bytes of the march
kernel (32 B per executed ray-step) / its mean HIP-event
duration.  cpu_baseline: the CPU oracle (oracle/, a port) on the same workload.

The procedural configs (BASELINE configs 2/3: "cloud", "cloud_shadow") march the build-defined Perlin-fBm x Worley medium instead of a
grid.  They are ALU-bound, so their roofline is VALU: FLOP_PER_DENSITY
algorithmic fp32 FLOP per density evaluation x the
evaluations per launch (vr option "count" = 1) / mean kernel duration, against
the 157.3 TFLOP/s fp32 vector peak.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--config grid512|grid128|grid4k|cloud|cloud_shadow]
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np
import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

import volumetricrenderer_amd as vr  # noqa: E402
from volumetricrenderer_amd import distributed as vrdist  # noqa: E402

HBM_PEAK_GBS = 8000.0      # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec
# the roofline's gated pass queues its K frames behind this many frames of the
# same loop (~0.8 ms of GPU work at config 5): the host queues the K frames
# meanwhile, so the GPU never waits for it between them.  Round 6 first gated
# with a ~2 ms sleep kernel (torch.cuda._sleep), which let the clocks drop:
# the pass then ran ~2 % slower than the timed window itself
# (profiles/r06/final3/trace_frames.txt: 0.1055 against 0.1035 ms per frame).
GATE_FRAMES = 8
FP32_PEAK_TFLOPS = 157.3   # MI355X_MICROARCH.md: fp32 vector peak
TA_PEAK_GLOOKUPS = 256 * 2.4   # L1 tag lookups: 1 per CU-cycle at 2.4 GHz (tools/tcp_calib.hip)
BYTES_PER_STEP = 32        # 4 trilinear taps x 8 texels x 1 B
# fp32 FLOP per executed grid ray-step (FMA = 2): per tap, texel coordinate 3 fma (6),
# 3 fractions (3), 7 lerps x (sub + fma) (21), x 1/255 (1) = 31; x 4 taps = 124;
# combine t0*t1*(t2+t3)*scale + acc (5); advance the ray point (3).  (SURVEY.md 8d
# estimates ~90.)  The CORNERH layout stores each footprint row as {a, b - a}, so its
# 4 x-lerp subtractions per tap are done once at layout build, not per step: 116.
FLOP_PER_STEP = 132
FLOP_PER_STEP_CORNERH = 132 - 16

CONFIGS = {
    # name: (volume N or None = procedural, width, height, max_steps, shadow steps, BASELINE configs index)
    "grid512": (512, 1920, 1080, 128, 0, 4),
    "grid128": (128, 1920, 1080, 128, 0, None),
    "cloud": (None, 1920, 1080, 128, 0, 1),
    "cloud_shadow": (None, 1920, 1080, 128, 8, 2),
    "grid4k": (128, 3840, 2160, 256, 0, 3),
}


def flop_per_density(octaves: int, cells_per_eval: float | None = None) -> float:
    """Algorithmic fp32 FLOP of one procedural density evaluation, counted on
    the algorithm the kernel runs (FMA = 2; add, sub, mul, min, max, floor,
    rint, sqrt = 1; integer hashing, table reads and int<->float conversions
    not counted).  Per Perlin octave 67: floor 3, fraction subs 6, quintic
    3 x 7, 8 gradient dots x 1 (u + v), 7 lerps x 3, scale 1, coordinate scale
    3, fbm fma 2, parameter updates 2.  Worley F1 (noise::cellular_table9,
    pruned): setup 9 (floor 3, the cube's cell offsets 6), 12 per cell
    computed (3 fma, squared distance 5, min) x cells_per_eval -- measured per
    launch with vr option "count" = 2: 8 for the unit cube, 35 when a sample
    also runs the 27-cell block --, the bound test 15 (3 min, T + 1 + 2 min g
    5 fma/min, sqrt, add, square, compare), the full block's own setup 12
    (rint 3, offsets 9) for the fraction (cells - 8) / 27 of samples that run
    it, final 1; the cell's feature-point normalisation is per cell, not per
    sample (LDS table), and is not counted.  The rest 11.
    cells_per_eval None: the unpruned 27-cell F1 (round 2's count, 625 FLOP
    at 4 octaves), kept as a secondary figure."""
    if cells_per_eval is None:
        return 67 * octaves + 346 + 11
    full = max(0.0, (cells_per_eval - 8.0) / 27.0)
    return 67 * octaves + 9 + 12 * cells_per_eval + 15 + 12 * full + 1 + 11


def roofline_of(r, proc, shadow, variant, local_steps, local_evals, local_cells, kern_ms):
    """The roofline object of one config's march: HBM
    gather bytes for a grid past the Infinity Cache, fp32 VALU for the
    cache-resident grid and the procedural medium."""
    # bytes a step must gather: 8 per tap whose channel is not uniform
    umask = r.get_option("uniform_mask") if proc is None and "_u" in variant else 0
    taps_loaded = 4 - bin(max(umask, 0)).count("1")
    bytes_per_step = 8 * taps_loaded
    gather = local_steps * bytes_per_step / (kern_ms * 1e-3) / 1e9
    gather32 = local_steps * BYTES_PER_STEP / (kern_ms * 1e-3) / 1e9
    if proc is None and "corner8" not in variant and "cornerh" not in variant:
        roofline = {"bound": "hbm", "achieved": round(gather, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                    "frac": round(gather / HBM_PEAK_GBS, 4), "traffic": None,
                    "achieved_def": f"{bytes_per_step} B algorithmic gather per executed ray-step (8 B per tap "
                                    f"of a non-uniform channel; {4 - taps_loaded} uniform) x steps per launch "
                                    "/ mean march-kernel duration (HIP events on its stream)",
                    **({"frac_32B": round(gather32 / HBM_PEAK_GBS, 4)} if taps_loaded < 4 else {})}
    elif proc is None:
        # cache-resident volume (cornerh / corner8 are auto only when they
        # fit the Infinity Cache): the march is VALU-bound (VALUBusy ~100 %,
        # profiles/r01_pmc/c8_4k.json), so the roofline is fp32 VALU
        fps = FLOP_PER_STEP_CORNERH if "cornerh" in variant else FLOP_PER_STEP
        fps -= (27 if "cornerh" in variant else 31) * (4 - taps_loaded)   # a uniform tap is a constant
        tf = local_steps * fps / (kern_ms * 1e-3) / 1e12
        roofline = {"bound": "valu", "achieved": round(tf, 2), "peak": FP32_PEAK_TFLOPS, "unit": "TFLOP/s",
                    "frac": round(tf / FP32_PEAK_TFLOPS, 4), "traffic": None,
                    "achieved_def": f"{fps} algorithmic fp32 FLOP per executed ray-step ({taps_loaded} "
                                    "sampled taps) x steps per launch / mean march-kernel duration (HIP events "
                                    "on its stream); the volume is cache-resident",
                    "gather_GBs": round(gather, 1)}
    else:
        defer = shadow > 0 and r.get_option("shadow_defer") == 1
        cpe = local_cells / max(1, local_evals)
        fpd = flop_per_density(proc.octaves, cpe)
        fpd27 = flop_per_density(proc.octaves)
        achieved = local_evals * fpd / (kern_ms * 1e-3) / 1e12
        a27 = local_evals * fpd27 / (kern_ms * 1e-3) / 1e12
        roofline = {"bound": "valu", "achieved": round(achieved, 2), "peak": FP32_PEAK_TFLOPS,
                    "unit": "TFLOP/s", "frac": round(achieved / FP32_PEAK_TFLOPS, 4), "traffic": None,
                    "achieved_def": f"{fpd:.1f} algorithmic fp32 FLOP per density evaluation (Perlin "
                                    f"{67 * proc.octaves} + pruned Worley at {cpe:.3f} cells per evaluation, "
                                    "measured with vr option count=2, + bound test, setup, rest) x "
                                    f"{local_evals} evaluations per launch / mean march-kernel duration "
                                    "(HIP events on its stream); no volume is read" +
                                    ("; with deferred shadow rays (vr option shadow_defer = 1) the frame is "
                                     "five launches -- primary march, scan, chunk map, shadow pass, resolve "
                                     "-- and the events bracket all of them" if defer else ""),
                    "worley_cells_per_eval": round(cpe, 4),
                    "flop_per_eval_27cell": fpd27,
                    "frac_27cell": round(a27 / FP32_PEAK_TFLOPS, 4)}
    return roofline


def cpu_baseline(volume_host, osd, gsd, march, width, height, budget_s=10.0, procedural=None):
    """Time the oracle on the same frame (all cores it is allowed), ~budget_s."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import vr_oracle as oracle

    threads = int(os.environ.get("OMP_NUM_THREADS", "0")) or len(os.sched_getaffinity(0))
    threads = max(1, min(threads, len(os.sched_getaffinity(0))))
    obj, glob = vr.shader_data_arrays(osd, gsd)
    m = oracle.from_params(march)
    # sample: every 8th 16-row band of the frame (1/8 of the rows, spread
    # over the whole silhouette), repeated until the budget is spent.
    t0 = time.perf_counter()
    rows = 0
    steps = 0
    reps = 0
    while True:
        if procedural is not None:
            _, s = oracle.render_procedural(oracle.procedural_from(procedural), obj, glob, m, width, height,
                                            oracle.FMT_RGBA8_UNORM, band_rows=16, band_stride=8,
                                            band_first=reps % 8, threads=threads)
        else:
            _, s = oracle.render(volume_host, obj, glob, m, width, height, oracle.FMT_RGBA8_UNORM,
                                 band_rows=16, band_stride=8, band_first=reps % 8, threads=threads)
        rows += vr.band_rows_packed(height, 16, 8, reps % 8)
        steps += s
        reps += 1
        el = time.perf_counter() - t0
        if el >= budget_s or reps >= 2000:
            break
    mray = rows * width * march.max_steps / el / 1e6
    model = ""
    try:
        with open("/proc/cpuinfo") as f:
            model = next((ln.split(":", 1)[1].strip() for ln in f if ln.startswith("model name")), "")
    except OSError:
        pass
    return {"value": round(mray, 3), "unit": "Mray/s", "cores": threads, "kind": "port",
            "host_cpu": model, "host_nproc": os.cpu_count(),
            "sample": f"{reps} band sets of every 8th 16-row band ({rows} rows of {height}) of the same "
                      f"{width}x{height}x{march.max_steps} frame and {'medium' if procedural else 'volume'}, "
                      f"{el:.1f} s; "
                      f"executed steps/s {steps / el:.4g}"}


def clock_warm(launch, ms, chunk=8):
    """Declared pre-warm (bench.py --clock-warm-ms, verdict r05 #1): queue
    frames in chunks until `ms` of continuous load have passed on the host
    clock, before the --warmup frames.  The GPU's frame period settles over
    the first ~20-40 ms of load, after an idle gap or host-side set-up alike,
    while the sampled shader clock reads ~2.35-2.4 GHz throughout
    (profiles/r06/warmup_trace.txt), so a frame count cannot size it.
    Returns the frames it queued."""
    if ms <= 0:
        return 0
    n = 0
    t0 = time.perf_counter()
    while (time.perf_counter() - t0) * 1e3 < ms:
        for _ in range(chunk):
            launch()
        n += chunk
        torch.cuda.synchronize()
    return n


def clock_warm_ranks(run8, settle, ms, world, dev="cpu"):
    """clock_warm for a collective frame loop: one timed chunk of 8 frames
    sizes the rest, agreed over the ranks (every rank must queue the same
    frames).  Returns the frames queued."""
    if ms <= 0:
        return 0
    run8()      # the first chunk may pay one-time set-up (e.g. the frame loop's communicator split)
    settle()
    t0 = time.perf_counter()
    run8()      # the second sizes the rest
    settle()
    chunks = max(0, int(np.ceil(ms / max(1e-3, (time.perf_counter() - t0) * 1e3))) - 1)
    if world > 1:
        ct = torch.tensor([chunks], dtype=torch.int64, device=dev)
        dist.all_reduce(ct, op=dist.ReduceOp.MAX)
        chunks = int(ct.item())
    for _ in range(chunks):
        run8()
    settle()
    return 8 * (chunks + 2)


def clock_warm_obj(ms, frames):
    return {"ms": ms, "frames": frames,
            "def": "untimed frames of this config queued back to back for this many ms of continuous load before "
                   "the --warmup frames (the frame period settles over the first ~20-40 ms of load; "
                   "profiles/r06/warmup_trace.txt)"}


def frame_check_of(got, ref):
    """'exact' when the pipeline's frame equals a plain one-GPU render
    bit for bit, else a description of the mismatch (bench.py exits 4)."""
    torch.cuda.synchronize()
    a, b = got.cpu().numpy(), ref.cpu().numpy()
    if a.shape != b.shape:
        return f"MISMATCH: shape {a.shape} vs {b.shape}"
    bad = np.any(a != b, axis=-1) if a.ndim == 3 else a != b
    if not bad.any():
        return "exact"
    rows = np.nonzero(bad.any(axis=1))[0]
    return f"MISMATCH: {int(bad.sum())} pixels differ in {rows.size} rows (first row {int(rows[0])})"


def other_config(name, steps, warmup, warm_ms=0.0):
    """Time one more BASELINE config on this GPU in the same process, after the
    headline window (verdict r03 #6): ms/frame, kernel ms (HIP events on its
    stream, every 4th frame), the roofline object.  Returns the result and the
    arguments of its CPU baseline."""
    N, W, H, S, shadow, cfg_idx = CONFIGS[name]
    fmt = vr.FMT_RGBA8_UNORM
    with vr.Renderer(0) as r:
        proc = None
        if N is None:
            r.set_procedural(shadow_steps=shadow)
            proc = r.procedural
        else:
            r.generate_volume(vr.scaled_recipe(N))
        osd, gsd = vr.reference_shader_data(1280.0 / 720.0)
        r.set_shader_data(osd, gsd)
        march = vr.march_defaults(max_steps=S)
        r.set_march(march)
        out = r.alloc_target(W, H, fmt)
        counter = torch.zeros(1, dtype=torch.int64, device="cuda")

        def units(mode):
            r.set_option("count", mode)
            counter.zero_()
            r.render(W, H, fmt, out=out, step_counter=counter)
            torch.cuda.synchronize()
            return int(counter.item())

        nsteps = units(0)
        evals, cells = (units(1), units(2)) if proc is not None else (nsteps, None)
        r.set_option("count", 0)
        launch = r.prepare_render(W, H, fmt, out)
        warm_frames = clock_warm(launch, warm_ms)
        for _ in range(warmup):
            launch()
        torch.cuda.synchronize()
        ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) if i % 4 == 0 else None
              for i in range(steps)]
        t0 = time.perf_counter()
        for i in range(steps):
            if ev[i] is not None:
                ev[i][0].record()
            launch()
            if ev[i] is not None:
                ev[i][1].record()
        torch.cuda.synchronize()
        el = time.perf_counter() - t0
        kern_ms = float(np.mean([e[0].elapsed_time(e[1]) for e in ev if e is not None]))
        variant = r.kernel_variant
        # grid media: the same frames two in flight, as the headline's loop runs
        # them -- consecutive frames alternate two streams and two targets
        inflight2 = None
        if True:   # (a procedural medium too since round 6: per-stream deferred scratch)
            streams = [torch.cuda.Stream(), torch.cuda.Stream()]
            outs = [out, r.alloc_target(W, H, fmt)]
            launches = [r.prepare_render(W, H, fmt, outs[k], stream=streams[k]) for k in range(2)]
            for i in range(warmup):
                launches[i & 1]()
            torch.cuda.synchronize()
            cur = torch.cuda.current_stream()
            g0, g1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            t0 = time.perf_counter()
            g0.record(cur)
            for st_ in streams:
                st_.wait_event(g0)
            for i in range(steps):
                launches[i & 1]()
            for st_ in streams:
                cur.wait_stream(st_)
            g1.record(cur)
            torch.cuda.synchronize()
            el2 = time.perf_counter() - t0
            gpu2_ms = g0.elapsed_time(g1)
            inflight2 = {"ms_per_step": round(el2 / steps * 1e3, 4), "value": round(W * H * S * steps / el2 / 1e6, 3),
                         "def": "the same frames, consecutive frames alternating two streams and two targets, wall "
                                "time per frame"}
        defer = proc is not None and shadow > 0 and r.get_option("shadow_defer_last") == 1
        # config 2 (procedural, no shadow rays) runs two in flight, as its own
        # N = 1 line does (bench.py --config cloud; 0.1606 against 0.1662 ms on
        # one stream, profiles/r06/c10); the others keep one stream (config 3
        # two in flight: 0.783 against 0.756; config 4 level)
        two = proc is not None and shadow == 0 and inflight2 is not None
        one_stream = None
        roof_ms = kern_ms
        if two:
            one_stream = {"ms_per_step": round(el / steps * 1e3, 4), "value": round(W * H * S * steps / el / 1e6, 3),
                          "kernel_ms_mean": round(kern_ms, 5),
                          "def": "the same frames on one stream (launches do not overlap)"}
            el = el2
            roof_ms = gpu2_ms / steps   # the window on the GPU clock (HIP events), per frame
            inflight2 = None
        res = {"metric": f"Mray/s (= W*H*steps/s) at {W}x{H} x {S} steps",
               "value": round(W * H * S * steps / el / 1e6, 3), "unit": "Mray/s", "steps": steps,
               "ms_per_step": round(el / steps * 1e3, 4), "kernel_ms_mean": round(kern_ms, 5),
               **({"frames_in_flight": 2} if two else {}),
               "config": {"workload": (f"{name}: {N}^3 RGBA8 grid, {W}x{H}, {S} steps, RGBA8 out" if proc is None
                                       else f"{name}: procedural {proc.octaves}-octave Perlin-Worley cloud, "
                                            f"{W}x{H}, {S} steps, shadow {shadow} steps, RGBA8 out"),
                          "baseline_config_index": cfg_idx,
                          "kernel": variant + ("_deferred" if defer else ""),
                          "executed_steps_per_frame": nsteps},
               "roofline": roofline_of(r, proc, shadow, variant, nsteps, evals, cells, roof_ms),
               "clock_warm": clock_warm_obj(warm_ms, warm_frames),
               **({"frames_in_flight_2": inflight2} if inflight2 else {}),
               **({"one_stream": one_stream} if one_stream else {})}
        if two:
            res["gpu_window_ms"] = round(gpu2_ms, 4)
            res["roofline"]["achieved_def"] += ("; two frames in flight on alternating streams, so the time is the "
                                                "timed window on the GPU clock (HIP events on the caller's stream "
                                                "around the frames, gpu_window_ms) per frame (kernel_ms_mean: the "
                                                "one-stream launches' mean)")
        if defer:
            res["shadow_defer_scratch_MB"] = round(r.get_option("shadow_defer_kib") / 1024.0, 1)
        vol = r.get_volume() if proc is None else None
    return res, (vol, osd, gsd, march, W, H, proc)


def main() -> int:
    # stdout carries exactly one JSON line (rank 0).  Libraries print to fd 1
    # too -- RCCL its version banner at communicator init -- so fd 1 is
    # pointed at stderr for the whole run and the JSON goes to a private
    # duplicate of the original stdout.
    sys.stdout.flush()
    json_out = os.fdopen(os.dup(1), "w")
    os.dup2(2, 1)
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--clock-warm-ms", type=float, default=150.0,
                    help="before each config's --warmup frames, queue untimed frames for this many ms of continuous "
                         "load (declared in the line as clock_warm; 0 = off)")
    ap.add_argument("--config", default="grid512", choices=sorted(CONFIGS))
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-budget", type=float, default=10.0)
    ap.add_argument("--cpu-budget-other", type=float, default=3.0, help="CPU baseline budget of each other config")
    ap.add_argument("--no-other-configs", action="store_true",
                    help="N = 1, default config: skip timing configs 2, 3, 4 after the headline window")
    ap.add_argument("--schedule", type=int, default=-1, help="vr option 'schedule' (-1 = auto)")
    ap.add_argument("--sharder", default="native", choices=["native", "torch"],
                    help="N > 1: native = the C++ frame loop over this library's own RCCL communicator "
                         "(libvr_shard.so; torch.distributed/gloo only carries its id and the barriers); "
                         "torch = BandSharder over torch.distributed")
    ap.add_argument("--backend", default="nccl", choices=["nccl", "gloo"],
                    help="torch sharder's backend; gloo: rehearse the N>1 path with several ranks on one GPU")
    ap.add_argument("--pipeline1", action="store_true", help=argparse.SUPPRESS)
    ap.add_argument("--n1-loop", default="native", choices=["native", "sharder"],
                    help="N = 1, grid media: native (default) = the frame loop of N > 1 (libvr_shard over a "
                         "one-rank communicator: 2 render streams, 2 frames in flight as the reference keeps them, "
                         "VulkanRenderer.cpp:13); sharder = one stream through BandSharder (rounds 1-5's N = 1 line, "
                         "whose launches do not overlap; always for a procedural medium)")
    ap.add_argument("--layout", type=int, default=0, help="vr layout preference (0 = auto; 15 = COL48)")
    ap.add_argument("--slab", action="store_true", help="COL48 layout + the LDS-slab march (vr_march_slab.hip)")
    ap.add_argument("--opt", action="append", default=[], help="vr option NAME=VALUE (experiments)")
    ap.add_argument("--inflight", type=int, default=1, choices=[1, 2],
                    help="N = 1, grid medium: 2 = consecutive frames alternate two streams and targets (throughput "
                         "mode; per-launch kernel times then overlap the next frame)")
    ap.add_argument("--render-streams", type=int, default=None, choices=[1, 2, 3, 4],
                    help="native loop: n = 2..4 consecutive frames render on n alternating streams and overlap "
                         "(vr_shard_set_render_streams), 1 = one render stream; default: RcclBandPipeline's (3 for "
                         "frames above 2560x1440, else 2)")
    ap.add_argument("--exchange", default="render", choices=["render", "comm"],
                    help="N > 1 (native loop, 2 render streams): each frame's exchange on its render stream, over one "
                         "communicator per buffer parity, no events (the default), or on a communication stream "
                         "ordered by events (vr_shard_set_exchange_streams)")
    ap.add_argument("--inflight-probe", action="store_true",
                    help="N = 1: also time the same frames with two in flight (frames_in_flight_2 in the line)")
    ap.add_argument("--spin", action="store_true",
                    help="moving camera: every frame gets new shader data, phi += 1.6 deg (the reference's "
                         "held A/D key, TestMain.cpp:171-184, :222-224), queued natively (vr_render_sequence "
                         "at N = 1, vr_shard_run_frames at N > 1)")
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    ndev = torch.cuda.device_count()
    dev = local % max(1, ndev)
    # N = 1: the native frame loop with a one-rank communicator, the same loop
    # as N > 1 (--n1-loop sharder / --inflight 2: the BandSharder paths)
    # (grid media: a procedural medium's frames cannot overlap, and its renders
    # run ~10 % slower inside the loop than through BandSharder)
    native = ((world > 1 and args.sharder == "native") or args.pipeline1
              or (world == 1 and args.n1_loop == "native" and args.inflight == 1
                  and CONFIGS[args.config][0] is not None))
    if native and ndev < world:
        raise SystemExit(f"--sharder native needs one GPU per rank ({world} ranks, {ndev} GPUs); "
                         "use --sharder torch --backend gloo to rehearse on fewer GPUs")
    if world > 1:
        torch.cuda.set_device(dev)
        if args.backend == "nccl" and not native:
            dist.init_process_group("nccl", device_id=torch.device("cuda", dev))
        else:
            dist.init_process_group("gloo")
    else:
        torch.cuda.set_device(0)
    N, W, H, S, shadow, cfg_idx = CONFIGS[args.config]

    r = vr.Renderer(dev)
    proc = None
    if N is None:
        r.set_procedural(shadow_steps=shadow)
        proc = r.procedural
    else:
        r.generate_volume(vr.scaled_recipe(N))
    osd, gsd = vr.reference_shader_data(1280.0 / 720.0)
    r.set_option("schedule", args.schedule)
    for o in args.opt:
        k, v = o.split("=")
        r.set_option(k, int(v))
    if args.slab:
        args.layout = 15
        r.set_option("slab", 1)
    if args.layout and N is not None:
        r.set_layout_preference(args.layout)
    r.set_shader_data(osd, gsd)
    march = vr.march_defaults(max_steps=S)
    r.set_march(march)
    fmt = vr.FMT_RGBA8_UNORM
    # N = 1, a procedural medium without shadow rays: two frames in flight
    # through BandSharder (frames reusing the cost order only read the ctx's
    # scratch and overlap; the native loop's procedural renders ran ~10 % slower)
    proc_inflight2 = (world == 1 and not native and proc is not None and shadow == 0 and args.n1_loop == "native"
                      and args.inflight == 1 and not args.spin)
    sharder = vrdist.BandSharder(r, W, H, fmt, band_rows=16, world=world, rank=rank,
                                 inflight=2 if proc_inflight2 else args.inflight)
    stream = torch.cuda.current_stream()

    # executed ray-steps per launch (this rank's bands), one untimed pass
    counter = torch.zeros(1, dtype=torch.int64, device="cuda")
    sharder.render_local(step_counter=counter)
    torch.cuda.synchronize()
    local_steps = int(counter.item())
    local_evals = local_steps
    local_cells = None
    if proc is not None:
        r.set_option("count", 1)
        counter.zero_()
        sharder.render_local(step_counter=counter)
        torch.cuda.synchronize()
        local_evals = int(counter.item())
        r.set_option("count", 2)   # Worley cells the pruned evaluations computed
        counter.zero_()
        sharder.render_local(step_counter=counter)
        torch.cuda.synchronize()
        local_cells = int(counter.item())
        r.set_option("count", 0)
    red_dev = "cuda" if args.backend == "nccl" and not native else "cpu"
    tot = torch.tensor([local_steps, local_evals, local_cells or 0], dtype=torch.int64, device=red_dev)
    if world > 1:
        dist.all_reduce(tot)
    frame_steps, frame_evals, frame_cells = (int(v) for v in tot.tolist())

    # HIP events around the march launch of every 4th frame: the sample of
    # launch durations the roofline uses.  Two event records per frame cost a
    # few microseconds of queue time between frames (and, at N > 1, host time)
    ev_every = 4
    warm_frames = 0
    busy_ms_frame = None
    gated_ms_frame = None
    frame_check = None
    window = None
    pipe = None
    if native:
        # No silent fallback: a multi-GPU number must come from the path its
        # label names.  If the native RCCL frame loop cannot be made, every
        # rank fails (RcclBandPipeline agrees on success before the collective
        # communicator init) and the bench exits non-zero.
        try:
            pipe = vrdist.RcclBandPipeline(r, W, H, fmt, band_rows=16, world=world, rank=rank,
                                           render_streams=args.render_streams,
                                           exchange_on_render=args.exchange == "render")
        except vr.VRError as e:
            print(f"rank {rank}: native RCCL frame loop unavailable: {e}", file=sys.stderr, flush=True)
            raise SystemExit(3)
    # a spinning camera: new shader data before every frame (phi += 1.6 deg, the
    # reference's held A/D key), so the frame pays the region-list reuse / GPU
    # rebuild (grid) or the cost sort (procedural) that a static camera skips.
    # The shader data of every frame is made before the clock starts (host
    # math, TestMain.cpp:219-245); the frames are queued natively.
    SPIN_DEG = 1.6
    sd = ([vr.reference_shader_data(1280.0 / 720.0, SPIN_DEG * i, 0.0) for i in range(args.warmup + args.steps)]
          if args.spin else None)
    if native:
        # Bracket: host barrier (gloo) for the rendezvous, then the device-side
        # RCCL barrier + synchronisation on both sides of the timed frames.  A
        # gloo barrier across 8 processes costs a sizeable fraction of a
        # millisecond -- several 1/8-frames -- so it stays outside the clock.
        # (sampling every warmup frame creates the loop's timing events now,
        # outside the window: ceil(steps / ev_every) pairs, created on first use)
        if not args.spin:   # (a spinning camera's frames are all distinct: its warm-up stays the frame count)
            warm_frames = clock_warm_ranks(lambda: pipe.run_frames(8), lambda: pipe.barrier(stream),
                                           args.clock_warm_ms, world, red_dev)
        pipe.run_frames(args.warmup, cameras=sd[:args.warmup] if sd else None, sample_every=1)
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()
        pipe.barrier(stream)
        e_w0, e_w1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        t0 = time.perf_counter()
        e_w0.record(stream)
        kern_ms = pipe.run_frames(args.steps, stream=stream, sample_every=ev_every,
                                  cameras=sd[args.warmup:] if sd else None)
        e_w1.record(stream)   # the caller's stream joins every render stream's last frame
        t_q = time.perf_counter()
        host_el = pipe.host_ms * args.steps * 1e-3
        pipe.barrier(stream)
        t_b = time.perf_counter()
        torch.cuda.synchronize()
        el = time.perf_counter() - t0
        window = {"host_queue_ms": round((t_q - t0) * 1e3, 4), "host_barrier_ms": round((t_b - t0) * 1e3, 4),
                  "gpu_window_ms": round(e_w0.elapsed_time(e_w1), 4), "host_window_ms": round(el * 1e3, 4),
                  "def": "the timed window on the host clock (t0 -> frames queued -> barrier returned -> synchronized) "
                         "and on the GPU clock (HIP events on the caller's stream before the first frame and after "
                         "the join of the render streams)"}
        if world > 1:
            dist.barrier()
        # parity of the timed path (verdict r05 #2): rank 0's last frame of the
        # window -- RCCL-gathered and assembled at N > 1 -- against a plain
        # one-GPU render of the same camera, untimed
        # (the copy now, the reference render after the passes below: a plain
        # render's other target geometry would make the loop's next frame
        # rebuild its region lists on the host)
        got = pipe.frame(stream)
        # untimed, after the window: the same K frames gated -- queued behind
        # GATE_FRAMES frames of the loop, so the GPU never waits for the host
        # between them and runs at the window's clocks -- with HIP events after
        # the gate's frames (the caller's stream joins the render streams) and
        # after the K frames' join: the GPU time per frame the roofline divides
        # by (the timed window's own GPU clock also holds the first frame's
        # launch latency)
        g0, g1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        pipe.run_frames(GATE_FRAMES, stream=stream,
                        cameras=[sd[args.warmup + i % args.steps] for i in range(GATE_FRAMES)] if sd else None)
        g0.record(stream)
        pipe.run_frames(args.steps, stream=stream, cameras=sd[args.warmup:] if sd else None)
        g1.record(stream)
        pipe.barrier(stream)
        torch.cuda.synchronize()
        gated_ms_frame = g0.elapsed_time(g1) / args.steps
        # and with every render sampled: the GPU busy time per frame (the
        # union of the renders' intervals; overlapping frames count once:
        # vr_shard_sampled_busy; the per-render events slow the frames a little)
        pipe.run_frames(args.steps, stream=stream, sample_every=1, cameras=sd[args.warmup:] if sd else None)
        busy_ms, _span = pipe.sampled_busy()
        busy_ms_frame = busy_ms / args.steps
        pipe.barrier(stream)
        torch.cuda.synchronize()
        if rank == 0:
            if sd:   # the window's last camera (the passes above ended on it too)
                r.set_shader_data(*sd[-1])
            frame_check = frame_check_of(got, r.render(W, H, fmt))
        if world > 1:
            dist.barrier()
    elif args.spin:
        r.render_sequence(W, H, fmt, sharder.local, sd[:args.warmup])
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        r.render_sequence(W, H, fmt, sharder.local, sd[args.warmup:])
        queued_el = time.perf_counter() - t0   # the host waits once the GPU's queue is full
        torch.cuda.synchronize()
        el = time.perf_counter() - t0
        # host time per frame (untimed for the rate): the same frames enqueued 8 at
        # a time on an idle GPU, so no enqueue waits for the GPU to drain its queue
        host_el = 0.0
        for c0 in range(0, args.steps, 8):
            torch.cuda.synchronize()
            t1 = time.perf_counter()
            r.render_sequence(W, H, fmt, sharder.local, sd[args.warmup + c0:args.warmup + min(c0 + 8, args.steps)])
            host_el += time.perf_counter() - t1
        torch.cuda.synchronize()
        # kernel time of every 4th frame: the same frames replayed (untimed),
        # events around each render
        launch = r.prepare_render(W, H, fmt, sharder.local)
        ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
              if i % ev_every == 0 else None for i in range(args.steps)]
        for i in range(args.steps):
            r.set_shader_data(*sd[args.warmup + i])
            if ev[i] is not None:
                ev[i][0].record()
            launch()
            if ev[i] is not None:
                ev[i][1].record()
        torch.cuda.synchronize()
        kern_ms = float(np.mean([e[0].elapsed_time(e[1]) for e in ev if e is not None]))
        # the executed steps of the sampled frames (untimed): the roofline's unit
        sampled = []
        for i in range(args.steps):
            if ev[i] is not None:
                r.set_shader_data(*sd[args.warmup + i])
                counter.zero_()
                sharder.render_local(step_counter=counter)
                torch.cuda.synchronize()
                sampled.append(int(counter.item()))
        local_steps = frame_steps = int(round(float(np.mean(sampled))))
    else:
        warm_frames = clock_warm_ranks(lambda: sharder.run_frames(8), torch.cuda.synchronize, args.clock_warm_ms, world,
                                       red_dev)
        sharder.run_frames(args.warmup)
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize()
        ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
              if i % ev_every == 0 else None for i in range(args.steps)]
        t0 = time.perf_counter()
        sharder.run_frames(args.steps, events=ev)
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()
        el = time.perf_counter() - t0
        kern_ms = float(np.mean([e[0].elapsed_time(e[1]) for e in ev if e is not None]))
        got = sharder.frame()   # collective: a frame gathered as the window's were, untimed
        if rank == 0:
            frame_check = frame_check_of(got, r.render(W, H, fmt))
    # A uniform channel (the recipe's constant G) is a constant tap with no
    # loads ("_u" kernels).  For comparison, the same K
    # frames with every channel loaded, timed after the main window (N = 1).
    all_loaded = None
    if world == 1 and not args.spin and "_u" in r.kernel_variant:
        skipped_variant = r.kernel_variant
        r.set_option("uniform_skip", 0)
        if native:   # the same loop as the headline
            pipe.run_frames(args.warmup)
            pipe.barrier(stream)
            t1 = time.perf_counter()
            k2 = pipe.run_frames(args.steps, stream=stream, sample_every=ev_every)
            pipe.barrier(stream)
            torch.cuda.synchronize()
            el2 = time.perf_counter() - t1
        else:
            sharder.run_frames(args.warmup)
            torch.cuda.synchronize()
            ev2 = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
                   if i % ev_every == 0 else None for i in range(args.steps)]
            t1 = time.perf_counter()
            sharder.run_frames(args.steps, events=ev2)
            torch.cuda.synchronize()
            el2 = time.perf_counter() - t1
            k2 = float(np.mean([e[0].elapsed_time(e[1]) for e in ev2 if e is not None]))
        all_loaded = {"kernel": r.kernel_variant, "ms_per_step": round(el2 / args.steps * 1e3, 4),
                      "kernel_ms_mean": round(k2, 5),
                      "value": round(W * H * S * args.steps / el2 / 1e6, 3)}
        r.set_option("uniform_skip", 1)
        assert r.kernel_variant == skipped_variant
    # The same K frames with two in flight (consecutive frames on two
    # alternating streams and targets, the reference's 2 frames in flight,
    # VulkanRenderer.cpp:13), timed after the main window under the same clock
    # (N = 1; --inflight-probe).  Launches then overlap, so their durations no
    # longer measure a frame: the headline keeps one stream, whose per-launch
    # time the roofline and the rocprof profile use -- and the probe is opt-in,
    # so that the default run's rocprof average holds only one-stream launches.
    inflight2 = None
    if (world == 1 and not native and not args.spin and proc is None and args.inflight == 1
            and args.inflight_probe):
        sh2 = vrdist.BandSharder(r, W, H, fmt, band_rows=16, world=1, rank=0, inflight=2)
        sh2.run_frames(args.warmup)
        torch.cuda.synchronize()
        t1 = time.perf_counter()
        sh2.run_frames(args.steps)
        torch.cuda.synchronize()
        el3 = time.perf_counter() - t1
        inflight2 = {"ms_per_step": round(el3 / args.steps * 1e3, 4),
                     "value": round(W * H * S * args.steps / el3 / 1e6, 3),
                     "def": "the same frames, consecutive frames alternating two streams and two targets "
                            "(bench.py --inflight 2), wall time per frame"}
        sh2.close()
    # the other BASELINE configs, timed in this process after the headline
    # window (N = 1 only; a multi-GPU run keeps to the headline)
    others, other_cpu = {}, {}
    if world == 1 and not args.spin and args.config == "grid512" and not args.no_other_configs:
        for name in ("grid4k", "cloud", "cloud_shadow"):
            others[name], other_cpu[name] = other_config(name, args.steps, args.warmup, args.clock_warm_ms)
    # the measured HBM roofline of this box: one-pass 16-B-per-lane streams of
    # 2 GiB (past the 256 MiB Infinity Cache), read-only and copy, 4 / 8 / 16
    # loads in flight per lane; the larger rate is the denominator
    bw = {}
    if rank == 0:
        for kind in ("read", "copy"):
            bw[kind] = r.measure_bandwidth(kind, 0, 2 << 30, 10)
    tt = torch.tensor([el, kern_ms, busy_ms_frame or 0.0], dtype=torch.float64, device=red_dev)
    if world > 1:
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
    el, kern_ms_max, busy_max = float(tt[0]), float(tt[1]), float(tt[2])

    collective_label = None
    if world > 1:
        if native:
            collective_label = "RCCL grouped send/recv to rank 0 over xGMI, native frame loop (libvr_shard)"
        else:
            backend = dist.get_backend()   # what the process group really is, not what was asked for
            collective_label = (f"torch.distributed gather to rank 0 ({backend}"
                                + (", host-staged: band sets copied through host memory)" if backend == "gloo"
                                   else ", device buffers)"))
    # vr_shard_run_frames renders a procedural medium on one stream (its frames cannot overlap)
    rs = pipe.render_streams if pipe is not None else (args.render_streams or 1)
    streams_eff = 1 if proc is not None else rs
    if rank == 0:
        ms_per_step = el / args.steps * 1e3
        value = W * H * S * args.steps / el / 1e6
        variant = r.kernel_variant
        # two render streams (native loop, N > 1): a launch overlaps the next, so
        # its duration is not a frame's -- the roofline takes the wall time per frame
        overlap = (native and streams_eff >= 2) or proc_inflight2 or (world == 1 and args.inflight == 2)
        # overlapping launches: the window on the GPU clock (HIP events on the
        # caller's stream around the frames) per frame -- what the kernel trace's
        # first-start-to-last-end span measures -- else the launches' mean
        roof_ms = ((gated_ms_frame or (window["gpu_window_ms"] / args.steps if window else ms_per_step))
                   if overlap else kern_ms)
        compositor = native and pipe is not None and pipe.compositor
        lead = pipe.lead_rows if compositor else 0   # rank 0's lead rows beside its assembly
        rows_part = native and pipe is not None and pipe.partition == "rows"
        serp = " serpentine" if native and pipe is not None and getattr(pipe, "serpentine", False) else ""
        if compositor:   # rank 0 renders nothing: the per-GPU figure is a renderer's average share
            nr = world - 1
            roofline = roofline_of(r, proc, shadow, variant, frame_steps // nr, frame_evals // nr,
                                   (frame_cells // nr) if local_cells is not None else None, roof_ms)
            roofline["achieved_def"] += (f"; rank 0 is a compositor (vr_shard_set_compositor): the work is the "
                                         f"frame's over its {nr} rendering ranks"
                                         + (f" (rank 0 also renders the frame's first {lead} rows, "
                                            "vr_shard_balance_lead)" if lead else ""))
        else:
            roofline = roofline_of(r, proc, shadow, variant, local_steps, local_evals, local_cells, roof_ms)
        if overlap:
            roofline["achieved_def"] += (f"; renders overlap ({streams_eff} render streams or two in flight), so "
                                         "the time is the timed window per frame, not a launch's duration "
                                         "(kernel_ms_mean: the overlapping launches' mean)"
                                         + (": the GPU time per frame of the same K frames run again after the window, "
                                            f"gated (queued behind {GATE_FRAMES} frames of the loop, so the GPU never "
                                            "waits for the host and keeps its clocks; HIP events after the gate's frames "
                                            "and after the join of the render streams: gpu_ms_per_frame_gated, "
                                            "gate_frames); the timed window's own clocks are "
                                            "in window, and ms_per_step is the host clock's"
                                            if gated_ms_frame else ": its wall time"))
        if gated_ms_frame:
            roofline["gpu_ms_per_frame_gated"] = round(gated_ms_frame, 5)
            roofline["gate_frames"] = GATE_FRAMES
            # the same units over the host wall time per frame of the timed window
            roofline["frac_wall"] = round(roofline["achieved"] * roof_ms / ms_per_step / roofline["peak"], 4)
        if busy_ms_frame and not compositor:
            # the same units over the GPU busy time per frame (union of the
            # renders' intervals, overlapping frames counted once)
            fb = roofline["achieved"] * roof_ms / busy_ms_frame / roofline["peak"]
            roofline.update({"kernel_busy_ms_per_frame": round(busy_ms_frame, 5), "frac_busy": round(fb, 4),
                             "kernel_busy_def": "union of the render intervals of K untimed frames run after the "
                                                "window with every render bracketed by HIP events on its render "
                                                "stream (vr_shard_sampled_busy) / K; frac_busy = the same "
                                                "algorithmic units / that time / peak"
                                                + (f"; max over ranks {busy_max:.5f} ms" if world > 1 else "")})
        if roofline["bound"] == "hbm":
            pk_kind = max(bw, key=lambda k: bw[k][0])
            pk = bw[pk_kind][0]
            roofline.update({"peak_measured": round(pk, 1), "peak_measured_kind": pk_kind,
                             "frac_measured": round(roofline["achieved"] / pk, 4),
                             **({"frac_measured_wall": round(roofline["achieved"] * roof_ms / ms_per_step / pk, 4)}
                                if gated_ms_frame else {}),
                             "peak_read": round(bw["read"][0], 1), "peak_copy": round(bw["copy"][0], 1),
                             "peak_measured_def": "the larger of a read-only stream (loads folded into a register, "
                                                  "bytes read / time) and a float4 copy (read + written bytes / time): "
                                                  "best of 10 one-pass 16-B-per-lane sweeps of 2 GiB at each of 4, 8 "
                                                  "and 16 loads in flight per lane, on this GPU (vr_measure_bandwidth; "
                                                  + ", ".join(f"{k} best {v[0]:.0f} GB/s at {v[2]} loads per lane, "
                                                              f"median {v[1]:.0f}" for k, v in bw.items()) + ")"})
        traffic = None
        ta = None
        tfile = os.path.join(ROOT, "profiles", "traffic.json")
        if os.path.exists(tfile):
            with open(tfile) as f:
                tj = json.load(f)
            if tj.get("config") == args.config and tj.get("kernel") == r.kernel_variant and world == 1:
                traffic = tj.get("hbm_bytes_per_launch")
                lookups = tj.get("l1_lookups_per_launch")
                if lookups:
                    # the unit that binds config 5: the texture
                    # address pipe, ~1 cycle per L1 lookup (quad x distinct 128-B line)
                    rate = lookups / (roof_ms * 1e-3) / 1e9   # (the wall time per frame when launches overlap)
                    ta = {"achieved": round(rate, 1), "peak": TA_PEAK_GLOOKUPS, "unit": "G L1 lookups/s",
                          "frac": round(rate / TA_PEAK_GLOOKUPS, 4), "lookups_per_launch": lookups,
                          "ta_busy_pmc": tj.get("ta_busy"),
                          "def": "PMC TCP_TOTAL_CACHE_ACCESSES_sum per launch (profiles/traffic.json) / the mean "
                                 "march-kernel duration; peak = 256 CUs x 1 lookup/cycle x 2.4 GHz "
                                 "(tools/tcp_calib.hip)"}
        out = {
            "metric": "Mray/s (= W*H*steps/s) at 1080p x 128 steps" if (W, H, S) == (1920, 1080, 128)
                      else f"Mray/s (= W*H*steps/s) at {W}x{H} x {S} steps",
            "value": round(value, 3),
            "unit": "Mray/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(ms_per_step, 4),
            "higher_is_better": True,
            "scaling": "strong",
            "vs_baseline": None,
            "dtype": "f32",
            "data": ("synthetic: reference noise recipe volume generated on the GPU (FastNoise2-style restatement)"
                     if proc is None else "synthetic: procedural Perlin-fBm x Worley medium evaluated per step"),
            "config": {"workload": (f"{args.config}: {N}^3 RGBA8 grid, {W}x{H}, {S} steps, RGBA8 out" if proc is None
                                    else f"{args.config}: procedural {proc.octaves}-octave Perlin-Worley cloud, "
                                         f"{W}x{H}, {S} steps, shadow {shadow} steps, RGBA8 out"),
                       "baseline_config_index": cfg_idx, "width": W, "height": H, "max_steps": S,
                       "volume": f"{N}^3 RGBA8" if N else "procedural",
                       "camera": ("reference (TestMain.cpp:219-245), spinning: phi += 1.6 deg per frame, new shader "
                                  "data every frame (TestMain.cpp:171-184)" if args.spin
                                  else "reference (TestMain.cpp:219-245)"),
                       "kernel": r.kernel_variant + ("_deferred" if proc is not None and shadow > 0
                                                      and r.get_option("shadow_defer") == 1 else ""),
                       "parallelism": (("one GPU, the native frame loop (libvr_shard, one-rank communicator)"
                                        + (f", {streams_eff} render streams: {streams_eff} frames in flight" if streams_eff >= 2
                                           else ", 1 render stream (a procedural medium's frames do not overlap)"
                                           if proc is not None else ", 1 render stream"))
                                       if native and world == 1 else
                                       ((f"row ranges x{world - 1}" if rows_part else f"bands16x{world - 1}{serp}")
                                        + ", rank 0 compositing" + (f" + {lead} lead rows" if lead else "") if compositor
                                        else (f"row ranges x{world}" if rows_part else f"bands16x{world}{serp}"))
                                       + (", 2 frames in flight (two streams and targets)"
                                          if args.inflight == 2 or proc_inflight2 else "")
                                       + (f", {rs} render stream{'s' if rs > 1 else ''}"
                                          + (f", exchange on {args.exchange} stream{'s' if args.exchange == 'render' else ''}"
                                             if rs >= 2 else "")
                                          if native else "")),
                       "collective": collective_label,
                       "executed_steps_per_frame": frame_steps},
            "executed_steps_per_s": round(frame_steps * args.steps / el, 1),
            "kernel_ms_mean": round(kern_ms, 5),
            **({"host_ms_per_frame": round(host_el / args.steps * 1e3, 4)} if args.spin or native else {}),
            **({"host_ms_per_frame_queued": round(queued_el / args.steps * 1e3, 4),
                "host_ms_def": "host time of vr_render_sequence per frame, frames enqueued 8 at a time on an idle "
                               "GPU (host_ms_per_frame_queued: the timed 64-frame call, which waits whenever the "
                               "GPU's queue is full)"} if args.spin and not native else {}),
            **({"region_lists": {"gpu_builds": r.get_option("region_gpu_builds"),
                                 "interval": r.get_option("region_interval")}} if args.spin and proc is None else {}),
            "frame_check": frame_check,
            **({"frame_check_def": "rank 0's last frame of the timed window ("
                                   + ("RCCL-gathered and assembled" if world > 1 else "the frame loop's")
                                   + ") against a plain one-GPU vr_render of the same camera, untimed: 'exact' = "
                                     "bit-identical"} if frame_check else {}),
            "clock_warm": clock_warm_obj(args.clock_warm_ms if warm_frames else 0.0, warm_frames),
            **({"window": window} if window else {}),
            **({"all_channels_loaded": all_loaded} if all_loaded else {}),
            **({"frames_in_flight_2": inflight2} if inflight2 else {}),
            "kernel_ms_mean_max_rank": round(kern_ms_max, 5),
            "roofline": dict(roofline, traffic=traffic,
                             **({"traffic_GBs": round(traffic / (roof_ms * 1e-3) / 1e9, 1),
                                 "traffic_frac": round(traffic / (roof_ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4),
                                 "traffic_def": "PMC bytes per frame (profiles/traffic.json: FETCH_SIZE x 2 + "
                                                "WRITE_SIZE, re-collected on this build in round 6) / the same "
                                                "time per frame; FETCH_SIZE counts the L2's fabric requests, "
                                                "Infinity-Cache hits included, and its x2 gfx950 correction is "
                                                "calibrated for 16-B-per-lane streams, not the march's 8-B "
                                                "gathers: an upper bound of the HBM bytes"}
                                if traffic else {}),
                             **({"ta_lookup": ta} if ta else {})),
        }
        if others:
            out["other_configs"] = others
        if not args.no_cpu_baseline and world == 1:
            out["cpu_baseline"] = cpu_baseline(None if proc is not None else r.get_volume(), osd, gsd, march, W, H,
                                               args.cpu_budget, procedural=proc)
            for name, (vol_o, osd_o, gsd_o, march_o, W_o, H_o, proc_o) in other_cpu.items():
                others[name]["cpu_baseline"] = cpu_baseline(vol_o, osd_o, gsd_o, march_o, W_o, H_o,
                                                            args.cpu_budget_other, procedural=proc_o)
        print(json.dumps(out), file=json_out, flush=True)
    rc = 0
    if rank == 0 and frame_check is not None and frame_check != "exact":
        print(f"bench.py: frame check failed: {frame_check}", file=sys.stderr, flush=True)
        rc = 4
    if native:
        pipe.close()
    sharder.close()
    r.close()
    if world > 1:
        dist.destroy_process_group()
    return rc


if __name__ == "__main__":
    sys.exit(main())
