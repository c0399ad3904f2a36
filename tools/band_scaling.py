"""Per-rank render time of the strong-scaled frame on ONE GPU: rank 0's band
set (16-row bands, stride N) for N = 1, 2, 4, 8, against the whole frame / N.
What a rank of bench.py --gpus N renders per frame, without the exchange.

    python tools/band_scaling.py [--size 512] [--config grid512] [--tpw 0] [--schedule -1]

--native: the frame STREAM of each rank instead of one launch -- the native
frame loop (libvr_shard, vr_shard_run_frames) in its solo rehearsal
(vr_shard_set_solo: this rank's band set only, no exchange), `--frames`
frames queued at once, timed with events on the caller's stream from before
the first render to after the last; ms per frame and the loop's host ms per
frame, with 1 and 2 render streams (vr_shard_set_render_streams), `--rounds`
interleaved rounds.
"""
import argparse
import os
import sys

import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import volumetricrenderer_amd as vr  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--size", type=int, default=512)
    ap.add_argument("--width", type=int, default=1920)
    ap.add_argument("--height", type=int, default=1080)
    ap.add_argument("--steps", type=int, default=128)
    ap.add_argument("--frames", type=int, default=20)
    ap.add_argument("--variants", default="-1:0:0", help="comma list of schedule:tiles_per_wave:split[:wedges]")
    ap.add_argument("--opt", action="append", default=[], help="vr option NAME=VALUE, set first")
    ap.add_argument("--ns", default="1,2,4,8")
    ap.add_argument("--band-rows", type=int, default=16)
    ap.add_argument("--all-ranks", action="store_true", help="time every rank's band set, report the slowest")
    ap.add_argument("--rank", type=int, default=0, help="--native without --all-ranks: the rank to rehearse")
    ap.add_argument("--native", action="store_true", help="per-rank frame streams through the native loop (solo)")
    ap.add_argument("--streams", default="1,2", help="--native: render streams to compare")
    ap.add_argument("--rounds", type=int, default=3, help="--native: interleaved rounds")
    ap.add_argument("--threads", type=int, default=1, help="--native: host threads of the frame loop (1 or 2)")
    ap.add_argument("--compositor", default="auto", choices=["auto", "on", "off", "on8"],
                    help="--native: rank 0 renders no bands and only assembles (vr_shard_set_compositor; auto: the "
                         "library's default, on from 8 ranks)")
    ap.add_argument("--rows", action="append", default=[],
                    help="--native, row ranges: explicit row starts (comma list, renderers + 1 entries); repeatable")
    ap.add_argument("--rebalance", action="store_true",
                    help="--native --all-ranks, row ranges: a second pass with the ranges split again by every "
                         "rank's measured render time (vr_row_partition_measured, as vr_shard_rebalance_rows does)")
    ap.add_argument("--lead-pct", type=int, default=-1,
                    help="--native, compositor over band sets: rank 0 also renders lead rows, counted as this %% of a "
                         "renderer (vr_shard_balance_lead); -1 = the pipeline's auto choice, 0 = no lead rows")
    ap.add_argument("--partition", default="auto", choices=["auto", "bands", "rows"],
                    help="--native: interleaved band sets or balanced contiguous row ranges (RcclBandPipeline)")
    ap.add_argument("--exchange", default="render", choices=["render", "comm"],
                    help="--native: the exchange on the render streams (default) or on a communication stream "
                         "(vr_shard_set_exchange_streams 1 / 0)")
    ap.add_argument("--serpentine", default="auto", choices=["auto", "on", "off"],
                    help="--native: band sets dealt serpentine (vr_shard_set_serpentine; auto = the library default)")
    ap.add_argument("--clock-warm-ms", type=float, default=150.0,
                    help="--native: whole frames for this long before the first timing (bench.py --clock-warm-ms)")
    ap.add_argument("--gate-ms", type=float, default=0.0,
                    help="--native: hold the stream with a spin kernel of this many ms while the host queues the "
                         "frames, so the timing is the GPU's alone (not the host's)")
    a = ap.parse_args()
    if a.native:
        return native(a)
    W, H = a.width, a.height
    with vr.Renderer(0) as r:
        r.generate_volume(vr.scaled_recipe(a.size))
        print(f"{a.size}^3, {W}x{H}x{a.steps}", flush=True)
        osd, gsd = vr.reference_shader_data(1280 / 720)
        r.set_shader_data(osd, gsd)
        r.set_march(vr.march_defaults(max_steps=a.steps))
        for o in a.opt:
            k, v = o.split("=")
            r.set_option(k, int(v))
        for var in a.variants.split(","):
            vals = [int(v) for v in var.split(":")]
            sched, tpw, split = vals[:3]
            wedges = vals[3] if len(vals) > 3 else 0
            r.set_option("schedule", sched)
            r.set_option("tiles_per_wave", tpw)
            r.set_option("split", split)
            if wedges:
                r.set_option("wedges", wedges)
            base = None
            for n in [int(v) for v in a.ns.split(",")]:
                ts = []
                for first in (range(n) if a.all_ranks else (0,)):
                    band = dict(band_rows=a.band_rows, band_stride=n, band_first=first)
                    out = r.alloc_target(W, H, 1, **band)
                    r.render(W, H, 1, out=out, **band)
                    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2 * a.frames)]
                    for i in range(a.frames):
                        ev[2 * i].record()
                        r.render(W, H, 1, out=out, **band)
                        ev[2 * i + 1].record()
                    torch.cuda.synchronize()
                    ts.append(float(np.median([ev[2 * i].elapsed_time(ev[2 * i + 1]) for i in range(a.frames)])))
                    if a.all_ranks:
                        print(f"    N={n} rank {first}: region_work_tiles {r.get_option('region_work_tiles')}", flush=True)
                t = max(ts)
                if a.all_ranks:
                    print(f"  N={n} band_rows {a.band_rows}: per-rank ms " + " ".join(f"{v:.4f}" for v in ts), flush=True)
                base = base or t
                print(f"{' '.join(a.opt)} schedule {sched} tpw {tpw} split {split} wedges {wedges} N={n}: rank-0 bands {t:.4f} ms, whole/N {base / n:.4f} ms, "
                      f"efficiency {base / n / t:.2f}", flush=True)


def native(a):
    """Per-rank frame streams of the native loop (solo rehearsal), 1 vs 2 render streams."""
    W, H = a.width, a.height
    with vr.Renderer(0) as r:
        r.generate_volume(vr.scaled_recipe(a.size))
        osd, gsd = vr.reference_shader_data(1280 / 720)
        r.set_shader_data(osd, gsd)
        r.set_march(vr.march_defaults(max_steps=a.steps))
        for o in a.opt:
            k, v = o.split("=")
            r.set_option(k, int(v))
        print(f"native frame streams: {a.size}^3, {W}x{H}x{a.steps}, {a.frames} frames per timing, "
              f"{a.threads} host thread(s), gate {a.gate_ms} ms, partition {a.partition}, exchange on {a.exchange} "
              "streams, "
              f"variant {r.kernel_variant} serpentine {a.serpentine} {' '.join(a.opt)}", flush=True)
        streams = [int(v) for v in a.streams.split(",")]
        if a.clock_warm_ms > 0:   # the GPU settles over the first 20-40 ms of load
            out = r.alloc_target(W, H, vr.FMT_RGBA8_UNORM)
            t0, k = time.perf_counter(), 0
            while (time.perf_counter() - t0) * 1e3 < a.clock_warm_ms:
                for _ in range(8):
                    r.render(W, H, vr.FMT_RGBA8_UNORM, out=out)
                torch.cuda.synchronize()
                k += 8
            print(f"  clock warm: {k} whole frames, {a.clock_warm_ms:.0f} ms", flush=True)
        base = {}
        for rows in a.rows:
            rl = [int(v) for v in rows.split(",")]
            print(f"  rows {rl}", flush=True)
            one_n(a, r, W, H, len(rl) - 1 + (1 if a.compositor == "on" else 0), streams, base, rl)
        for n in ([] if a.rows else [int(v) for v in a.ns.split(",")]):
            info = one_n(a, r, W, H, n, streams, base, None)
            if a.rebalance and a.all_ranks and n > 1 and info["ranges"]:
                first_r = min(info["ranges"])   # 0, or 1 with rank 0 as a compositor
                prev = [info["ranges"][k][0] for k in sorted(info["ranges"])] + [H]
                ms = [info["kms"][k] for k in sorted(info["ranges"])]
                pct = 100 if first_r == 1 else max(50, 100 - 2 * (n - 1))
                old = r.get_option("row_first_pct")
                r.set_option("row_first_pct", pct)
                new = r.row_partition_measured(W, H, prev, ms)
                r.set_option("row_first_pct", old)
                print(f"  rebalanced: ranges {prev} -> {new} (render ms per rank " + " ".join(f"{v:.4f}" for v in ms) + ")",
                      flush=True)
                one_n(a, r, W, H, n, streams, base, new)


def one_n(a, r, W, H, n, streams, base, rows):
    """One world size's per-rank frame streams; rows: explicit row starts."""
    from volumetricrenderer_amd.distributed import RcclBandPipeline
    res = {ns: [] for ns in streams}   # per stream count: per round, the slowest rank's ms/frame
    per_rank = {ns: {} for ns in streams}   # per stream count, rank: ms/frame per round
    host = {ns: [] for ns in streams}
    # one rank's pipeline at a time: its streams get HIP's hardware
    # queues to themselves (GPU_MAX_HW_QUEUES = 4 per process), as in
    # the N-process run; pipelines of all ranks alive at once would
    # share queues and serialise each other's render streams
    per_round = {ns: [[] for _ in range(a.rounds)] for ns in streams}
    ranges, kms = {}, {}
    for first in (range(n) if a.all_ranks else (min(a.rank, n - 1),)):
        for ns in streams:
            p = RcclBandPipeline(r, W, H, vr.FMT_RGBA8_UNORM, band_rows=a.band_rows, world=n, rank=first,
                                 loopback=True, solo=True, render_streams=ns, host_threads=a.threads,
                                 exchange_on_render=a.exchange == "render",
                                 compositor=(None if a.compositor == "auto" or n < 2 or (a.compositor == "on8" and n < 8)
                                             else a.compositor in ("on", "on8")),
                                 partition="rows" if rows else a.partition, rows=rows,
                                 lead_pct=("auto" if a.lead_pct < 0 or n < 2 or (a.compositor == "on8" and n < 8)
                                           else (a.lead_pct or None)),
                                 serpentine=None if a.serpentine == "auto" else a.serpentine == "on")
            p.run_frames(8)   # region lists, code objects
            p.barrier()
            if first == 0 and p.lead_rows and ns == streams[0]:
                print(f"  N={n}: rank 0 lead rows {p.lead_rows}", flush=True)
            for k in range(a.rounds):
                p.run_frames(4)
                p.barrier()
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                if a.gate_ms > 0:   # ~2.1 GHz shader clock under this load
                    torch.cuda._sleep(int(a.gate_ms * 1e-3 * 2.1e9))
                e0.record()
                p.run_frames(a.frames)
                e1.record()
                torch.cuda.synchronize()
                ms = e0.elapsed_time(e1) / a.frames
                per_round[ns][k].append(ms)
                per_rank[ns].setdefault(first, []).append(ms)
                host[ns].append(p.host_ms)
            if p.row_range is not None and ns == streams[-1] and not (p.compositor and first == 0):
                ranges[first] = p.row_range
                kms[first] = p.run_frames(16, sample_every=1)
            p.close()
    for ns in streams:
        res[ns] = [max(v) for v in per_round[ns]]
    for ns in streams:
        t = float(np.median(res[ns]))
        if n == 1:
            base[ns] = t
        b = base.get(ns)
        eff = f", efficiency {b / n / t:.2f} (vs N=1, same streams)" if b else ""
        print(f"N={n} render_streams {ns}{' rebalanced' if rows else ''}: slowest rank {t:.4f} ms/frame (rounds "
              + " ".join(f"{v:.4f}" for v in res[ns]) + f"), host {max(host[ns]):.4f} ms/frame{eff}",
              flush=True)
        if a.all_ranks and n > 1:
            print("  per rank (median ms/frame): " + " ".join(
                f"{k}:{float(np.median(v)):.4f}" for k, v in sorted(per_rank[ns].items())), flush=True)
    return {"ranges": ranges, "kms": kms}


if __name__ == "__main__":
    main()
