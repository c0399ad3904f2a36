"""Copy a tools/round_profiles.sh run from gpurun_out/ into profiles/ (tracked):
the bench line of each config -> profiles/r01_bench_<config>.json and the
rocprofv3 --kernel-trace --stats summary of the same bench command ->
profiles/r01_<config>_kernel_stats.csv, plus a check that the stats' mean
march-kernel duration agrees with the bench's HIP-event mean.

    python tools/collect_profiles.py [round-tag r01] [configs...]
"""
import csv
import json
import os
import shutil
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def main():
    tag = sys.argv[1] if len(sys.argv) > 1 else "r01"
    configs = sys.argv[2:] or ["grid512", "grid128", "grid4k", "cloud", "cloud_shadow"]
    out = os.path.join(ROOT, "profiles")
    for c in configs:
        log = os.path.join(ROOT, "gpurun_out", f"bench_{c}.log")
        line = [ln for ln in open(log).read().splitlines() if ln.startswith("{")][-1]
        bench = json.loads(line)
        with open(os.path.join(out, f"{tag}_bench_{c}.json"), "w") as f:
            f.write(line + "\n")
        stats = os.path.join(ROOT, "gpurun_out", f"prof_{c}", "run_kernel_stats.csv")
        if not os.path.exists(stats):   # rocprofv3 nests its output under host/pid dirs
            for dp, _, fs in os.walk(os.path.join(ROOT, "gpurun_out", f"prof_{c}")):
                for fn in fs:
                    if fn.endswith("kernel_stats.csv"):
                        stats = os.path.join(dp, fn)
        shutil.copy(stats, os.path.join(out, f"{tag}_{c}_kernel_stats.csv"))
        march = [r for r in csv.DictReader(open(stats)) if "march" in r["Name"]]
        # a "_u<channel>" bench kernel (uniform channel skipped) is the march_regions_u
        # instance whose last template argument is that channel's bit; the bench's
        # all-channels comparison run adds plain march_regions to the same trace
        variant = bench["config"].get("kernel", "")
        if "_u" in variant:
            bit = {"R": 1, "G": 2, "B": 4, "A": 8}[variant[-1]]
            march = [r for r in march if f", {bit}>(" in r["Name"]] or march
        if variant.endswith("_deferred"):
            # deferred shadow rays: a frame is five launches; their mean durations add up
            # to what the bench's events bracket
            passes = [r for r in csv.DictReader(open(stats))
                      if any(k in r["Name"] for k in ("march_proc_defer", "proc_shadow_scan", "proc_shadow_map",
                                                       "proc_shadow_eval", "proc_shadow_resolve"))]
            parts = ", ".join(f"{r['Name'].split('namespace)::')[-1].split('(')[0]} {float(r['AverageNs']) / 1e6:.4f}"
                              for r in passes)
            tot = sum(float(r["AverageNs"]) for r in passes) / 1e6
            print(f"{c:13s} bench {bench['value']:>14,.1f} {bench['unit']}  kernel(events) "
                  f"{bench['kernel_ms_mean']:.4f} ms  rocprof passes sum {tot:.4f} ms ({parts})  "
                  f"roofline {bench['roofline']['frac']}")
            continue
        top = max(march, key=lambda r: float(r["TotalDurationNs"]))
        # the timed launches only: the last `steps` dispatches of that kernel in the trace
        timed = ""
        trace = stats.replace("kernel_stats.csv", "kernel_trace.csv")
        if os.path.exists(trace):
            rows = [r for r in csv.DictReader(open(trace)) if r.get("Kernel_Name") == top["Name"]]
            last = rows[-bench["steps"]:]
            if last:
                ms = sum(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in last) / len(last) / 1e6
                timed = f" (timed {len(last)}: {ms:.4f} ms)"
        print(f"{c:13s} bench {bench['value']:>14,.1f} {bench['unit']}  kernel(events) {bench['kernel_ms_mean']:.4f} ms  "
              f"rocprof {top['Name'][:60]} avg {float(top['AverageNs']) / 1e6:.4f} ms x{top['Calls']}{timed}  "
              f"roofline {bench['roofline']['frac']}")


if __name__ == "__main__":
    main()
