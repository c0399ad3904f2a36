"""Per-instruction TA / TD / L1 figures of each tools/lds_dma_calib kernel."""
import collections
import csv
import glob
import sys

N_INSTR = 2048 * 4 * 64   # blocks x waves x loads per launch


def main():
    out = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/ldscal"
    vals = collections.defaultdict(dict)
    for f in glob.glob(f"{out}/*/run_counter_collection.csv") + glob.glob(f"{out}/*/*/run_counter_collection.csv"):
        acc = collections.defaultdict(list)
        for r in csv.DictReader(open(f)):
            k = r["Kernel_Name"].split("(")[0]
            if k.startswith(("void k_", "k_")):
                acc[(k, r["Counter_Name"])].append(float(r["Counter_Value"]))
        for (k, c), v in acc.items():
            vals[k][c] = sum(v) / len(v)
    dur = collections.defaultdict(list)
    for f in glob.glob(f"{out}/trace/**/run_kernel_trace.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            k = r["Kernel_Name"].split("(")[0]
            if k.startswith(("void k_", "k_")):
                dur[k].append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
    for k in sorted(vals):
        v = vals[k]
        d = sorted(dur[k])[len(dur[k]) // 2] if dur[k] else 0
        print(f"{k:32s} lookups {v.get('TCP_TOTAL_CACHE_ACCESSES_sum', 0) / N_INSTR:6.2f}  "
              f"TA {v.get('TA_TA_BUSY_sum', 0) / N_INSTR:6.2f}  TD {v.get('TD_TD_BUSY_sum', 0) / N_INSTR:6.2f}  "
              f"L2req {v.get('TCP_TCC_READ_REQ_sum', 0) / N_INSTR:6.2f}  {d / 1e3:8.1f} us")


if __name__ == "__main__":
    main()
