"""Per-instruction L1 lookups / TA busy / time of each tools/tcp_calib pattern."""
import collections
import csv
import glob

N_INSTR = 1024 * 4 * 64   # blocks x waves x loads per pattern launch


def main():
    vals = collections.defaultdict(dict)
    for f in glob.glob("gpurun_out/calib/*/run_counter_collection.csv"):
        acc = collections.defaultdict(list)
        for r in csv.DictReader(open(f)):
            if ("k_pattern" in r["Kernel_Name"] or "k_wide" in r["Kernel_Name"]):
                acc[(r["Kernel_Name"].split("(")[0], r["Counter_Name"])].append(float(r["Counter_Value"]))
        for (k, c), v in acc.items():
            vals[k][c] = sum(v) / len(v)
    dur = collections.defaultdict(list)
    for r in csv.DictReader(open("gpurun_out/calib/trace/run_kernel_trace.csv")):
        if ("k_pattern" in r["Kernel_Name"] or "k_wide" in r["Kernel_Name"]):
            dur[r["Kernel_Name"].split("(")[0]].append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
    for k in sorted(vals):
        v = vals[k]
        d = sorted(dur[k])[len(dur[k]) // 2] if dur[k] else 0
        print(f"{k:45s} lookups/instr {v.get('TCP_TOTAL_CACHE_ACCESSES_sum', 0) / N_INSTR:6.2f}  "
              f"TA busy/instr {v.get('TA_TA_BUSY_sum', 0) / N_INSTR:6.2f}  "
              f"L2 req/instr {v.get('TCP_TCC_READ_REQ_sum', 0) / N_INSTR:6.2f}  {d / 1e3:8.1f} us")


if __name__ == "__main__":
    main()
