"""Summarise tools/pmc.sh output: mean per march-kernel dispatch + derived."""
import collections
import csv
import glob
import json
import sys

CPI = 2.74   # --cpi

def load(tag, kernel="march"):
    agg = collections.defaultdict(list)
    for f in sorted(glob.glob(f"gpurun_out/pmc_{tag}/p*/run_counter_collection.csv")):
        for row in csv.DictReader(open(f)):
            if kernel not in row["Kernel_Name"]:
                continue
            agg[row["Counter_Name"]].append(float(row["Counter_Value"]))
    return {k: sum(v) / len(v) for k, v in agg.items()}


def derived(c):
    d = {}
    if "GRBM_GUI_ACTIVE" in c:
        d["gpu_cycles_per_xcd"] = c["GRBM_GUI_ACTIVE"] / 8
    if "SQ_INSTS_VALU" in c and "GRBM_GUI_ACTIVE" in c:
        # VALU wave-instructions per SIMD-cycle (1,024 SIMDs; GRBM_GUI_ACTIVE
        # sums the 8 XCDs), and the VALU issue utilisation: that times the
        # kernel's mean calibrated SIMD cycles per wave64 instruction (its
        # static opcode mix weighted by tools/isa_cost.py, profiles/valu_calib.txt;
        # --cpi, default 2.74 = the procedural density's, tools/proc_isa_report.py).
        # (Round 4's valu_busy divided SQ_ACTIVE_INST_VALU, a per-wave
        # count, by per-SIMD quad-cycles and read above 1.)
        ipc = c["SQ_INSTS_VALU"] / (1024 * c["GRBM_GUI_ACTIVE"] / 8)
        d["valu_insts_per_simd_cycle"] = ipc
        d["valu_issue_util"] = ipc * CPI
    for k in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY", "SQ_WAIT_INST_LDS", "SQ_ACTIVE_INST_LDS"):
        if k in c and "SQ_WAVE_CYCLES" in c:
            d[k + "_frac"] = c[k] / c["SQ_WAVE_CYCLES"]
    if "TCC_HIT_sum" in c:
        d["l2_hit"] = c["TCC_HIT_sum"] / max(1.0, c["TCC_HIT_sum"] + c["TCC_MISS_sum"])
    if "TCP_TCC_READ_REQ_sum" in c and "TCP_TOTAL_CACHE_ACCESSES_sum" in c:
        d["l1_miss_ratio"] = c["TCP_TCC_READ_REQ_sum"] / max(1.0, c["TCP_TOTAL_CACHE_ACCESSES_sum"])
    if "FETCH_SIZE" in c:
        d["fetch_MB_x2"] = c["FETCH_SIZE"] * 1024 * 2 / 1e6   # gfx950: FETCH_SIZE under-counts 2x
    cyc = c.get("GRBM_GUI_ACTIVE", 0) / 8
    if cyc:
        for k, n in (("TA_TA_BUSY_sum", "ta_busy"), ("TD_TD_BUSY_sum", "td_busy")):
            if k in c:
                d[n] = c[k] / (256 * cyc)   # 256 CUs
    vm = c.get("SQ_INSTS_VMEM_RD", 0)
    if vm:
        for k, n in (("TA_TA_BUSY_sum", "ta_cycles_per_vmem_inst"), ("TD_TD_BUSY_sum", "td_cycles_per_vmem_inst"),
                     ("TCP_TOTAL_CACHE_ACCESSES_sum", "l1_lookups_per_vmem_inst")):
            if k in c:
                d[n] = c[k] / vm
    if "SQ_ACTIVE_INST_LDS" in c and cyc:
        d["lds_issue_busy_per_cu"] = c["SQ_ACTIVE_INST_LDS"] / (256 * cyc)   # LDS issue cycles per CU cycle
    if "SQ_LDS_BANK_CONFLICT" in c and c.get("SQ_INSTS_LDS"):
        d["lds_conflict_cycles_per_lds_inst"] = c["SQ_LDS_BANK_CONFLICT"] / c["SQ_INSTS_LDS"]
    if "TCC_EA0_RDREQ_sum" in c:
        d["ea_rdreq_MB_64B"] = c["TCC_EA0_RDREQ_sum"] * 64 / 1e6
    return d


if __name__ == "__main__":
    # TAG or TAG:KERNEL (substring of the kernel name; default "march") [--cpi X]
    args = sys.argv[1:]
    if "--cpi" in args:
        i = args.index("--cpi")
        CPI = float(args[i + 1])
        del args[i:i + 2]
    for arg in args:
        tag, _, kern = arg.partition(":")
        c = load(tag, kern or "march")
        print(arg, json.dumps({k: round(v, 4) for k, v in {**c, **derived(c)}.items()}, indent=0))
