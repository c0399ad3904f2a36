"""Write profiles/traffic.json from a tools/pmc.sh run of the bench config.

HBM bytes per march-kernel launch = FETCH_SIZE*1024*2 + WRITE_SIZE*1024
(KB units; x2 on FETCH_SIZE per MI355X_MICROARCH.md sec. HBM: gfx950 tallies
128-B reads at 64 B).  Counters come from separate --pmc passes.  When the run
has a TCP_TOTAL_CACHE_ACCESSES_sum / TA_TA_BUSY_sum / GRBM_GUI_ACTIVE pass, the
L1 lookups per launch and the TA busy fraction go in too: the TA-lookup
roofline of the bench line (bench.py).
"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from pmc_summary import load  # noqa: E402

tag, config, out = sys.argv[1], sys.argv[2], sys.argv[3]
c = load(tag)
kernel = None
for line in open(f"gpurun_out/pmc_{tag}/p1.log"):
    if line.startswith("variant "):
        kernel = line.split()[1]
fetch = c["FETCH_SIZE"] * 1024 * 2
write = c["WRITE_SIZE"] * 1024
res = {"config": config, "kernel": kernel, "hbm_bytes_per_launch": round(fetch + write),
       "fetch_bytes": round(fetch), "write_bytes": round(write),
       "raw": {k: c[k] for k in ("FETCH_SIZE", "WRITE_SIZE") if k in c},
       "method": "rocprofv3 --pmc FETCH_SIZE and --pmc WRITE_SIZE in separate passes over tools/prof_case.py "
                 "(20 launches, mean per march launch); FETCH_SIZE x2 per the gfx950 correction"}
if "TCP_TOTAL_CACHE_ACCESSES_sum" in c:
    res["l1_lookups_per_launch"] = round(c["TCP_TOTAL_CACHE_ACCESSES_sum"])
    res["raw"]["TCP_TOTAL_CACHE_ACCESSES_sum"] = c["TCP_TOTAL_CACHE_ACCESSES_sum"]
    res["method"] += "; a third pass TCP_TOTAL_CACHE_ACCESSES_sum TA_TA_BUSY_sum GRBM_GUI_ACTIVE SQ_INSTS_VMEM_RD"
if "TA_TA_BUSY_sum" in c and c.get("GRBM_GUI_ACTIVE"):
    res["ta_busy"] = round(c["TA_TA_BUSY_sum"] / (256 * c["GRBM_GUI_ACTIVE"] / 8), 4)   # 256 CUs, 8 XCDs
    res["raw"].update({k: c[k] for k in ("TA_TA_BUSY_sum", "GRBM_GUI_ACTIVE", "SQ_INSTS_VMEM_RD") if k in c})
os.makedirs(os.path.dirname(out), exist_ok=True)
json.dump(res, open(out, "w"), indent=1)
print(json.dumps(res))
