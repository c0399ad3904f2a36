"""Write profiles/traffic.json from a tools/pmc.sh run of the bench config.

HBM bytes per march-kernel launch = FETCH_SIZE*1024*2 + WRITE_SIZE*1024
(KB units; x2 on FETCH_SIZE per MI355X_MICROARCH.md sec. HBM: gfx950 tallies
128-B reads at 64 B).  Counters come from separate --pmc passes.
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
os.makedirs(os.path.dirname(out), exist_ok=True)
json.dump(res, open(out, "w"), indent=1)
print(json.dumps(res))
