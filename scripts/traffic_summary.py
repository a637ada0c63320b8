#!/usr/bin/env python3
"""profiles/<round>/pmc_*_<kernel>.csv -> profiles/traffic.json.

HBM bytes per stencil launch from rocprofv3 FETCH_SIZE / WRITE_SIZE (KiB per
dispatch), corrected as MI355X_MICROARCH.md's HBM section prescribes for
gfx950: FETCH_SIZE reports half the bytes of wide (16 B/lane) coalesced
streaming reads, so it is doubled; WRITE_SIZE is exact for 16-B streaming
stores.  Each counter came from its own --pmc pass.
"""
import csv
import json
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
rnd = sys.argv[1] if len(sys.argv) > 1 else "r01"
size = int(sys.argv[2]) if len(sys.argv) > 2 else 65536
d = os.path.join(ROOT, "profiles", rnd)
out = {}
for k in ("bit", "byte"):
    vals = {}
    for c in ("FETCH_SIZE", "WRITE_SIZE"):
        p = os.path.join(d, f"pmc_{c}_{k}.csv")
        if not os.path.exists(p):
            continue
        v = [float(r["Counter_Value"]) for r in csv.DictReader(open(p)) if "step_kernel" in r["Kernel_Name"]]
        vals[c] = statistics.median(v) * 1024.0
    if len(vals) == 2:
        fetch = 2.0 * vals["FETCH_SIZE"]
        out[f"{k}_{size}"] = round(fetch + vals["WRITE_SIZE"])
        out[f"{k}_{size}_detail"] = {"fetch_bytes_corrected": round(fetch), "fetch_size_raw_bytes": round(vals["FETCH_SIZE"]),
                                     "write_bytes": round(vals["WRITE_SIZE"]), "source": f"profiles/{rnd}/pmc_*_{k}.csv",
                                     "correction": "FETCH_SIZE x2 (gfx950, 16 B/lane streaming reads)"}
with open(os.path.join(ROOT, "profiles", "traffic.json"), "w") as f:
    json.dump(out, f, indent=1)
print(json.dumps(out, indent=1))
