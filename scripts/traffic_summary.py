#!/usr/bin/env python3
"""profiles/<round>/pmc_{FETCH,WRITE}_SIZE_<variant>.csv -> profiles/traffic.json.

HBM bytes per stencil launch from rocprofv3 FETCH_SIZE / WRITE_SIZE (KiB per
dispatch, each counter from its own --pmc pass), read as
MI355X_MICROARCH.md's HBM section prescribes for gfx950:

* 16-B-per-lane streaming kernels (step_kernel, byte and one-generation
  bit): FETCH_SIZE reports half the bytes of wide coalesced reads, so it is
  doubled; WRITE_SIZE is exact for 16-B streaming stores.
* the temporal byte kernel moves 2 x 16 B per lane: calibrated as above;
* the temporal bit kernel loads and stores 4 B per lane (natural-word tiles,
  rounds 1-2) or 8 B per lane (interleaved-pair tiles, tstep_bit_kernel,
  round 3), access widths the guide lists as uncalibrated:
  copies of 1 GiB with 4-B / 8-B lanes read FETCH_SIZE = 0.500 GiB,
  WRITE_SIZE = 1.000 GiB (profiles/r01/calib_4b_*.csv, recorded by the
  4-B calibration kernel retired in round 4 -- in git history before
  commit 31896c8; profiles/r03/calib_8b_*.csv from scripts/calib_8b.hip), so
  the same x2 / x1 applies.

Only full-length launches are summarised (the median over the dispatches of
the dominant kernel).
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

VARIANTS = {  # variant -> (kernel-name substrings (any round's name), calibrated access)
    "bit_onegen": (("step_kernel<life::(anonymous namespace)::BitEnc",), True),
    "byte_onegen": (("step_kernel<life::(anonymous namespace)::ByteEnc",), True),
    "bit_temporal": (("tstep_bit_kernel<", "tstep_kernel<false"), True),  # 8 B (r03) / 4 B per lane (calib_8b / 4b)
    "byte_temporal": (("tstep_byte_kernel<", "tstep_kernel<true"), True),  # 2 x 16 B per lane
    "bit_flow": (("tflow_kernel<",), True),  # sc1; one dispatch = PASSES[var] passes
}
# dataflow launches run several passes per dispatch: the PMC job times a
# 80-generation call at 20 generations per pass (profiles/r02/jobs/r2r.sh);
# FLOW_PASSES overrides (profiles/r05/z: a 96-generation call, 8 x 12)
PASSES = {"bit_flow": int(os.environ.get("FLOW_PASSES", "4"))}

out = {}
for var, (needle, calibrated) in VARIANTS.items():
    vals = {}
    for c in ("FETCH_SIZE", "WRITE_SIZE"):
        p = os.path.join(d, f"pmc_{c}_{var}.csv")
        if not os.path.exists(p):
            continue
        rows = [r for r in csv.DictReader(open(p))
                if any(n in r["Kernel_Name"] for n in needle) and r["Counter_Name"] == c]
        if not rows:
            continue
        # the longest dispatches are the full-length launches
        durs = [int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in rows]
        full = [float(r["Counter_Value"]) for r, t in zip(rows, durs) if t >= 0.8 * max(durs)]
        vals[c] = statistics.median(full) * 1024.0 / PASSES.get(var, 1)
    if len(vals) != 2:
        continue
    key = f"{var}_{size}"
    if calibrated:
        fetch = 2.0 * vals["FETCH_SIZE"]
        out[key] = round(fetch + vals["WRITE_SIZE"])
        out[key + "_detail"] = {"fetch_bytes_corrected": round(fetch), "fetch_size_raw_bytes": round(vals["FETCH_SIZE"]),
                                "write_bytes": round(vals["WRITE_SIZE"]), "source": f"profiles/{rnd}/pmc_*_{var}.csv",
                                "correction": "FETCH_SIZE x2 (gfx950; 16 B/lane per MI355X_MICROARCH.md, 4 B / 8 B "
                                              "per lane by the recorded calibration runs profiles/r01/calib_4b_*.csv "
                                              "and profiles/r03/calib_8b_*.csv)", "calibrated": True}
    else:
        out[key] = None
        out[key + "_detail"] = {"fetch_size_raw_bytes": round(vals["FETCH_SIZE"]),
                                "write_size_raw_bytes": round(vals["WRITE_SIZE"]),
                                "source": f"profiles/{rnd}/pmc_*_{var}.csv", "calibrated": False,
                                "note": "4 B/lane loads and stores: access width uncalibrated on gfx950 "
                                        "(MI355X_MICROARCH.md, HBM); raw counter values, not HBM bytes"}
# merge: entries of other rounds / variants stay
path = os.path.join(ROOT, "profiles", "traffic.json")
try:
    with open(path) as f:
        merged = json.load(f)
except (OSError, ValueError):
    merged = {}
merged.update(out)
with open(path, "w") as f:
    json.dump(merged, f, indent=1)
print(json.dumps(out, indent=1))
