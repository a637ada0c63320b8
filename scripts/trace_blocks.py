#!/usr/bin/env python3
"""Timeline of a rocprofv3 kernel trace (measurement tool): every dispatch
from the first one whose name matches --from (default: the last 40
dispatches), start / end in us relative to the first shown, duration, queue,
grid and a short kernel name.

  python3 scripts/trace_blocks.py gpurun_out/r06/a/trace_loop96/run_kernel_trace.csv [--last 40]
"""
import argparse
import csv
import re


def short(name):
    name = re.sub(r"life::\(anonymous namespace\)::", "", name)
    name = re.sub(r"\(.*$", "", name)
    return name[:70]


def main():
    p = argparse.ArgumentParser()
    p.add_argument("csv")
    p.add_argument("--last", type=int, default=40)
    p.add_argument("--skip", type=int, default=0, help="omit this many dispatches at the end")
    a = p.parse_args()
    rows = list(csv.DictReader(open(a.csv)))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    rows = rows[:len(rows) - a.skip] if a.skip else rows
    rows = rows[-a.last:]
    t0 = int(rows[0]["Start_Timestamp"])
    for r in rows:
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        print(f"{(s - t0) / 1e3:9.1f} {(e - t0) / 1e3:9.1f} {(e - s) / 1e3:8.1f}  q{r['Queue_Id']:>2} "
              f"grid {int(r['Grid_Size_X']) // max(1, int(r['Workgroup_Size_X'])):6d}  {short(r['Kernel_Name'])}")


if __name__ == "__main__":
    main()
