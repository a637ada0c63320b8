"""Summarise rocprofv3 PMC databases (rocpd sqlite, counters_collection view):
per kernel name, the mean of every counter over its dispatches and the mean
duration.  usage: pmc_summary.py DB [DB ...] [--match SUBSTR]"""
import sqlite3
import sys
from collections import defaultdict

args = [a for a in sys.argv[1:] if not a.startswith("--")]
match = None
if "--match" in sys.argv:
    match = sys.argv[sys.argv.index("--match") + 1]
    args.remove(match)
for db in args:
    con = sqlite3.connect(db)
    cols = [r[1] for r in con.execute("pragma table_info(counters_collection)")]
    rows = con.execute("select * from counters_collection").fetchall()
    name_c = cols.index("kernel_name") if "kernel_name" in cols else None
    cnt_c, val_c = cols.index("counter_name"), cols.index("value")
    disp_c = cols.index("dispatch_id")
    agg = defaultdict(lambda: defaultdict(float))
    disp = defaultdict(set)
    dur = {}
    for r in rows:
        k = r[name_c]
        if match and match not in k:
            continue
        agg[k][r[cnt_c]] += r[val_c]
        disp[k].add(r[disp_c])
    for k in agg:
        n = len(disp[k])
        short = k[:110]
        print(f"== {db}\n  {short}  dispatches={n}")
        for c, v in sorted(agg[k].items()):
            print(f"    {c:28s} {v / n:16.4g}")
