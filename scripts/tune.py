#!/usr/bin/env python3
"""A/B the stencil variants (rows per lane x prefetch depth) in ONE process,
interleaved over rounds, at the bench workload (random 50% N^2, 1 GPU).

Prints one JSON line per (kernel, rows, depth): median / min kernel ms and
the algorithmic GB/s, plus the live count after the run (every variant must
agree: they compute the same generations).
"""
import argparse
import json
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "mpi-and-open-mp_amd"))
import life_mi355x as lm  # noqa: E402

p = argparse.ArgumentParser()
p.add_argument("--size", type=int, default=65536)
p.add_argument("--kernels", default="bit,byte")
p.add_argument("--rows", default="16,32,64")
p.add_argument("--depths", default="2,4,8")
p.add_argument("--gens", type=int, default=10)
p.add_argument("--rounds", type=int, default=3)
p.add_argument("--temporal", default="", help="bit temporal tile heights to A/B, e.g. 48,64,80,96")
a = p.parse_args()

if a.temporal:
    heights = [int(v) for v in a.temporal.split(",")]
    tk = a.kernels.split(",")[0]
    life = lm.Life(a.size, a.size, kernel=tk)
    K = life.layout().generations_per_exchange
    life.fill_random(1, 0.5)
    res = {v: [] for v in heights}
    for rnd in range(a.rounds):
        for v in heights:
            lm.tune_temporal(v, tk)
            life.step(K)
            life.sync()
            life.set_timing(True)
            life.step(K * a.gens)
            ms, n, b = life.kernel_stats()
            upd, valu = life.kernel_work()
            life.set_timing(False)
            res[v].append((ms, b, upd, valu))
    for v in heights:
        med = statistics.median(m for m, *_ in res[v])
        _, b, upd, valu = res[v][0]
        print(json.dumps({"kernel": tk + "-temporal", "rows_per_wave": v, "K": K, "median_ms_per_launch": round(med, 4),
                          "gens_per_launch": round(upd / (b / (0.25 if tk == "bit" else 2.0)), 3),
                          "Gcells_per_s": round(upd / med / 1e6, 1),
                          "hbm_GBps": round(b / med / 1e6, 1), "valu_Tops": round(valu / med / 1e9, 2),
                          "live": life.live_count()}), flush=True)
    life.close()
    sys.exit(0)

variants = [(r, d) for r in map(int, a.rows.split(",")) for d in map(int, a.depths.split(","))]
for kernel in a.kernels.split(","):
    life = lm.Life(a.size, a.size, kernel=kernel)
    life.fill_random(1, 0.5)
    res = {v: [] for v in variants}
    lives = {}
    for rnd in range(a.rounds):
        for v in variants:
            lm.tune(*v, kernel=kernel)
            life.step(2)  # warm
            life.sync()
            life.set_timing(True)
            life.step(a.gens)
            ms, n, b = life.kernel_stats()
            life.set_timing(False)
            res[v].append((ms, b))
            lives[v] = life.live_count()
    for v in variants:
        mss = [m for m, _ in res[v]]
        b = res[v][0][1]
        med = statistics.median(mss)
        print(json.dumps({"kernel": kernel, "rows": v[0], "depth": v[1], "median_ms": round(med, 4),
                          "min_ms": round(min(mss), 4), "GBps_median": round(b / med / 1e6, 1),
                          "GBps_best": round(b / min(mss) / 1e6, 1), "live": lives[v]}), flush=True)
    life.close()
