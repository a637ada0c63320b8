#!/usr/bin/env python3
"""Rate of step(1) calls -- one generation per life_dev_step, the way a caller
that steps and inspects every generation drives the library (measurement
tool): 65536^2 random 50 %, per encoding, kernel time per call from HIP
events and the algorithmic HBM rate (one read + one write of the encoding)
against the live copy ceiling.  One JSON line per encoding."""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "mpi-and-open-mp_amd"))
import life_mi355x as lm  # noqa: E402

p = argparse.ArgumentParser()
p.add_argument("--size", type=int, default=65536)
p.add_argument("--calls", type=int, default=30)
p.add_argument("--kernels", default="byte,bit")
a = p.parse_args()
copy = lm.measure_copy(0, 2 << 30, 5)
for kernel in a.kernels.split(","):
    with lm.Life(a.size, a.size, kernel=kernel) as life:
        life.fill_random(1, 0.5)
        for _ in range(5):
            life.step(1)
        life.sync()
        life.set_timing(True)
        t0 = time.perf_counter()
        for _ in range(a.calls):
            life.step(1)
        life.sync()
        dt = time.perf_counter() - t0
        ms, launches, bpl = life.kernel_stats()
        cells = float(a.size) ** 2
        alg = cells * (0.25 if kernel == "bit" else 2.0)
        print(json.dumps({"kernel": kernel, "path": life.last_path(),
                          "layout_K": life.layout().generations_per_exchange,
                          "Gcell_per_s": round(cells * a.calls / dt / 1e9, 1), "kernel_ms": round(ms, 4),
                          "alg_GBps": round(alg / (ms * 1e-3) / 1e9, 1), "copy_ceiling_GBps": round(copy, 1),
                          "frac_of_copy_ceiling": round(alg / (ms * 1e-3) / 1e9 / copy, 4)}), flush=True)
