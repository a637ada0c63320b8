#!/usr/bin/env python3
"""Is the driver-shaped call (generations 5..25 of the random soup) slower
than a cooled-soup call because of the soup or because of the GPU's clock
state?  Times the same 20-generation call (a fresh grid, 5 warm-up
generations) after different amounts of unrelated GPU work: none, and N
generations of another 65536^2 grid stepped just before.  Measurement tool
only."""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "mpi-and-open-mp_amd"))
import life_mi355x as lm  # noqa: E402

n = 65536
out = []
for heat in [0, 100, 400, 0, 400, 100]:
    if heat:
        with lm.Life(n, n, kernel="bit") as h:
            h.fill_random(99, 0.5)
            h.step(heat)
            h.sync()
    with lm.Life(n, n, kernel="bit") as life:
        life.fill_random(1, 0.5)
        life.step(5)
        life.sync()
        life.set_timing(True)
        t = time.perf_counter()
        life.step(20)
        life.sync()
        dt = time.perf_counter() - t
        ms, _, _ = life.kernel_stats()
    out.append({"heat_gens": heat, "wall_ms": round(dt * 1e3, 4), "kernel_ms": round(ms, 4),
                "gcell_s": round(n * n * 20 / dt / 1e9, 1)})
    print(json.dumps(out[-1]), flush=True)
