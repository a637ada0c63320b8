#!/usr/bin/env python3
"""Repeat small one-generation / tile cases against the oracle many times in
ONE process after large allocations (measurement tool: hunts nondeterminism
such as reads of uninitialised memory that only show once freed buffers are
recycled)."""
import sys
import os
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "mpi-and-open-mp_amd"))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
import numpy as np  # noqa: E402
import life_mi355x as lm  # noqa: E402
import oracle as O  # noqa: E402

for n in (65536, 32768):  # leave big freed allocations behind, full of soup
    with lm.Life(n, n, kernel="byte") as big:
        big.fill_random(3, 0.5)
        big.step(40)
        big.sync()
bad = 0
cases = [(17, 3), (17, 5), (31, 33), (1, 7), (3, 5), (63, 65), (40, 300)]
for it in range(int(sys.argv[1]) if len(sys.argv) > 1 else 40):
    for (nx, ny) in cases:
        for kernel in ("bit", "byte"):
            seed = 1 + it % 3
            g0 = O.fill_random(nx, ny, seed, 0.5)
            with lm.Life(nx, ny, kernel=kernel, small_grid=False) as life:
                life.fill_random(seed, 0.5)
                life.step(1)
                got = life.gather()
                want = O.life_run(g0, 1)
                if not (got == want).all():
                    bad += 1
                    diff = np.argwhere(got != want)
                    print(f"MISMATCH it={it} {kernel} {nx}x{ny} seed={seed} path={life.last_path()} "
                          f"cells={len(diff)} first={diff[:6].tolist()}", flush=True)
    if it % 10 == 0:
        print(f"iteration {it} bad={bad}", flush=True)
print(f"done bad={bad}", flush=True)
