"""Diagnostic: sweep kernel vs the CPU oracle; prints where the first
mismatching cells are (rows, columns, words) for each case."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "mpi-and-open-mp_amd"), os.path.join(ROOT, "oracle")]
import life_mi355x as lm  # noqa: E402
import oracle as O  # noqa: E402

cases = [(kernel, nx, ny, steps) for kernel in ("byte", "bit")
         for nx, ny, steps in ((4096, 500, (16, 16)), (4096, 4096, (16,)), (4096, 4096, (32, 32)),
                               (32768, 256, (16,)), (8192, 8192, (16,)), (65536, 512, (16,)))]
for kernel, nx, ny, steps in cases:
    g0 = O.fill_random(nx, ny, nx + ny, 0.5)
    want = O.life_run(g0, sum(steps), 16)
    with lm.Life(nx, ny, kernel=kernel, small_grid=False) as life:
        life.upload(g0)
        for s in steps:
            life.step(s)
        got = life.gather()
        K = life.layout().generations_per_exchange
    bad = np.argwhere(got != want)
    print(f"{kernel} {nx}x{ny} steps {steps} K {K}: {len(bad)} bad cells", flush=True)
    if len(bad):
        ys = np.unique(bad[:, 0])
        xs = np.unique(bad[:, 1])
        print("  rows", ys[:20], "... n", len(ys))
        print("  cols", xs[:40], "... n", len(xs))
        print("  words", np.unique(xs // 32)[:40])
