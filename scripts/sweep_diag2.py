"""Diagnostic: byte vs bit sweep at full size; prints mismatch locations."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "mpi-and-open-mp_amd")]
import life_mi355x as lm  # noqa: E402

for n, steps in ((32768, (16,)), (32768, (16, 16)), (65536, (16,))):
    out = {}
    for kernel in ("bit", "byte"):
        with lm.Life(n, n, kernel=kernel) as life:
            life.fill_random(1, 0.5)
            for s in steps:
                life.step(s)
            out[kernel] = life.gather()
            K = life.layout().generations_per_exchange
    bad = np.argwhere(out["bit"] != out["byte"])
    print(f"{n}^2 steps {steps} byte K {K}: {len(bad)} bad cells", flush=True)
    if len(bad):
        ys = np.unique(bad[:, 0]); xs = np.unique(bad[:, 1])
        print("  rows", ys[:30], "... n", len(ys), "last", ys[-5:])
        print("  cols", xs[:40], "... n", len(xs), "last", xs[-5:])
    del out
