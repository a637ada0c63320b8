import os, sys, hashlib
sys.path.insert(0, "mpi-and-open-mp_amd"); sys.path.insert(0, "oracle")
import numpy as np, life_mi355x as lm, oracle as O
want = O.fill_random(4096, 4096, 1, 0.5)
for trial in range(3):
    for kernel in ("bit", "byte"):
        for small in (False, True):
            with lm.Life(4096, 4096, kernel=kernel, small_grid=small) as life:
                life.fill_random(1, 0.5)
                g = life.gather()
                bad = np.argwhere(g != want)
                print(trial, kernel, small, "mismatches", len(bad), bad[:5].tolist() if len(bad) else "", flush=True)
