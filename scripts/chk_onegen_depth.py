import os, sys
sys.path.insert(0, "mpi-and-open-mp_amd"); sys.path.insert(0, "oracle")
import numpy as np
import life_mi355x as lm
import oracle as O
for kernel in ("bit", "byte"):
    for (nx, ny) in [(17, 3), (17, 16), (17, 17), (40, 300), (31, 33)]:
        g0 = O.fill_random(nx, ny, 1, 0.5)
        want = O.life_run(g0, 1)
        res = []
        for rows in (16, 32):
            for depth in (2, 8, 18):
                lm.tune(rows, depth, kernel=kernel)
                with lm.Life(nx, ny, kernel=kernel, small_grid=False) as life:
                    life.upload(g0)
                    life.step(1)
                    got = life.gather()
                    res.append((rows, depth, life.last_path(), bool((got == want).all())))
        print(kernel, nx, ny, res, flush=True)
