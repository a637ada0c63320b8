#!/usr/bin/env python3
"""Per-generation cost of a step call against its number of passes, per-launch
tiles vs the dataflow form (measurement tool).  65536^2 random grid, m = 10
generations per pass; each call timed by the wall clock between syncs (the
bench's clock) after a 5-generation warm call.

  LIFE_FLOW_MIN_PASSES=2 python3 scripts/pass_study.py OUT.jsonl
"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "mpi-and-open-mp_amd"))
import life_mi355x as lm  # noqa: E402


def main():
    out = open(sys.argv[1], "a")
    n = 65536
    for flow in (0, 1):
        for passes in (2, 3, 4, 8, 16):
            for rep in range(2):
                with lm.Life(n, n, kernel="bit", flow=flow) as life:
                    life.configure(lm.OPT_BLOCK_GENS, 10)
                    life.fill_random(1, 0.5)
                    life.step(5)
                    life.sync()
                    life.set_timing(True)
                    t = time.perf_counter()
                    life.step(10 * passes)
                    path = life.last_path()
                    life.sync()
                    dt = time.perf_counter() - t
                    ms, launches, _ = life.kernel_stats()
                    rec = {"flow": flow, "passes": passes, "rep": rep, "path": path, "ms_per_gen": dt * 1e3 / (10 * passes),
                           "kernel_ms_per_pass": ms, "launches": launches,
                           "Tcell_s": n * n * 10 * passes / dt / 1e12}
                    print(json.dumps(rec), flush=True)
                    out.write(json.dumps(rec) + "\n")


if __name__ == "__main__":
    main()
