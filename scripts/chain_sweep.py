"""Chained vs independent temporal tiles at 65536^2 (one process): kernel time
per 32-generation launch from the library's HIP-event timers, for chain off,
chain on with the default segment sizing (resident workgroups per CU x CUs) and explicit
workgroups per launch.  One JSON line per (kernel, mode, round)."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "mpi-and-open-mp_amd"))
import life_mi355x as lm  # noqa: E402

N = int(sys.argv[1]) if len(sys.argv) > 1 else 65536
modes = [("tiles", False), ("chain", True), ("chain700", 700), ("chain1536", 1536), ("chain2304", 2304)]
for kernel in ("bit", "byte"):
    with lm.Life(N, N, kernel=kernel, small_grid=False) as life:
        for rnd in range(2):
            for name, ch in modes:
                # same state sequence for every mode (the grid cools as it runs,
                # and a cooler grid runs faster: no order effects)
                life.configure(lm.OPT_CHAIN, int(ch) if ch is not True else 1)
                life.fill_random(1, 0.5)
                life.step(64)
                life.sync()
                life.set_timing(True)
                life.step(128)
                life.sync()
                ms, n, _ = life.kernel_stats()
                upd, _ = life.kernel_work()
                life.set_timing(False)
                print(json.dumps({"kernel": kernel, "mode": name, "round": rnd, "ms_per_launch": round(ms, 4),
                                  "launches": n, "tcells": round(upd / (ms * 1e-3) / 1e12, 2),
                                  "checksum": life.checksum()}), flush=True)
