#!/usr/bin/env python3
"""Speed-up plot of a times.txt (the reference's plot_life.py, 6-cartesian/
plot_life.py:4-17: T1/TN per line, saved as life_accel.png), against the
number of GPUs of each run.

times.txt holds one elapsed-seconds line per run, as the reference's.  The
reference's files hold 1..28 ranks, line k = k ranks; scripts/run_life.sh runs
1, 2, 4, 8 GPUs and writes those counts to times.gpus beside times.txt.  The
counts come from --counts, else from that sidecar, else 1, 2, 3, ... (the
reference's convention).

  python scripts/plot_life.py [times.txt] [life_accel.png] [--counts 1,2,4,8]
"""
import os
import sys


def speedups(times):
    return [times[0] / t for t in times]


def gpu_counts(src, n, arg=None):
    if arg:
        counts = [int(x) for x in arg.split(",")]
    else:
        side = os.path.splitext(src)[0] + ".gpus"
        counts = [int(x) for x in open(side).read().split()] if os.path.exists(side) else list(range(1, n + 1))
    if len(counts) != n:
        raise SystemExit(f"{n} times but {len(counts)} GPU counts")
    return counts


def main(argv):
    counts_arg = None
    if "--counts" in argv:
        k = argv.index("--counts")
        counts_arg = argv[k + 1]
        argv = argv[:k] + argv[k + 2:]
    src = argv[1] if len(argv) > 1 else "times.txt"
    dst = argv[2] if len(argv) > 2 else "life_accel.png"
    times = [float(line) for line in open(src) if line.strip()]
    counts = gpu_counts(src, len(times), counts_arg)
    s = speedups(times)
    for n, t, v in zip(counts, times, s):
        print(f"{n} GPU(s): {t:.6f} s  speed-up {v:.2f}  efficiency {v * counts[0] / n:.2f}")
    import matplotlib

    matplotlib.use("Agg")
    import matplotlib.pyplot as plt

    plt.plot(counts, s, marker="o", label="T1 / TN")
    plt.plot(counts, [n / counts[0] for n in counts], linestyle="--", label="ideal")
    plt.xlabel("GPUs")
    plt.ylabel("T1 / TN")
    plt.xticks(counts)
    plt.legend()
    plt.grid(True)
    plt.savefig(dst)


if __name__ == "__main__":
    main(sys.argv)
