#!/usr/bin/env python3
"""Speed-up plot of a times.txt (the reference's plot_life.py, 6-cartesian/
plot_life.py:4-17: T1/TN per line, saved as life_accel.png).  Lines are the
elapsed seconds of runs on 1, 2, 4, ... GPUs (scripts/run_life.sh); the
reference's files hold 1..28 ranks, one per line, and plot the same way.

  python scripts/plot_life.py [times.txt] [life_accel.png]
"""
import sys


def speedups(times):
    return [times[0] / t for t in times]


def main():
    src = sys.argv[1] if len(sys.argv) > 1 else "times.txt"
    dst = sys.argv[2] if len(sys.argv) > 2 else "life_accel.png"
    times = [float(line) for line in open(src) if line.strip()]
    s = speedups(times)
    for i, v in enumerate(s):
        print(f"run {i + 1}: {times[i]:.6f} s  speed-up {v:.2f}")
    import matplotlib

    matplotlib.use("Agg")
    import matplotlib.pyplot as plt

    plt.plot(range(1, len(s) + 1), s, marker="o")
    plt.xlabel("run (1, 2, 4, ... GPUs)")
    plt.ylabel("T1 / TN")
    plt.grid(True)
    plt.savefig(dst)


if __name__ == "__main__":
    main()
