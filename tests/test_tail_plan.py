"""The launch-tail planner (life::tail_plan, csrc/life_plan.cpp; CPU only).

launch_tstep re-tiles the bottom tile rows of a full-width bit launch as
half-height tiles, banded in the last tile column like the full tiles (round
6), so that the launch's last round is short items filling the slots the
full tiles leave.  Checked here with a g++ harness against a
Python heap simulation of the same list schedule:

* tail_makespan2 (grouped slots) == the heap simulation for every count;
* the plan's own makespan is the simulated makespan of its split, it covers
  the region's rows exactly once, never loses to no split, and is the
  optimum over every split point; round 4's rule (mode 1) is never better.
"""
import heapq
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "mpi-and-open-mp_amd", "csrc")

HARNESS = r"""
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include "life_host.h"
int main(int argc, char **argv) {
    if (!strcmp(argv[1], "span")) {  // ntx B F n2 slots c
        printf("%.9f\n", life::tail_makespan2(atoll(argv[2]), atoll(argv[3]), atoll(argv[4]), atoll(argv[5]),
                                              atoll(argv[6]), atof(argv[7])));
        return 0;
    }
    long long v[8];
    for (int i = 0; i < 8; i++) v[i] = atoll(argv[2 + i]);
    const life::TailPlan p = life::tail_plan(v[0], v[1], v[2], v[3], v[4], v[5], v[6], v[7], atoi(argv[10]),
                                             atof(argv[11]));
    printf("%lld %lld %.9f\n", (long long)p.F, (long long)p.n2, p.makespan);
    return 0;
}
"""


@pytest.fixture(scope="module")
def exe(tmp_path_factory):
    d = tmp_path_factory.mktemp("tail")
    (d / "h.cpp").write_text(HARNESS)
    out = d / "h"
    subprocess.run(["g++", "-O2", "-std=c++17", "-Wall", f"-I{CSRC}", f"-I{os.path.join(ROOT, 'include')}",
                    str(d / "h.cpp"), os.path.join(CSRC, "life_plan.cpp"), "-o", str(out)], check=True)
    return str(out)


def run(exe, *args):
    return subprocess.run([exe, *map(str, args)], capture_output=True, text=True, check=True).stdout.split()


def row_items(ntx, B, rows):
    return 0 if rows <= 0 else ((ntx - 1) * rows + -(-rows // B) if B > 1 else ntx * rows)


def heap_span(ntx, B, F, n2, slots, c):
    free, end = [0.0] * slots, 0.0
    for d, n in ((1.0, row_items(ntx, B, F)), (c + (1 - c) * 0.5, row_items(ntx, B, n2))):
        for _ in range(n):
            t = heapq.heappop(free) + d
            end = max(end, t)
            heapq.heappush(free, t)
    return end


def geometry(W, m, R=24, NW=8):
    """tile_geom's columns / bands of a W-pair-wide shard and the full / half tile heights at m generations"""
    ntx = -(-W // 62)
    o = W - 62 * (ntx - 1)
    gsh = 2
    while (1 << gsh) < o + 2:
        gsh += 1
    B = 64 >> gsh if gsh <= 5 else 1
    return ntx, B, NW * R - 2 * m, NW * (R // 2) - 2 * m


@pytest.mark.parametrize("ntx,B,F,n2,slots", [(5, 4, 7, 2, 13), (17, 1, 30, 4, 64), (9, 2, 0, 11, 8), (3, 16, 40, 0, 3),
                                              (1, 1, 5, 5, 1), (5, 4, 196, 0, 768), (5, 4, 180, 36, 768)])
@pytest.mark.parametrize("c", [0.0, 0.06, 0.2])
def test_grouped_schedule_is_the_list_schedule(exe, ntx, B, F, n2, slots, c):
    got = float(run(exe, "span", ntx, B, F, n2, slots, c)[0])
    assert got == pytest.approx(heap_span(ntx, B, F, n2, slots, c), abs=1e-9)


SHAPES = [(1024, 65536), (512, 65536), (512, 32768), (256, 32768), (256, 8192), (300, 5000), (64, 4096), (200, 5000),
          (1024, 16384), (700, 9000), (130, 40000)]


@pytest.mark.parametrize("W,h", SHAPES)
@pytest.mark.parametrize("m", [5, 10, 12])
def test_plan_covers_and_is_optimal(exe, W, h, m):
    slots, c = 768, 0.06
    ntx, B, T, T2 = geometry(W, m)
    nty = -(-h // T)
    F, n2, span = run(exe, "plan", ntx, B, 0, nty, h, T, T2, slots, 2, c)
    F, n2, span = int(F), int(n2), float(span)
    assert 0 <= F <= nty
    if F < nty:  # the half tiles cover rows [F T, h) exactly: no half row beyond the region
        rest = h - F * T
        assert n2 * T2 >= rest > (n2 - 1) * T2
    else:
        assert n2 == 0
    assert span == pytest.approx(heap_span(ntx, B, F, n2, slots, c), abs=1e-9)
    whole = heap_span(ntx, B, nty, 0, slots, c)
    assert span <= whole + 1e-9
    if row_items(ntx, B, nty) > slots and row_items(ntx, B, nty) % slots:  # (an underfilled launch is left whole)
        best = min(float(run(exe, "span", ntx, B, f, -(-(h - f * T) // T2), slots, c)[0]) for f in range(nty))
        assert span <= min(best, whole) + 1e-9
        rule = float(run(exe, "plan", ntx, B, 0, nty, h, T, T2, slots, 1, c)[2])
        assert span <= rule + 1e-9


def test_known_shapes(exe):
    """configs[3]'s N = 8 block (16384 x 32768, 256 pairs, 833 tiles on 768
    slots) at 12 generations per pass: the full tiles fill one round and the
    bottom 36 tile rows run as banded half tiles (153 items): 1.53 tile-times
    instead of 2; 65536^2 at m = 10 (the driver's passes): 8.59 instead of
    9."""
    for W, h, m, want, F in [(256, 32768, 12, 1.53, 180), (1024, 65536, 10, 8.59, None)]:
        ntx, B, T, T2 = geometry(W, m)
        nty = -(-h // T)
        f, n2, span = run(exe, "plan", ntx, B, 0, nty, h, T, T2, 768, 2, 0.06)
        assert float(span) == pytest.approx(want, abs=0.011)
        if F is not None:
            assert int(f) == F
