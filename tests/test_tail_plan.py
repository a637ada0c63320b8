"""The launch-tail planner (life::tail_plan, csrc/life_plan.cpp; CPU only).

launch_tstep re-tiles the bottom tile rows of a full-width bit launch as
3/4- and half-height tiles (banded in the last tile column like the full
tiles) so that the launch's last rounds are short items filling the slots
the full tiles leave (configs[3]'s N = 8
block, 833 tiles on 768 slots, runs ~1.5 tile-times per pass with half tiles
only).  Checked here with a g++ harness against a Python heap simulation of
the same list schedule:

* tail_makespan3 (grouped slots) == the heap simulation for every count;
* the plan's own makespan is the simulated makespan of its split, it covers
  the region's rows exactly once, never loses to no split or to half tiles
  only, and is within 2 % of the exhaustive optimum over (F, n34).
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
    if (!strcmp(argv[1], "span")) {  // ntx B F n34 n2 slots c
        printf("%.9f\n", life::tail_makespan3(atoll(argv[2]), atoll(argv[3]), atoll(argv[4]), atoll(argv[5]),
                                              atoll(argv[6]), atoll(argv[7]), atof(argv[8])));
        return 0;
    }
    if (!strcmp(argv[1], "best")) {  // exhaustive optimum over (F, n34): ntx B nty h T T34 T2 slots c
        const long long ntx = atoll(argv[2]), B = atoll(argv[3]), nty = atoll(argv[4]), h = atoll(argv[5]),
                        T = atoll(argv[6]), T34 = atoll(argv[7]), T2 = atoll(argv[8]), slots = atoll(argv[9]);
        const double c = atof(argv[10]);
        double best = life::tail_makespan3(ntx, B, nty, 0, 0, slots, c);
        for (long long f = nty - 1; f >= 0; --f) {
            const long long rest = h - f * T;
            for (long long n = 0; n <= (rest + T34 - 1) / T34; ++n) {
                if (n && (n - 1) * T34 >= rest) continue;
                const long long k = rest > n * T34 ? (rest - n * T34 + T2 - 1) / T2 : 0;
                const double t = life::tail_makespan3(ntx, B, f, n, k, slots, c);
                if (t < best) best = t;
            }
        }
        printf("%.9f\n", best);
        return 0;
    }
    long long v[9];
    for (int i = 0; i < 9; i++) v[i] = atoll(argv[2 + i]);
    const life::TailPlan p = life::tail_plan(v[0], v[1], v[2], v[3], v[4], v[5], v[6], v[7], v[8], atoi(argv[11]),
                                             atof(argv[12]));
    printf("%lld %lld %lld %.9f\n", (long long)p.F, (long long)p.n34, (long long)p.n2, p.makespan);
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


def heap_span(ntx, B, F, n34, n2, slots, c):
    free, end = [0.0] * slots, 0.0
    for d, n in ((1.0, row_items(ntx, B, F)), (c + (1 - c) * 0.75, row_items(ntx, B, n34)),
                 (c + (1 - c) * 0.5, row_items(ntx, B, n2))):
        for _ in range(n):
            t = heapq.heappop(free) + d
            end = max(end, t)
            heapq.heappush(free, t)
    return end


def geometry(W, m, R=24, NW=8):
    """tile_geom's columns / bands of a W-pair-wide shard and the three tile heights at m generations"""
    ntx = -(-W // 62)
    o = W - 62 * (ntx - 1)
    gsh = 2
    while (1 << gsh) < o + 2:
        gsh += 1
    B = 64 >> gsh if gsh <= 5 else 1
    return ntx, B, NW * R - 2 * m, NW * (R * 3 // 4) - 2 * m, NW * (R // 2) - 2 * m


@pytest.mark.parametrize("ntx,B,F,n34,n2,slots", [(5, 4, 7, 3, 2, 13), (17, 1, 30, 0, 4, 64), (9, 2, 0, 12, 11, 8),
                                                   (3, 16, 40, 9, 0, 3), (1, 1, 5, 5, 5, 1), (5, 4, 196, 0, 0, 768)])
@pytest.mark.parametrize("c", [0.0, 0.06, 0.2])
def test_grouped_schedule_is_the_list_schedule(exe, ntx, B, F, n34, n2, slots, c):
    got = float(run(exe, "span", ntx, B, F, n34, n2, slots, c)[0])
    assert got == pytest.approx(heap_span(ntx, B, F, n34, n2, slots, c), abs=1e-9)


SHAPES = [(1024, 65536), (512, 65536), (512, 32768), (256, 32768), (256, 8192), (300, 5000), (64, 4096), (200, 5000),
          (300, 2600), (1024, 16384), (700, 9000), (130, 40000)]


@pytest.mark.parametrize("W,h", SHAPES)
@pytest.mark.parametrize("m", [5, 10, 12])
def test_plan_covers_and_beats_the_alternatives(exe, W, h, m):
    slots, c = 768, 0.06
    ntx, B, T, T34, T2 = geometry(W, m)
    nty = -(-h // T)
    F, n34, n2, span = run(exe, "plan", ntx, B, 0, nty, h, T, T34, T2, slots, 3, c)
    F, n34, n2, span = int(F), int(n34), int(n2), float(span)
    assert 0 <= F <= nty
    if F < nty:  # the split covers rows [F T, h) exactly: no partial row beyond the region
        rest = h - F * T
        assert n34 * T34 + n2 * T2 >= rest
        assert (n2 == 0 and (n34 - 1) * T34 < rest) or (n2 > 0 and n34 * T34 < rest and (n2 - 1) * T2 < rest - n34 * T34)
    else:
        assert n34 == n2 == 0
    assert span == pytest.approx(heap_span(ntx, B, F, n34, n2, slots, c), abs=1e-9)
    whole = heap_span(ntx, B, nty, 0, 0, slots, c)
    half = float(run(exe, "plan", ntx, B, 0, nty, h, T, T34, T2, slots, 2, c)[3])
    assert span <= whole + 1e-9 and span <= half + 1e-9
    # exhaustive optimum of the same model over (F, n34) (grouped schedule, exact)
    if row_items(ntx, B, nty) > slots:  # (an underfilled launch is left whole)
        best = float(run(exe, "best", ntx, B, nty, h, T, T34, T2, slots, c)[0])
        assert span <= best * 1.02 + 1e-9, (span, best)


def test_known_shapes(exe):
    """configs[3]'s N = 8 block (16384 x 32768, 256 pairs) at 12 generations per
    pass: 1.53 tile-times with half tiles only, 1.295 with 3/4 + half tiles;
    65536^2 at 12: 9.0 (no split helps with half tiles) -> 8.765."""
    for W, h, m, two, three in [(256, 32768, 12, 1.53, 1.295), (1024, 65536, 12, 9.0, 8.765)]:
        ntx, B, T, T34, T2 = geometry(W, m)
        nty = -(-h // T)
        assert float(run(exe, "plan", ntx, B, 0, nty, h, T, T34, T2, 768, 2, 0.06)[3]) == pytest.approx(two)
        assert float(run(exe, "plan", ntx, B, 0, nty, h, T, T34, T2, 768, 3, 0.06)[3]) == pytest.approx(three)
