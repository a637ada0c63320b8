"""Host-only planning arithmetic of the runtime (csrc/life_plan.cpp), checked
on the CPU: a small C++ harness is linked against life_plan.cpp alone with
g++ (no HIP) and prints the plans.

* life::gather_plan -- the rank-mode fan-in of life_collect
  (6-cartesian/life_cart.c:281-305, 5-gather/life_mpi.c:177-179): which
  rank's block arrives in which staging slot and where it lands in the
  frame.  For world 1..8 and every partition shape, every rank appears once,
  the two receive slots alternate and hold the largest block, and placing the
  pieces (OR-ing the shared LIFEBITS bytes) rebuilds the frame exactly.
* life::flow_chunk_passes -- the dataflow launch's 32-bit queue head never
  wraps: passes x tiles + resident workgroups stays within 2^31.
"""
import os
import subprocess

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "mpi-and-open-mp_amd", "csrc")

HARNESS = r"""
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include "life_host.h"
int main(int argc, char **argv) {
    if (!strcmp(argv[1], "chunk")) {
        printf("%lld\n", (long long)life::flow_chunk_passes(atoll(argv[2]), atoll(argv[3]), atoll(argv[4])));
        return 0;
    }
    const long long nx = atoll(argv[2]), ny = atoll(argv[3]);
    const int d0 = atoi(argv[4]), d1 = atoi(argv[5]), kernel = atoi(argv[6]), fmt = atoi(argv[7]);
    life::GatherPiece p[64];
    int64_t slot = 0;
    const int n = life::gather_plan(nx, ny, d0, d1, kernel, fmt, p, 64, &slot);
    printf("%d %lld %lld\n", n, (long long)slot, (long long)life::gather_frame_row_bytes(nx, fmt));
    for (int k = 0; k < n; k++)
        printf("%d %d %lld %lld %lld %lld %d %d\n", p[k].rank, p[k].slot, (long long)p[k].bytes,
               (long long)p[k].row_bytes, (long long)p[k].rows, (long long)p[k].dst, p[k].shared_first,
               p[k].shared_last);
    return 0;
}
"""


@pytest.fixture(scope="module")
def plan_exe(tmp_path_factory):
    d = tmp_path_factory.mktemp("plan")
    (d / "h.cpp").write_text(HARNESS)
    exe = d / "h"
    subprocess.run(["g++", "-O1", "-std=c++17", "-Wall", f"-I{CSRC}", f"-I{os.path.join(ROOT, 'include')}",
                    str(d / "h.cpp"), os.path.join(CSRC, "life_plan.cpp"), "-o", str(exe)], check=True)
    return str(exe)


def run(exe, *args):
    return subprocess.run([exe, *map(str, args)], capture_output=True, text=True, check=True).stdout.split("\n")


def gather_plan(exe, nx, ny, d0, d1, kernel, fmt):
    lines = run(exe, "gather", nx, ny, d0, d1, kernel, fmt)
    n, slot, frb = map(int, lines[0].split())
    pieces = [tuple(map(int, ln.split())) for ln in lines[1:1 + n]]
    return n, slot, frb, pieces


SHAPES = [(64, 48), (1000, 37), (257, 131), (4096, 1024), (13, 9), (8192, 100)]


@pytest.mark.parametrize("fmt", [0, 1, 2], ids=["dense", "vtk", "bits"])
@pytest.mark.parametrize("world", [1, 2, 3, 4, 5, 6, 7, 8])
def test_gather_plan_rebuilds_frame(plan_exe, lm, world, fmt):
    for nx, ny in SHAPES:
        for policy in ("cart", "rows", "cols"):
            try:
                d0, d1 = lm.dims_choose(nx, ny, world, policy)
            except RuntimeError:
                continue  # a shape with empty blocks
            n, slot, frb, pieces = gather_plan(plan_exe, nx, ny, d0, d1, 1, fmt)
            assert n == world
            root = world - 1
            assert pieces[0][0] == root and pieces[0][1] == -1  # the root's own block first
            assert [p[0] for p in pieces[1:]] == list(range(world - 1))  # fan-in in rank order
            assert [p[1] for p in pieces[1:]] == [k % 2 for k in range(world - 1)]  # alternating slots
            assert slot == max(p[2] for p in pieces)
            # rebuild the frame from per-rank exports of a known grid
            rng = np.random.default_rng(nx * 131 + ny + world)
            grid = (rng.random((ny, nx)) < 0.5).astype(np.uint8)
            if fmt == 0:
                want = grid.reshape(-1)
            elif fmt == 1:
                want = np.stack([grid + ord("0"), np.full_like(grid, ord("\n"))], axis=2).reshape(-1)
            else:
                want = np.packbits(grid, axis=1, bitorder="little").reshape(-1)
            frame = np.full(ny * frb, 0xAA, dtype=np.uint8)
            for p in pieces:
                if p[6]:
                    frame[p[5] + np.arange(p[4]) * frb] = 0  # shared first bytes start at 0
            for rank, _slot, nbytes, rb, rows, dst, sf, sl in pieces:
                L = lm.layout_query(nx, ny, (d0, d1), rank, "bit")
                blk = grid[L.y0:L.y0 + L.h, L.x0:L.x0 + L.w]
                if fmt == 0:
                    exp = blk
                elif fmt == 1:
                    exp = np.stack([blk + ord("0"), np.full_like(blk, ord("\n"))], axis=2).reshape(L.h, -1)
                else:  # the bits kernel: block cells from bit x0 & 7 of the first byte
                    s = L.x0 & 7
                    pad = np.zeros((L.h, s + L.w), dtype=np.uint8)
                    pad[:, s:] = blk
                    exp = np.packbits(pad, axis=1, bitorder="little")
                assert exp.shape == (rows, rb) and nbytes == rows * rb
                for y in range(rows):
                    o = dst + y * frb
                    row = exp[y]
                    a, b = (1 if sf else 0), (rb - 1 if sl else rb)
                    frame[o + a:o + b] = row[a:b]
                    if sf:
                        frame[o] |= row[0]
                    if sl and (rb > 1 or not sf):
                        frame[o + rb - 1] |= row[rb - 1]
            np.testing.assert_array_equal(frame, want, err_msg=f"{nx}x{ny} dims {d0}x{d1} fmt {fmt}")


def test_gather_plan_rejects(plan_exe):
    assert run(plan_exe, "gather", 64, 64, 2, 2, 1, 3)[0].split()[0] == "-1"  # unknown format


@pytest.mark.parametrize("tiles,grid", [(1, 0), (6494, 768), (34 * 191, 768), (1 << 20, 1024), (3, 5),
                                        ((1 << 31) - 10, 768), ((1 << 31) + 1, 1)])
def test_flow_chunk_passes(plan_exe, tiles, grid):
    limit = 1 << 31
    n = int(run(plan_exe, "chunk", tiles, grid, 0)[0])
    if tiles + grid > limit:
        assert n == 0
        return
    assert n >= 1 and n * tiles + grid <= limit < (n + 1) * tiles + grid
    # a cap below the bound wins; a cap above it does not
    assert int(run(plan_exe, "chunk", tiles, grid, 3)[0]) == min(3, n)
    assert int(run(plan_exe, "chunk", tiles, grid, n + 5)[0]) == n
