"""The CPU oracle against the reference's own outputs (tests/golden/golden.json,
produced by oracle/make_golden.py from the reference programs compiled from
source).  Pins the checker before any GPU result is compared to it."""
import hashlib
import json
import os

import numpy as np
import pytest

from conftest import GOLDEN

with open(os.path.join(GOLDEN, "golden.json")) as _f:
    G = json.load(_f)


def md5(b: bytes) -> str:
    return hashlib.md5(b).hexdigest()


@pytest.mark.parametrize("name", sorted(G["patterns"]))
def test_oracle_every_frame_of_reference_patterns(oracle, lm, name):
    """Every VTK frame life2d wrote (md5 of the whole file) is reproduced by
    oracle.life_step + the VTK writer."""
    steps, save, grid = lm.load_cfg(os.path.join(GOLDEN, "cfg", name + ".cfg"))
    frames = G["patterns"][name]["frames"]
    g = grid
    for i in range(steps):
        if i % save == 0:
            h, live = frames[str(i)]
            assert md5(lm.vtk_bytes(g)) == h, f"{name} frame {i}"
            assert int(g.sum()) == live
        g = oracle.life_step(g)
    assert len(frames) == len(range(0, steps, save))


def test_numpy_restatement_agrees(oracle):
    for nx, ny in [(1, 1), (2, 3), (10, 10), (40, 20), (33, 65)]:
        g = oracle.fill_random(nx, ny, 5, 0.5)
        a = g
        for _ in range(6):
            a = oracle.np_life_step(a)
        np.testing.assert_array_equal(a, oracle.life_run(g, 6))


@pytest.mark.parametrize("case", [c for c in G["random"] if c["nx"] * c["ny"] <= 1 << 20],
                         ids=lambda c: f'{c["nx"]}x{c["ny"]}s{c["seed"]}')
def test_oracle_random_vs_reference_life_step(oracle, case):
    g = oracle.fill_random(case["nx"], case["ny"], case["seed"], case["density"])
    assert md5(g.tobytes()) == case["init_md5"]
    done = 0
    for gens in sorted(case["gens"], key=int):
        g = oracle.life_run(g, int(gens) - done, threads=4)
        done = int(gens)
        h, live = case["gens"][gens]
        assert md5(g.tobytes()) == h, f"after {gens} generations"
        assert int(g.sum()) == live


def test_p46gun_big_gen10000(oracle, lm):
    """configs[1]: the state after 10000 generations (549 live cells)."""
    steps, _, grid = lm.load_cfg(os.path.join(GOLDEN, "cfg", "p46gun_big.cfg"))
    assert steps == 10000
    rec = G["p46gun_big"]
    assert md5(lm.vtk_bytes(grid)) == rec["frame0_md5"] == rec["reference_committed_frame0_md5"]
    g = oracle.life_run(grid, 10000, threads=4)
    assert md5(lm.vtk_bytes(g)) == rec["gen10000_md5"]
    assert int(g.sum()) == rec["gen10000_live"] == 549


def test_mpi_variants_match_serial_reference():
    """Recorded when the fixtures were made: the reference's MPI programs
    (life_cart 2-D, life_mpi row strips) reproduce life2d frame by frame."""
    checks = G["mpi_crosscheck"]
    assert isinstance(checks, list) and checks
    for c in checks:
        assert c["identical_to_life2d"] == c["frames"], c


@pytest.mark.reference
def test_oracle_vs_linked_reference_life_step(oracle):
    """Direct cross-check against the reference's life_step linked from
    /root/reference (only where oracle/_ref was built)."""
    if oracle.ref_lib() is None:
        pytest.skip("oracle/_ref not built (reference not mounted)")
    for nx, ny in [(1, 1), (1, 9), (2, 2), (5, 3), (64, 64), (97, 31)]:
        g = oracle.fill_random(nx, ny, nx + ny, 0.45)
        np.testing.assert_array_equal(oracle.ref_life_run(g, 9), oracle.life_run(g, 9))


def test_checksum_definition(oracle):
    """oracle.checksum is the documented life_dev_checksum: one live cell at
    (x, y) contributes mix64(y*nx + x + 1); contributions add mod 2^64."""
    def mix(v):
        t = (v * 0x9E3779B97F4A7C15) % 2**64
        return t ^ (t >> 29)

    g = np.zeros((7, 11), np.uint8)
    assert oracle.checksum(g) == 0
    g[3, 5] = 1
    assert oracle.checksum(g) == mix(3 * 11 + 5 + 1)
    g[6, 10] = 1
    assert oracle.checksum(g) == (mix(3 * 11 + 5 + 1) + mix(6 * 11 + 10 + 1)) % 2**64
    big = oracle.fill_random(300, 200, 5, 0.5)
    ys, xs = np.nonzero(big)
    assert oracle.checksum(big) == sum(mix(int(y) * 300 + int(x) + 1) for y, x in zip(ys, xs)) % 2**64
    # block form (a shard's owned cells at global origin x0, y0) sums to the whole
    parts = sum(oracle.checksum(big[y0:y0 + 100, x0:x0 + 150], x0, y0, 300)
                for y0 in (0, 100) for x0 in (0, 150)) % 2**64
    assert parts == oracle.checksum(big)


def test_ref_mpirun_cfg_and_rate(oracle, lm, tmp_path):
    """oracle/ref_mpirun.py (bench.py's cpu_baseline "reference" leg): the .cfg
    it writes loads back to the same grid (the reference's format,
    life_cart.c:92-109), and the reference life_cart under mpiexec -n 4 yields
    a positive steady-state rate."""
    import ref_mpirun

    g = oracle.fill_random(96, 64, 7, 0.5)
    path = str(tmp_path / "r.cfg")
    ref_mpirun.write_cfg(path, 96, 64, ref_mpirun.cfg_body(g), 11, 12)
    steps, save, back = lm.load_cfg(path)
    assert (steps, save) == (11, 12)
    assert np.array_equal(back, g)
    if not ref_mpirun.available():
        pytest.skip("oracle/_ref/life_cart or mpiexec not built here")
    r = ref_mpirun.steady_rate(oracle.fill_random(256, 256, 3, 0.5), 4, target_s=0.5, probe_gens=10)
    assert r["kind"] == "reference" and r["cores"] == 4 and r["value"] > 0


def test_fill_random_window_matches_full_grid(oracle):
    """The windowed generator (the 65536^2 band test's initial band) is the
    full grid's cells, x taken modulo nx across the seam."""
    nx, ny = 300, 40
    g = oracle.fill_random(nx, ny, 7, 0.5)
    w = oracle.fill_random_window(nx, -50, 3, 120, 20, 7, 0.5)
    np.testing.assert_array_equal(w, np.roll(g, 50, axis=1)[3:23, :120])
    np.testing.assert_array_equal(oracle.fill_random_window(nx, 0, 0, nx, ny, 7, 0.5), g)
