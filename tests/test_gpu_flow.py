"""The dataflow form of the bit tiles (LIFE_OPT_FLOW): whole passes of a step
call as ONE persistent launch whose workgroups pull (pass, tile) items and
wait for the tiles their windows read (life_kernels.hip tflow_kernel).  The
hand-off between workgroups (agent-scope loads, write-through or fenced
stores, per-tile pass counters) is what can go wrong, so the bar is
bit-exact against the oracle (3-life/life2d.c:104-130 restated) on shapes
with full and partial tile rows / columns and a short last tile row, and
census-equal to the per-launch tiles at sizes where many passes overlap on
a loaded chip.
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

# nx (multiple of 64: x wraps inside the pairs), ny, generations, m
# (2048 x 8000: 24 tile rows, the rotation wraps several times per call;
# 4032 = 63 pairs: a second tile column owning one pair)
# (a call takes the dataflow form from 4 passes on)
# A last tile column owning o <= 30 pairs runs as banded items of 64 / G tile
# rows (G = 2^ceil(log2(o + 2)) lanes), the rows padded to whole groups:
# 4096 / 4032 / 128 / 64 (G = 4, 16 rows per item), 8192 (o = 4, G = 8),
# 16384 (o = 8, G = 16, 4 rows: the configs[3] N = 8 block's width), 32768
# wide in test_flow_fullsize_census (o = 16, G = 32).
CASES = [(2048, 1000, 87, 20), (1024, 3000, 64, 16), (4096, 1100, 43, 10), (1984, 700, 135, 32), (64, 900, 37, 8),
         (2112, 2000, 61, 12), (128, 2048, 85, 20), (2048, 8000, 81, 20), (4032, 600, 90, 21),
         (8192, 3000, 61, 12), (16384, 1500, 50, 12)]


@pytest.mark.parametrize("flow", [1, 2])
@pytest.mark.parametrize("nx,ny,gens,m", CASES)
def test_flow_parity(gpu, oracle, nx, ny, gens, m, flow):
    g0 = oracle.fill_random(nx, ny, seed=21, density=0.45)
    want = oracle.life_run(g0, gens)
    with gpu.Life(nx, ny, kernel="bit", small_grid=False) as life:
        life.configure(gpu.OPT_FLOW, flow)
        life.configure(gpu.OPT_BLOCK_GENS, m)
        life.upload(g0)
        life.set_timing(True)
        life.step(gens)
        assert life.last_path() == "flow"
        avg_ms, launches, _ = life.kernel_stats()
        assert launches >= gens // m  # the passes were timed as one launch each
        np.testing.assert_array_equal(life.gather(), want)
        assert life.live_count() == int(want.sum())


@pytest.mark.parametrize("flow", [1, 2])
@pytest.mark.parametrize("n,m", [(16384, 20), (32768, 10), (65536, 16)])
def test_flow_fullsize_census(gpu, n, m, flow):
    """Many overlapped passes on a loaded chip: the census (checksum + live
    count) equals the per-launch tiles' after the same generations."""
    gens = 7 * m + 3
    with gpu.Life(n, n, kernel="bit") as ref:
        ref.configure(gpu.OPT_FLOW, 0)  # the per-launch tiles
        ref.configure(gpu.OPT_BLOCK_GENS, m)
        ref.fill_random(5, 0.5)
        ref.step(gens)
        assert ref.last_path() == "tiles"
        want = (ref.checksum(), ref.live_count())
    with gpu.Life(n, n, kernel="bit") as life:
        life.configure(gpu.OPT_FLOW, flow)
        life.configure(gpu.OPT_BLOCK_GENS, m)
        life.fill_random(5, 0.5)
        life.step(gens)
        assert life.last_path() == "flow"
        assert (life.checksum(), life.live_count()) == want


def test_flow_back_to_back_and_chunked(gpu, oracle):
    """Consecutive dataflow calls on one device: odd then even
    pass counts (buffer parity flips between calls, 5 then 4 passes), a changed pass size
    (the scratch is reused or regrown), and a call split over several
    persistent launches (LIFE_OPT_FLOW_CHUNK: the 32-bit queue head's
    chunking, forced small) -- each stage bit-exact against the oracle."""
    nx, ny = 2048, 1000
    g = oracle.fill_random(nx, ny, seed=31, density=0.45)
    with gpu.Life(nx, ny, kernel="bit", small_grid=False, flow=1) as life:
        life.upload(g)
        for gens, m, chunk in [(107, 20, 0), (81, 20, 0), (50, 12, 0), (89, 12, 3), (100, 20, 1), (41, 10, 2)]:
            life.configure(gpu.OPT_BLOCK_GENS, m)
            life.configure(gpu.OPT_FLOW_CHUNK, chunk)
            life.set_timing(True)
            life.step(gens)
            assert life.last_path() == "flow"
            if chunk:
                _, launches, _ = life.kernel_stats()
                assert launches >= gens // m  # timed per pass, however the passes were chunked
            g = oracle.life_run(g, gens)
            np.testing.assert_array_equal(life.gather(), g, err_msg=f"{gens} generations, m={m}, chunk={chunk}")


def test_flow_needs_four_passes(gpu, oracle):
    """2-3 passes run as per-launch tiles (the dataflow form's start-up cost
    is not repaid, life_dev.hip kFlowMinPasses), 4 take the dataflow form."""
    nx, ny = 2048, 700
    g = oracle.fill_random(nx, ny, seed=37, density=0.5)
    with gpu.Life(nx, ny, kernel="bit", small_grid=False, flow=1) as life:
        life.upload(g)
        life.configure(gpu.OPT_BLOCK_GENS, 10)
        for gens, path in [(20, "tiles"), (39, "tiles"), (40, "flow"), (45, "flow")]:
            life.step(gens)
            assert life.last_path() == path, gens
            g = oracle.life_run(g, gens)
        np.testing.assert_array_equal(life.gather(), g)


def test_flow_default_automatic(gpu):
    """The default (LIFE_OPT_FLOW 3) takes the dataflow form when a pass is
    under 5 rounds of resident workgroups -- the per-launch tiles' tail then
    idles the chip (32768^2: 2.2 rounds, +8 %, profiles/r05/a) -- except 1 to
    1.5 rounds, and the per-launch tiles at 65536^2 (8.6 rounds, where they
    win by 3 %)."""
    with gpu.Life(2048, 1000, kernel="bit", small_grid=False) as life:
        life.fill_random(3, 0.5)
        life.step(100)
        assert life.last_path() == "flow"
    with gpu.Life(65536, 65536, kernel="bit") as life:
        life.fill_random(3, 0.5)
        life.step(48)
        assert life.last_path() == "tiles"
    # round 6: a pass of 1 to 1.5 rounds (configs[3]'s N = 8 block, 833 tiles)
    # runs per-launch tiles with the banded half-height tail (+12 %, r06d)
    with gpu.Life(16384, 32768, kernel="bit") as life:
        life.fill_random(3, 0.5)
        life.step(48)
        assert life.last_path() == "tiles"
    with gpu.Life(2048, 1000, kernel="bit", small_grid=False, flow=0) as life:
        life.fill_random(3, 0.5)
        life.step(100)
        assert life.last_path() == "tiles"


def test_flow_rejected_options(gpu):
    with gpu.Life(256, 256, kernel="bit") as life:
        with pytest.raises(RuntimeError):
            life.configure(gpu.OPT_FLOW, 4)
        with pytest.raises(RuntimeError):
            life.configure(gpu.OPT_FLOW_CHUNK, -1)
        with pytest.raises(RuntimeError):  # the byte dataflow form (value | 4) was removed
            life.configure(gpu.OPT_FLOW, 5)


def test_flow_is_bit_only(gpu):
    """The byte encoding always runs per-launch tiles (its dataflow form
    trailed them by 13 % at 65536^2 and was removed)."""
    with gpu.Life(2048, 1000, kernel="byte", small_grid=False, flow=1) as life:
        life.fill_random(3, 0.5)
        life.step(70)
        assert life.last_path() == "tiles"
