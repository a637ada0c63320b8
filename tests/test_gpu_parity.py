"""GPU parity: the HIP path (through the C ABI) against the CPU oracle.

Bit-exact on every cell.  The oracle restates 3-life/life2d.c:104-130 and is
itself pinned to the reference (tests/test_oracle.py).
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

SIZES = [(1, 1), (1, 5), (5, 1), (2, 3), (3, 2), (16, 16), (17, 3), (31, 33), (63, 64), (64, 63),
         (65, 65), (127, 5), (128, 128), (129, 130), (200, 1), (1000, 37), (257, 300)]


@pytest.mark.parametrize("kernel", ["byte", "bit"])
@pytest.mark.parametrize("nx,ny", SIZES)
def test_single_shard(gpu, oracle, kernel, nx, ny):
    g0 = oracle.fill_random(nx, ny, seed=nx * 1000 + ny, density=0.4)
    with gpu.Life(nx, ny, shards=1, kernel=kernel) as life:
        life.upload(g0)
        np.testing.assert_array_equal(life.gather(), g0)
        life.step(1)
        np.testing.assert_array_equal(life.gather(), oracle.life_run(g0, 1))
        life.step(6)
        want = oracle.life_run(g0, 7)
        np.testing.assert_array_equal(life.gather(), want)
        assert life.live_count() == int(want.sum())


@pytest.mark.parametrize("kernel", ["byte", "bit"])
@pytest.mark.parametrize("nx,ny,seed", [(1000, 37, 1), (4096, 64, 2), (333, 777, 3)])
def test_fill_random_matches_oracle(gpu, oracle, kernel, nx, ny, seed):
    with gpu.Life(nx, ny, kernel=kernel) as life:
        life.fill_random(seed, 0.5)
        np.testing.assert_array_equal(life.gather(), oracle.fill_random(nx, ny, seed, 0.5))


@pytest.mark.parametrize("kernel", ["byte", "bit"])
@pytest.mark.parametrize("shards,dims,nx,ny", [
    (2, (0, 0), 100, 40), (4, (0, 0), 65, 33), (8, (0, 0), 300, 130), (6, (0, 0), 47, 29),
    (4, (1, 4), 70, 50), (4, (4, 1), 70, 50), (3, (3, 1), 5, 9), (2, (1, 2), 3, 2),
    (8, (4, 2), 4, 2), (4, (2, 2), 260, 260),
])
def test_multi_shard_local(gpu, oracle, kernel, shards, dims, nx, ny):
    """P logical shards on one GPU, halo through the LOCAL transport: the same
    plan and pack/unpack kernels the RCCL transport runs."""
    g0 = oracle.fill_random(nx, ny, seed=shards * 7 + nx, density=0.45)
    with gpu.Life(nx, ny, shards=shards, kernel=kernel, dims=dims, transport=gpu.XPORT_LOCAL) as life:
        life.upload(g0)
        np.testing.assert_array_equal(life.gather(), g0)
        done = 0
        for total in (1, 4, 10):
            life.step(total - done)
            done = total
            want = oracle.life_run(g0, total)
            np.testing.assert_array_equal(life.gather(), want, err_msg=f"generation {total}")
        assert life.live_count() == int(want.sum())


def test_byte_equals_bit_long(gpu, oracle):
    nx, ny, gens = 1024, 768, 200
    g0 = oracle.fill_random(nx, ny, seed=11, density=0.5)
    out = {}
    for k in ("byte", "bit"):
        with gpu.Life(nx, ny, kernel=k) as life:
            life.upload(g0)
            life.step(gens)
            out[k] = life.gather()
    np.testing.assert_array_equal(out["byte"], out["bit"])
    np.testing.assert_array_equal(out["bit"], oracle.life_run(g0, gens, threads=4))


def test_timing_stats(gpu):
    with gpu.Life(4096, 4096, kernel="bit") as life:
        life.fill_random(1)
        life.set_timing(True)
        life.step(5)
        ms, n, b = life.kernel_stats()
        assert n == 5 and ms > 0 and b == pytest.approx(4096 * 4096 * 0.25)
