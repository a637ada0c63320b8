"""GPU path against the reference's own frames (tests/golden/golden.json):
every VTK frame of the reference patterns, p46gun_big generation 10000
(configs[1]), random grids stepped by the reference life_step, and the C
driver's files byte for byte (configs[0]: glider, 100 frames)."""
import hashlib
import json
import os
import subprocess

import numpy as np
import pytest

from conftest import GOLDEN, ROOT

pytestmark = pytest.mark.gpu

with open(os.path.join(GOLDEN, "golden.json")) as _f:
    G = json.load(_f)
DRIVER = os.path.join(ROOT, "mpi-and-open-mp_amd", "driver", "life_mi355x")


def md5(b: bytes) -> str:
    return hashlib.md5(b).hexdigest()


@pytest.mark.parametrize("shards", [1, 4])
@pytest.mark.parametrize("kernel", ["byte", "bit"])
@pytest.mark.parametrize("name", sorted(G["patterns"]))
def test_pattern_every_frame(gpu, oracle, name, kernel, shards):
    """Every frame the reference writes: the oracle's grid is pinned to the
    reference frame's md5, the GPU grid compared with it cell by cell."""
    steps, save, grid = gpu.load_cfg(os.path.join(GOLDEN, "cfg", name + ".cfg"))
    ny, nx = grid.shape
    if shards > 1 and (nx < 2 or ny < 2):
        pytest.skip("grid too small for 2x2")
    frames = G["patterns"][name]["frames"]
    want = grid.copy()
    with gpu.Life(nx, ny, shards=shards, kernel=kernel, transport=gpu.XPORT_LOCAL) as life:
        life.upload(grid)
        for i in range(steps):
            if i % save == 0:
                assert md5(gpu.vtk_bytes(want)) == frames[str(i)][0], f"oracle {name} frame {i}"
                out = np.full_like(grid, 0xA5)
                np.testing.assert_array_equal(life.gather(out), want, err_msg=f"{name} frame {i}")
            life.step(1)
            want = oracle.life_step(want)


@pytest.mark.parametrize("small", [False, "lds", True, "vgpr1"], ids=["stream", "lds", "vgpr", "vgpr1"])
@pytest.mark.parametrize("kernel", ["byte", "bit"])
def test_p46gun_big_gen10000(gpu, kernel, small):
    """configs[1] at full length: md5 28998c4b... (549 live) after 10000 generations."""
    _, _, grid = gpu.load_cfg(os.path.join(GOLDEN, "cfg", "p46gun_big.cfg"))
    with gpu.Life(500, 500, kernel=kernel, small_grid=small) as life:
        life.upload(grid)
        life.step(10000)
        g = life.gather()
        assert md5(gpu.vtk_bytes(g)) == G["p46gun_big"]["gen10000_md5"]
        assert life.live_count() == 549


@pytest.mark.parametrize("kernel", ["byte", "bit"])
@pytest.mark.parametrize("case", G["random"], ids=lambda c: f'{c["nx"]}x{c["ny"]}s{c["seed"]}')
def test_random_vs_reference_life_step(gpu, oracle, kernel, case):
    """Random grids stepped by the reference's own life_step.  The expected
    grid is the oracle's, pinned to the reference's md5 first, then compared
    cell by cell, so a mismatch prints the differing cells (an
    md5-only assert left the all-zero 17x3 result unexplained)."""
    nx, ny = case["nx"], case["ny"]
    want = oracle.fill_random(nx, ny, case["seed"], case["density"])
    assert md5(want.tobytes()) == case["init_md5"]
    with gpu.Life(nx, ny, kernel=kernel, small_grid=False) as life:
        life.fill_random(case["seed"], case["density"])
        np.testing.assert_array_equal(life.gather(), want, err_msg="initial grid")
        done = 0
        for gens in sorted(case["gens"], key=int):
            want = oracle.life_run(want, int(gens) - done)
            assert md5(want.tobytes()) == case["gens"][gens][0], f"oracle after {gens}"
            life.step(int(gens) - done)
            done = int(gens)
            np.testing.assert_array_equal(life.gather(), want, err_msg=f"after {gens} generations")
            assert life.live_count() == case["gens"][gens][1]


@pytest.mark.parametrize("args", [[], ["--gpus", "4"], ["--kernel", "byte"], ["--gpus", "4", "--partition", "rows"],
                                  ["--gpus", "2", "--partition", "cols", "--kernel", "byte"]])
def test_driver_glider_frames(gpu, tmp_path, args):
    """configs[0]: `prog glider_10x10.cfg` writes vtk/life_%06d.vtk files
    byte-identical to the reference's and prints one "%f\\n" line."""
    r = subprocess.run([DRIVER, os.path.join(GOLDEN, "cfg", "glider_10x10.cfg")] + args, cwd=tmp_path,
                       capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr
    lines = r.stdout.splitlines()
    assert len(lines) == 1 and float(lines[0]) >= 0.0
    frames = G["patterns"]["glider_10x10"]["frames"]
    files = sorted(os.listdir(tmp_path / "vtk"))
    assert files == [f"life_{i:06d}.vtk" for i in range(100)]
    for i in range(100):
        assert md5((tmp_path / "vtk" / f"life_{i:06d}.vtk").read_bytes()) == frames[str(i)][0], i


def test_driver_p46gun_big(gpu, tmp_path):
    r = subprocess.run([DRIVER, os.path.join(GOLDEN, "cfg", "p46gun_big.cfg"), "--steps", "10001",
                        "--save-steps", "10000"], cwd=tmp_path, capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr
    assert md5((tmp_path / "vtk" / "life_000000.vtk").read_bytes()) == G["p46gun_big"]["frame0_md5"]
    assert md5((tmp_path / "vtk" / "life_010000.vtk").read_bytes()) == G["p46gun_big"]["gen10000_md5"]


def test_driver_bits_frames_and_resume(gpu, tmp_path):
    """--format bits writes packed frames equal to the reference's frames;
    --resume from generation 40 continues the reference's frame sequence:
    generations and frame numbers are absolute (--steps 100 ends where the
    uninterrupted run ends, the first resumed frame is life_000040)."""
    frames = G["patterns"]["glider_10x10"]["frames"]
    r = subprocess.run([DRIVER, os.path.join(GOLDEN, "cfg", "glider_10x10.cfg"), "--format", "bits"], cwd=tmp_path,
                       capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr
    for i in (0, 1, 39, 40, 99):
        gen, g = gpu.load_bits(str(tmp_path / "vtk" / f"life_{i:06d}.bits"))
        assert gen == i and md5(gpu.vtk_bytes(g)) == frames[str(i)][0], i
    run2 = tmp_path / "resumed"
    run2.mkdir()
    r = subprocess.run([DRIVER, "--resume", str(tmp_path / "vtk" / "life_000040.bits"), "--steps", "100",
                        "--save-steps", "10"], cwd=run2, capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr
    assert sorted(os.listdir(run2 / "vtk")) == [f"life_{i:06d}.vtk" for i in range(40, 100, 10)]
    for i in range(40, 100, 10):
        assert md5((run2 / "vtk" / f"life_{i:06d}.vtk").read_bytes()) == frames[str(i)][0], i


LAUNCH_VARS = ("RANK", "WORLD_SIZE", "LOCAL_RANK", "PMI_RANK", "PMI_SIZE", "OMPI_COMM_WORLD_RANK",
               "OMPI_COMM_WORLD_SIZE", "MASTER_ADDR", "MASTER_PORT")


@pytest.mark.parametrize("launch", [{"RANK": "0", "WORLD_SIZE": "1", "LOCAL_RANK": "0"},
                                    {"PMI_RANK": "0", "PMI_SIZE": "1"},
                                    {"OMPI_COMM_WORLD_RANK": "0", "OMPI_COMM_WORLD_SIZE": "1"}, "--rank-mode"],
                         ids=["torchrun", "mpich", "openmpi", "flag"])
def test_driver_rank_mode_glider(gpu, tmp_path, launch):
    """Under a launcher the driver runs one-process-per-GPU (life_dev_create_rank,
    an RCCL communicator, the root rank writes the frames): at world 1 the
    frames are the reference's, byte for byte."""
    env = {k: v for k, v in os.environ.items() if k not in LAUNCH_VARS}
    args = [DRIVER, os.path.join(GOLDEN, "cfg", "glider_10x10.cfg")]
    if isinstance(launch, dict):
        env.update(launch)
    else:
        args.append(launch)
    r = subprocess.run(args, cwd=tmp_path, env=env, capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr
    assert len(r.stdout.splitlines()) == 1
    frames = G["patterns"]["glider_10x10"]["frames"]
    for i in range(100):
        assert md5((tmp_path / "vtk" / f"life_{i:06d}.vtk").read_bytes()) == frames[str(i)][0], i


def test_driver_refuses_gpus_under_launcher(gpu, tmp_path):
    env = dict(os.environ, RANK="0", WORLD_SIZE="1")
    r = subprocess.run([DRIVER, os.path.join(GOLDEN, "cfg", "glider_10x10.cfg"), "--gpus", "2"], cwd=tmp_path,
                       env=env, capture_output=True, text=True, timeout=60)
    assert r.returncode == 1 and "under a launcher" in r.stderr


def test_driver_random_density_checked(gpu, tmp_path):
    r = subprocess.run([DRIVER, "--random", "1,-0.5", "--nx", "64", "--ny", "64", "--steps", "2"], cwd=tmp_path,
                       capture_output=True, text=True, timeout=60)
    assert r.returncode == 1 and "density" in r.stderr


@pytest.mark.parametrize("kernel", ["byte", "bit"])
@pytest.mark.parametrize("nx,ny,shards", [(10, 10, 1), (37, 11, 1), (257, 131, 4), (1024, 300, 8), (5, 3, 1)])
def test_gather_vtk_equals_host_format(gpu, oracle, kernel, nx, ny, shards):
    """Device-formatted VTK text (life_dev_gather_vtk) == life_save_vtk of the
    gathered cells, for widths that are and are not multiples of 8."""
    g0 = oracle.fill_random(nx, ny, seed=nx * ny, density=0.5)
    with gpu.Life(nx, ny, shards=shards, kernel=kernel, transport=gpu.XPORT_LOCAL) as life:
        life.upload(g0)
        life.step(3)
        assert life.gather_vtk() == gpu.vtk_bytes(life.gather())


def test_driver_large_cfg_parallel_parse(gpu, tmp_path):
    """A multi-MB .cfg goes through the driver's mapped, multi-threaded parser
    (line-aligned chunks): frame 0 == the numpy loader's grid, with negative
    and out-of-range coordinates wrapped; one token per line (pairs split
    across chunk boundaries) takes the sequential pairing path; a malformed
    token is an error (the reference's fscanf loop would spin forever)."""
    rng = np.random.default_rng(3)
    n = 1536
    ys, xs = np.nonzero(rng.random((n, n)) < 0.5)
    xs = xs + n * rng.integers(-2, 3, xs.size)  # periodic wrap on load (life_cart.c:106-109)
    head = f"2\n1\n{n} {n}\n"
    for name, body in (("lines", "".join(f"{x} {y}\n" for x, y in zip(xs, ys))),
                       ("tokens", "".join(f"{x}\n{y}\n" for x, y in zip(xs, ys)))):
        p = tmp_path / f"{name}.cfg"
        p.write_text(head + body)
        assert p.stat().st_size > 8 << 20  # several parser threads
        run = tmp_path / name
        run.mkdir()
        r = subprocess.run([DRIVER, str(p), "--format", "bits", "--steps", "1"], cwd=run, capture_output=True,
                           text=True, timeout=120)
        assert r.returncode == 0, r.stderr
        want = gpu.load_cfg(str(p))[2]
        _, got = gpu.load_bits(str(run / "vtk" / "life_000000.bits"))
        np.testing.assert_array_equal(got, want)
    bad = tmp_path / "bad.cfg"
    bad.write_text(head + "1 2\n3 x4\n")
    r = subprocess.run([DRIVER, str(bad)], cwd=tmp_path, capture_output=True, text=True, timeout=60)
    assert r.returncode == 1 and "cannot read config" in r.stderr


@pytest.mark.parametrize("kernel", ["byte", "bit"])
def test_gather_vtk_8192_four_shards(gpu, oracle, kernel):
    """The device VTK formatter at scale: 8192^2 over 2x2 shards (life_cart.c's
    gather-then-save path, :159-187) == the host formatting of the gathered
    grid, byte for byte (134 MB of cell text)."""
    n = 8192
    with gpu.Life(n, n, shards=4, kernel=kernel, transport=gpu.XPORT_LOCAL) as life:
        life.fill_random(77, 0.5)
        life.step(37)
        assert life.gather_vtk() == gpu.vtk_bytes(life.gather())
