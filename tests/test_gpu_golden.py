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
def test_pattern_every_frame(gpu, name, kernel, shards):
    steps, save, grid = gpu.load_cfg(os.path.join(GOLDEN, "cfg", name + ".cfg"))
    ny, nx = grid.shape
    if shards > 1 and (nx < 2 or ny < 2):
        pytest.skip("grid too small for 2x2")
    frames = G["patterns"][name]["frames"]
    with gpu.Life(nx, ny, shards=shards, kernel=kernel, transport=gpu.XPORT_LOCAL) as life:
        life.upload(grid)
        out = np.empty_like(grid)
        for i in range(steps):
            if i % save == 0:
                life.gather(out)
                assert md5(gpu.vtk_bytes(out)) == frames[str(i)][0], f"{name} frame {i}"
            life.step(1)


@pytest.mark.parametrize("small", [False, True], ids=["stream", "lds"])
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
def test_random_vs_reference_life_step(gpu, kernel, case):
    nx, ny = case["nx"], case["ny"]
    with gpu.Life(nx, ny, kernel=kernel, small_grid=False) as life:
        life.fill_random(case["seed"], case["density"])
        assert md5(life.gather().tobytes()) == case["init_md5"]
        done = 0
        for gens in sorted(case["gens"], key=int):
            life.step(int(gens) - done)
            done = int(gens)
            g = life.gather()
            assert md5(g.tobytes()) == case["gens"][gens][0], f"after {gens}"
            assert life.live_count() == case["gens"][gens][1]


@pytest.mark.parametrize("args", [[], ["--gpus", "4"], ["--kernel", "byte"]])
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
