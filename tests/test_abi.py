"""The C-ABI library: builds, loads without a GPU, exports every symbol the
header declares; the driver keeps the reference's CLI contract."""
import os
import re
import subprocess

import pytest

from conftest import ROOT

HEADER = os.path.join(ROOT, "include", "life_mi355x.h")
DRIVER = os.path.join(ROOT, "mpi-and-open-mp_amd", "driver", "life_mi355x")


def declared_functions():
    text = open(HEADER).read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return sorted(set(re.findall(r"\b(life_[a-z_]+)\s*\(", text)))


def test_header_lists_what_the_binding_knows(lm):
    assert declared_functions() == sorted(lm.ABI_SYMBOLS)


def test_library_exports_every_declared_symbol(lm):
    out = subprocess.run(["nm", "-D", "--defined-only", lm.LIB_PATH], capture_output=True, text=True,
                         check=True).stdout
    exported = set(re.findall(r"\bT (life_[a-z_]+)$", out, flags=re.M))
    missing = [f for f in declared_functions() if f not in exported]
    assert not missing, missing
    lib = lm._lib()
    for f in declared_functions():
        assert getattr(lib, f) is not None


def test_library_is_gfx950_only(lm, tmp_path):
    """The fat binary carries gfx950 code objects and nothing else."""
    fat = tmp_path / "fatbin"
    subprocess.run(["objcopy", "-O", "binary", "--only-section=.hip_fatbin", lm.LIB_PATH, str(fat)], check=True)
    ids = set(re.findall(rb"amdgcn-amd-amdhsa-[-a-z0-9]*?(gfx[0-9a-z]+)", fat.read_bytes()))
    assert ids == {b"gfx950"}, ids


def test_no_cpu_fallback_without_gpu(lm):
    """The device path fails loudly when no GPU is visible (no silent CPU path)."""
    from conftest import gpu_available

    if gpu_available():
        pytest.skip("a GPU is visible")
    with pytest.raises(lm.LifeError):
        lm.Life(16, 16)


def test_strerror(lm):
    lib = lm._lib()
    assert lib.life_strerror(0) == b"success"
    assert lib.life_strerror(-1) == b"invalid argument"


def test_driver_usage_contract():
    """life_cart.c:53-56: wrong argc -> usage on stdout, exit status 0."""
    assert os.path.exists(DRIVER), "driver not built"
    r = subprocess.run([DRIVER], capture_output=True, text=True)
    assert r.returncode == 0
    assert r.stdout == f"Usage: {DRIVER} input file.\n"


def test_driver_rejects_bad_config(tmp_path):
    bad = tmp_path / "bad.cfg"
    bad.write_text("10\n0\n5 5\n")  # save_steps == 0: SIGFPE in the reference
    r = subprocess.run([DRIVER, str(bad)], capture_output=True, text=True)
    assert r.returncode == 1 and "save_steps" in r.stderr
