"""bench.py's multi-shard line proves itself:
`--gpus N` on this one-GPU box drives N logical shards with the LOCAL
transport -- the same layouts, halo plan, pack/unpack kernels and
ring / interior / exchange streams as the RCCL path -- and the JSON line must
carry parity_vs_1gpu (the same grid and generations as one shard on GPU 0,
census checksum + live count) and the per-phase timings."""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def run_bench(*args):
    # more shards than this box has GPUs: an explicit rehearsal
    extra = ["--rehearse-shards"] if "--gpus" in args else []
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--no-cpu-baseline", *extra, *args],
                       capture_output=True, text=True, timeout=300, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout
    return json.loads(lines[0])


@pytest.mark.parametrize("kernel", ["bit", "byte"])
def test_strong_scaling_4_shards_full_size(kernel):
    """configs[3] at N = 4: 65536^2 split 2x2 (MPI_Dims_create), LOCAL shards."""
    out = run_bench("--gpus", "4", "--scaling", "strong", "--kernel", kernel, "--steps", "40", "--warmup", "8")
    assert out["scaling"] == "strong"
    # a rehearsal says what it ran on: one GPU, four shards, no RCCL communicator (LOCAL copies)
    c = out["config"]
    assert out["n_gpus"] == 1 and c["shards"] == 4 and c["devices"] == 1 and c["rehearsal"] is True, c
    assert c["rccl_nranks"] == 0 and len(c["pci_bus_ids"]) == 1, c
    assert out["config"]["dims"] == [2, 2] and out["config"]["nx"] == out["config"]["ny"] == 65536
    p = out["parity_vs_1gpu"]
    assert p["ok"] is True and p["live"] > 0, p
    ph = out["phases"]
    assert ph["blocks"] > 0 and ph["block_ms"] > 0 and ph["interior_ms"] > 0 and ph["halo_ms"] > 0


@pytest.mark.parametrize("args", [("--gpus", "2", "--size", "8192", "--steps", "45", "--warmup", "4"),
                                  ("--gpus", "2", "--size", "8192", "--partition", "rows", "--steps", "45",
                                   "--warmup", "4"),
                                  ("--gpus", "3", "--size", "4096", "--partition", "cols", "--steps", "33",
                                   "--warmup", "0"),
                                  ("--gpus", "8", "--scaling", "strong", "--size", "8192", "--steps", "20",
                                   "--warmup", "5", "--parity-seconds", "0")])
def test_multi_shard_bench_parity(args):
    """Weak scaling 2-D (default) / row strips / column strips, and strong 4x2 blocks whose
    parity leg is a fresh 3K+1-generation run (--parity-seconds 0)."""
    out = run_bench(*args)
    p = out["parity_vs_1gpu"]
    assert p["ok"] is True, p
    if "--parity-seconds" in args:
        assert p["same_run"] is False and p["generations"] == 3 * out["config"]["generations_per_exchange"] + 1
    else:
        assert p["same_run"] is True
    assert out["phases"]["blocks"] > 0


def test_weak_scaling_default_is_cartesian_8():
    """configs[4] at N = 8: the weak line's
    default partition is life_cart's MPI_Dims_create {4, 2} -- a 262144 x
    131072 global grid of 65536^2 blocks, four halo peers per block -- and it
    proves itself against the same grid run as one shard."""
    out = run_bench("--gpus", "8", "--scaling", "weak", "--steps", "40", "--warmup", "8")
    assert out["scaling"] == "weak" and out["config"]["dims"] == [4, 2]
    assert (out["config"]["nx"], out["config"]["ny"]) == (262144, 131072)
    assert out["config"]["partition"] == "cart"
    assert out["parity_vs_1gpu"]["ok"] is True, out["parity_vs_1gpu"]
    c = out["call"]  # the host enqueue cost of the 8-shard pass is in the line
    assert c["passes"] == 4 and c["host_enqueue_ms"] >= c["pass_enqueue_max_ms"] > 0, c
    assert 0 < c["device_span_ms"] <= c["elapsed_ms"], c


def test_single_gpu_line_is_valu_roofline():
    """N = 1, temporal bit kernel: the roofline names the binding resource
    (VALU issue) and keeps the HBM figures beside it."""
    out = run_bench("--steps", "32", "--warmup", "16", "--size", "16384")
    r = out["roofline"]
    assert r["bound"] == "valu" and 0 < r["frac"] < 1 and r["unit"] == "Tlane-op/s"
    # achieved = the algorithmic ops of the owned cells (22 per 64-cell pair row and generation); the issued
    # ops (ghost rows, edge lanes) are larger
    updates = r["algorithmic_ops_per_launch"] * 64.0 / 22.0
    assert updates == pytest.approx(16384 * 16384 * r["generations_per_launch"], rel=1e-3)  # rounded to 3 digits
    assert r["issued"]["ops_per_launch"] > r["algorithmic_ops_per_launch"] and r["issued"]["frac"] > r["frac"]
    assert r["hbm"]["achieved"] > 0 and r["hbm"]["peak"] == 8000.0
    assert "parity_vs_1gpu" not in out and out["scaling"] == "weak"
    assert out["n_gpus"] == 1 and out["config"]["shards"] == 1 and out["config"]["rehearsal"] is False
    c = out["call"]  # one event pair around the call's launches: span <= the bench clock
    assert c["passes"] == 3 and 0 < c["device_span_ms"] <= c["elapsed_ms"] and c["host_enqueue_ms"] > 0, c
