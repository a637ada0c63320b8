"""One-process-per-GPU (rank) mode on the single-GPU test box.

The RCCL multi-rank data path needs one GPU per rank (RCCL rejects two ranks
on one device), so the box cannot run world > 1.  What it can run is
everything around it: the torch-first process set-up bench.py uses under
torch.distributed.run, the gloo bootstrap of the RCCL unique id, a one-rank
RCCL communicator (ncclCommInitRank) and the census all-reduce over it, and
the rank-mode gather.  The halo plan and message matching of world > 1 are
covered by tests/test_gloo_plan.py (2-8 gloo ranks on the CPU).
"""
import json
import os
import subprocess
import sys

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.parametrize("kernel", ["bit", "byte"])
@pytest.mark.parametrize("nx,ny,gens", [(256, 130, 40), (257, 131, 7)])
def test_rank_mode_world1(gpu, oracle, kernel, nx, ny, gens):
    """life_dev_create_rank with a unique id: RCCL communicator of one rank;
    live_count goes through ncclAllReduce, gather through the rank path."""
    g0 = oracle.fill_random(nx, ny, seed=5, density=0.45)
    with gpu.Life.for_rank(nx, ny, 0, 1, gpu.unique_id(), 0, kernel=kernel) as life:
        life.upload(g0)
        life.step(gens)
        want = oracle.life_run(g0, gens)
        np.testing.assert_array_equal(life.gather(), want)
        assert life.live_count() == int(want.sum())


def test_bench_rank_mode_torchrun():
    """bench.py --rank-mode under torch.distributed.run (1 process): the exact
    bootstrap the driver's N > 1 scaling bench uses, and its JSON line."""
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "1",
           "--master-addr", "127.0.0.1", "--master-port", "29517", os.path.join(ROOT, "bench.py"),
           "--rank-mode", "--size", "4096", "--steps", "64", "--warmup", "32", "--no-cpu-baseline"]
    p = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=240)
    assert p.returncode == 0, p.stdout[-2000:] + p.stderr[-4000:]
    lines = [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, p.stdout
    out = json.loads(lines[0])
    assert out["n_gpus"] == 1 and out["value"] > 0
    # the line names its RCCL communicator: one rank (world 1, an id was broadcast), one device
    assert out["config"]["rccl_nranks"] == 1 and out["config"]["devices"] == 1, out["config"]
    # same grid, same generations as the single-process form
    import oracle as O

    g = O.fill_random(4096, 4096, 1, 0.5)
    assert out["config"]["live_cells_end"] == int(O.life_run(g, 96, 8).sum())
