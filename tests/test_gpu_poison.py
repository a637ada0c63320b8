"""The parity matrix again on POISONED buffers.

With LIFE_POISON=1 every buffer a shard allocates (both grid buffers with
their aprons, pitch padding and slack rows, the column staging, the sink)
starts as 0xA5 bytes instead of zeros, and every gather destination starts as
0xA5 (tests/conftest.py).  0xA5 is no dead cell in either encoding (byte:
not 0/1; bit: alternate cells alive), so a cell a kernel should have written
but did not, an apron read before its halo arrived, or a host copy that did
not land fails here on EVERY run -- a zeroed buffer would pass whenever the
expected grid is sparse (round 3's all-zero 17x3 result).

The test functions are the parity tests themselves (one-generation, tiles,
dataflow tiles, small grids, LOCAL shards, the deep-halo schedules -- whose
passes must never read an output buffer's stale apron rows beyond the
extension -- RCCL / LOCAL loopback, the reference's random grids), collected a second time in this module, where the
autouse fixture sets LIFE_POISON before each device is created.
"""
import pytest

from test_gpu_golden import test_random_vs_reference_life_step  # noqa: F401
from test_gpu_loopback import (test_loopback_initall_gather_and_frames,  # noqa: F401
                               test_loopback_no_overlap_and_toggle, test_loopback_parity)
from test_gpu_parity import (test_deep_halo, test_deep_halo_exchange_count,  # noqa: F401
                             test_gather_bits, test_multi_shard_local, test_single_shard,
                             test_small_grid_path, test_small_grid_windowed, test_temporal_multi_shard_local,
                             test_temporal_single_shard, test_wide_periodic_tile_columns)

pytestmark = pytest.mark.gpu


@pytest.fixture(autouse=True)
def poison(monkeypatch):
    monkeypatch.setenv("LIFE_POISON", "1")


def test_dead_grid_stays_dead_on_poison(gpu):
    """The round-3 shape (17x3, bit, one generation) from an all-dead grid:
    the step's output buffer starts as 0xA5, so only cells the kernel wrote
    can come back dead."""
    import numpy as np

    with gpu.Life(17, 3, kernel="bit", small_grid=False) as life:
        life.upload(np.zeros((3, 17), np.uint8))
        life.step(1)
        np.testing.assert_array_equal(life.gather(), np.zeros((3, 17), np.uint8))
