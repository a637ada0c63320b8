import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (os.path.join(ROOT, "mpi-and-open-mp_amd"), os.path.join(ROOT, "oracle"), ROOT):
    if p not in sys.path:
        sys.path.insert(0, p)

GOLDEN = os.path.join(ROOT, "tests", "golden")
REFERENCE = "/root/reference"


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through liblife_mi355x.so)")
    config.addinivalue_line("markers", "reference: needs the reference mounted at /root/reference")


def gpu_available() -> bool:
    try:
        import ctypes

        hip = ctypes.CDLL("libamdhip64.so")
        n = ctypes.c_int(0)
        return hip.hipGetDeviceCount(ctypes.byref(n)) == 0 and n.value > 0
    except OSError:
        return False


@pytest.fixture(scope="session")
def oracle():
    import oracle as O

    O.lib()
    return O


@pytest.fixture(scope="session")
def lm():
    import life_mi355x

    life_mi355x._lib()
    # gathers into fresh buffers see poison, not np.empty's leftovers, where
    # the device copy did not land
    life_mi355x.GATHER_FILL = 0xA5
    return life_mi355x


@pytest.fixture(scope="session")
def gpu(lm):
    if not gpu_available():
        pytest.fail("no HIP device visible: -m gpu tests need an MI355X")
    return lm
