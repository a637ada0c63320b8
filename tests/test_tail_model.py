"""The launch-tail model behind LIFE_TAIL_SPLIT 2 (CPU only).

launch_tstep (mpi-and-open-mp_amd/csrc/life_kernels.hip, tail_makespan)
picks how many bottom tile rows of a pass run as half-height tiles with a
closed form of a list schedule: full tiles dealt round-robin over the
resident slots, then half tiles (half the duration) into the earliest free
slots.  scripts/tail_model.py restates that closed form (closed_form) next to
a heap simulation of the same schedule (makespan); they must agree for every
count, or the split the kernel picks is not the one the model argues for.
"""
import importlib.util
import os

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
spec = importlib.util.spec_from_file_location("tail_model", os.path.join(ROOT, "scripts", "tail_model.py"))
tm = importlib.util.module_from_spec(spec)
spec.loader.exec_module(tm)


@pytest.mark.parametrize("slots", [1, 3, 8, 13, 64])
def test_closed_form_is_the_list_schedule(slots):
    for full in range(0, 4 * slots + 3):
        for half in range(0, 5 * slots + 3):
            if full == 0 and half == 0:
                continue
            assert tm.closed_form(full, half, slots) == pytest.approx(tm.makespan(full, half, slots)), (full, half)


def test_model_split_never_worse_than_no_split():
    """At the measured shapes (768 slots) the chosen split is never slower in
    the model than no split and never better than the best simulated split."""
    for W, h in [(1024, 65536), (512, 65536), (512, 32768), (256, 32768), (300, 5000)]:
        for m in (8, 10, 12):
            T, T2, ntx, B = tm.geom(W, m)
            nty = -(-h // T)
            n = tm.items(ntx, B, nty)
            best = min(tm.makespan(tm.items(ntx, B, F), -(-max(h - F * T, 0) // T2) * ntx, 768) for F in range(nty + 1))
            got = tm.model_split(W, h, m, 768)
            assert best - 1e-9 <= got <= tm.makespan(n, 0, 768) + 1e-9, (W, h, m)
