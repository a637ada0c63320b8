"""DESIGN.md 6's predicted strong-scaling table is reproducible from the
committed round-5 validation logs (CPU only): scripts/strong_table.py over
profiles/r05/l's unpartitioned 65536^2 line and the RCCL-loopback lines of
configs[3]'s per-GPU blocks gives the efficiencies DESIGN quotes."""
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
L = os.path.join(ROOT, "profiles", "r05", "l")
LOGS = ["bench_default.log", "loop_32768x65536.log", "loop_32768x32768.log", "loop_16384x32768.log"]


@pytest.mark.skipif(not all(os.path.exists(os.path.join(L, f)) for f in LOGS), reason="r05/l logs not present")
def test_strong_table_matches_design():
    out = subprocess.run([sys.executable, os.path.join(ROOT, "scripts", "strong_table.py"),
                          *[os.path.join(L, f) for f in LOGS]], capture_output=True, text=True, check=True).stdout
    rows = [r for r in out.splitlines() if r.startswith("| ") and r[2].isdigit()]
    eff = {int(r.split("|")[1]): float(r.split("|")[-2]) for r in rows}
    assert eff == {2: 0.76, 4: 0.72, 8: 0.59}, out
    design = open(os.path.join(ROOT, "DESIGN.md")).read()
    for n, e in eff.items():
        assert f"| {n} |" in design and f"| {e:.2f} |" in design
