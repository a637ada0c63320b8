"""Per-workgroup timeline of the last bit tile launch (diagnostics builds only:
LIFE_WG_TRACE=1, loaded through LIFE_MI355X_LIB).  Runs the bench shape
(65536^2 or WG_TRACE_SHAPE=WxH, 20 generations from a 50 % soup) and summarises when workgroups
started and ended, how many ran at once per CU and XCD, and how long each took.
    usage: LIFE_MI355X_LIB=build_exp/trace/liblife_mi355x.so python scripts/wg_trace.py [gens] [out.npy]
"""
import ctypes
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "mpi-and-open-mp_amd"))
import life_mi355x as lm  # noqa: E402

gens = int(sys.argv[1]) if len(sys.argv) > 1 else 20
kernel = os.environ.get("WG_TRACE_KERNEL", "bit")  # byte: stamps after the load, the generations, the stores
nx, ny = (int(v) for v in os.environ.get("WG_TRACE_SHAPE", "65536x65536").split("x"))
flow = int(os.environ.get("WG_TRACE_FLOW", "0"))  # 1/2: the dataflow launch (one per call), items 0..3 stamped
with lm.Life(nx, ny, shards=1, kernel=kernel, flow=flow) as life:
    life.fill_random(1, 0.5)
    life.step(5)
    life.step(gens)
    life.live_count()
    L = lm._lib()
    n = 16 * 65536
    buf = (ctypes.c_uint64 * n)()
    fn = L.life_debug_wg_trace
    fn.argtypes = [ctypes.c_void_p, ctypes.c_int64]
    assert fn(buf, n) == 0
t = np.frombuffer(buf, dtype=np.uint64).reshape(-1, 16)
t = t[t[:, 0] > 0]
if flow:
    # per workgroup: start, hw id, then (pulled, dependencies met, stored) of its first 4 items
    t0 = int(t[:, 0].min())
    st = np.where(t[:, 2:14] > 0, (t[:, 2:14].astype(np.int64) - t0) / 100.0, np.nan).reshape(-1, 4, 3)
    wait = st[:, :, 1] - st[:, :, 0]
    body = st[:, :, 2] - st[:, :, 1]
    turn = st[:, 1:, 0] - st[:, :-1, 2]
    q = lambda v: " ".join(f"{np.nanpercentile(v, p):.1f}" for p in (10, 50, 90, 99))  # noqa: E731
    print(f"flow: {len(t)} workgroups; per item (pct 10/50/90/99, us)")
    for i in range(4):
        print(f"  item {i}: pulled at {q(st[:, i, 0])} | dep wait {q(wait[:, i])} | body {q(body[:, i])}")
    print(f"  turnover (stored -> next pulled): {q(turn)}")
    ends = st[:, :, 2].ravel()
    ts = np.linspace(0, np.nanmax(ends), 31)
    busy = [int(np.nansum((st[:, :, 1] <= x) & (st[:, :, 2] > x))) for x in ts]
    print("items computing over time (first 4 per workgroup only):", busy)
    sys.exit(0)
t0 = int(t[:, 0].min())
start = (t[:, 0].astype(np.int64) - t0) / 100.0  # us
tiles = np.where(t[:, 2:] > 0, (t[:, 2:].astype(np.int64) - t0) / 100.0, np.nan)  # end of each tile
end = np.nanmax(tiles, axis=1)
hw = t[:, 1] & 0xFFFFFFFF
xcc = (t[:, 1] >> 32) & 0xF
cu = (hw >> 8) & 0xF
sh = (hw >> 12) & 1
se = (hw >> 13) & 0x7
cuid = (xcc.astype(np.int64) * 8 + se.astype(np.int64)) * 32 + sh.astype(np.int64) * 16 + cu.astype(np.int64)
dur = end - start
ok = end > start
print(f"workgroups {len(t)} (ended {ok.sum()}), span {end.max():.1f} us")
print("start  pct 0/50/90/99/100: " + " ".join(f"{np.percentile(start, p):.1f}" for p in (0, 50, 90, 99, 100)))
print("end    pct 0/10/50/90/100: " + " ".join(f"{np.percentile(end[ok], p):.1f}" for p in (0, 10, 50, 90, 100)))
print("dur    pct 0/10/50/90/100: " + " ".join(f"{np.percentile(dur[ok], p):.1f}" for p in (0, 10, 50, 90, 100)))
u, c = np.unique(cuid, return_counts=True)
print(f"CUs used {len(u)}; workgroups per CU min/median/max {c.min()}/{int(np.median(c))}/{c.max()}")
print("per XCC workgroups:", np.bincount(xcc.astype(np.int64), minlength=8).tolist())
# concurrency: workgroups resident at time t, sampled
ts = np.linspace(0, end.max(), 41)
conc = [int(((start <= x) & (end > x)).sum()) for x in ts]
print("resident over time:", conc)
# per-CU busy span vs kernel span
last = {}
for i, k in enumerate(cuid):
    last[k] = max(last.get(k, 0), end[i])
lv = np.array(list(last.values()))
print("per-CU last end pct 0/10/50/90/100: " + " ".join(f"{np.percentile(lv, p):.1f}" for p in (0, 10, 50, 90, 100)))
# duration vs how many workgroups shared the CU at the midpoint of each
mid = (start + end) / 2
share = np.array([int(((cuid == cuid[i]) & (start <= mid[i]) & (end > mid[i])).sum()) for i in range(len(t))])
for s_ in np.unique(share):
    m = share == s_
    print(f"  sharing {s_}: {m.sum()} workgroups, median dur {np.median(dur[m]):.1f} us")
ntile = np.sum(~np.isnan(tiles), axis=1)
if ntile.max() > 1:  # skewed segments: time per tile (the first includes the prologue); byte: per phase
    per = np.diff(np.concatenate([start[:, None], tiles], 1), axis=1)
    print("per tile median by position:", [round(float(np.nanmedian(per[:, k])), 1) for k in range(int(ntile.max()))])
if len(sys.argv) > 2:
    np.save(sys.argv[2], np.concatenate([np.stack([start, end, cuid, xcc], 1), tiles], 1))
