#!/usr/bin/env python3
"""List-scheduling model of one bit-tile launch: a pass of
full tiles (NW x R window rows, T = NW*R - 2m owned) and, for the bottom tile
rows, half-height tiles (T2 = NW*R/2 - 2m owned, half the duration), dealt in
order to `slots` resident workgroups.  Prints, per shape, the ideal length
in tile-times (tiles / slots), no split, round 4's rule (split the last tile
row when the last round is under half full), the split launch_tstep makes
now (LIFE_TAIL_SPLIT 2: every boundary searched with the closed form
`tail_makespan`, restated here as `closed_form`) and the best split by
simulation -- the 32768^2 pass is 2.17 ideal, 2.5 at best, which is why
geometry alone does not fix the small shapes.

    python3 scripts/tail_model.py [slots]

Round 6: the product's planner is life::tail_plan (csrc/life_plan.cpp): the
same list schedule simulated over slot groups, half tiles banded in the last
tile column like the full ones and lasting c + (1 - c) / 2 of a full tile
(c = 0.06), checked against a heap simulation and an exhaustive search by
tests/test_tail_plan.py.  This script keeps round 5's closed form (unbanded
half tiles of exactly half the duration) for the comparison.
"""
import heapq
import sys


def makespan(nfull, nhalf, slots, dh=0.5):
    free = [0.0] * slots
    end = 0.0
    for d, n in ((1.0, nfull), (dh, nhalf)):
        for _ in range(n):
            t = heapq.heappop(free) + d
            end = max(end, t)
            heapq.heappush(free, t)
    return end


def closed_form(full, half, slots):
    """life_kernels.hip tail_makespan: full tiles dealt round-robin, the half
    tiles filling the last full round's idle slots (two per slot) first."""
    r, rem = divmod(full, slots)
    if half == 0:
        return float(r + (1 if rem else 0))
    if rem == 0:
        return r + 0.5 * (-(-half // slots))
    gap = 2 * (slots - rem)
    if half <= gap:
        return float(r + 1)
    return r + 1 + 0.5 * (-(-(half - gap) // slots))


def geom(W, m, R=24, NW=8):
    T, T2 = NW * R - 2 * m, NW * R // 2 - 2 * m
    ntx = -(-W // 62)
    o = W - 62 * (ntx - 1)
    gsh = 2
    while (1 << gsh) < o + 2:
        gsh += 1
    B = 64 >> gsh if gsh <= 5 else 1  # banded last column: B tile rows per item
    return T, T2, ntx, B


def items(ntx, B, rows):
    return (ntx - 1) * rows + -(-rows // B) if B > 1 else ntx * rows


def model_split(W, h, m, slots):  # life_kernels.hip launch_tstep, LIFE_TAIL_SPLIT 2
    T, T2, ntx, B = geom(W, m)
    nty = -(-h // T)
    n = items(ntx, B, nty)
    if n <= slots or n % slots == 0:
        return makespan(n, 0, slots)
    best, bq = closed_form(n, 0, slots), 0
    for q in range(1, nty):
        F = nty - q
        t = closed_form(items(ntx, B, F), -(-(h - F * T) // T2) * ntx, slots)
        if t < best - 1e-9:
            best, bq = t, q
    F = nty - bq
    return makespan(items(ntx, B, F), -(-(h - F * T) // T2) * ntx if bq else 0, slots)


def rule_split(W, h, m, slots):  # round 4's rule (LIFE_TAIL_SPLIT 1)
    T, T2, ntx, B = geom(W, m)
    nty = -(-h // T)
    n = items(ntx, B, nty)
    rem = n % slots
    if n > slots and rem and rem <= slots // 2:
        q = 1
        while q < nty and (-(-(q * T) // T2)) * ntx < slots:
            q += 1
        F = nty - q
        return makespan(items(ntx, B, F), -(-(h - F * T) // T2) * ntx, slots)
    return makespan(n, 0, slots)


def main():
    slots = int(sys.argv[1]) if len(sys.argv) > 1 else 768
    for name, W, h in [("65536^2", 1024, 65536), ("32768x65536", 512, 65536), ("32768^2", 512, 32768),
                       ("16384x32768", 256, 32768)]:
        for m in (10, 12):
            T, T2, ntx, B = geom(W, m)
            nty = -(-h // T)
            n = items(ntx, B, nty)
            best = min((makespan(items(ntx, B, F), -(-max(h - F * T, 0) // T2) * ntx, slots), F)
                       for F in range(nty + 1))
            print(f"{name:12s} m={m:2d} tiles={n:5d} ideal={n / slots:.2f} no-split={makespan(n, 0, slots):.2f} "
                  f"rule={rule_split(W, h, m, slots):.2f} model={model_split(W, h, m, slots):.2f} best={best[0]:.2f} (full tile rows {best[1]} of {nty})")


if __name__ == "__main__":
    main()
