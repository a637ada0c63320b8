// life_host.h -- host-only planning helpers of the runtime (life_plan.cpp):
// no HIP types, so CPU tests compile life_plan.cpp with g++ alone and check
// them without a GPU (tests/test_host_plan.py).
#pragma once
#include <stdint.h>

#include "life_mi355x.h"

namespace life {

// life_halo_plan with `loop` (bit 0: x, bit 1: y): that axis, with dims == 1,
// is exchanged too, the shard being its own neighbour (LIFE_OPT_LOOPBACK).
int halo_plan(int64_t nx, int64_t ny, int dims0, int dims1, int rank, int kernel, int loop, life_halo_op *ops,
              int max_ops);

// The dataflow queue head is 32-bit: one launch may hold at most
// kFlowMaxHead pulls (its items plus one extra pull per resident workgroup).
// flow_chunk_passes: passes of `tiles` items each one launch of `grid`
// resident workgroups may take (at most `cap` when cap > 0); 0 when not even
// one pass fits.  Host-only (life_plan.cpp).
constexpr int64_t kFlowMaxHead = (int64_t)1 << 31;
int64_t flow_chunk_passes(int64_t tiles, int64_t grid, int64_t cap);

// life_collect's fan-in (life_cart.c:281-305, 5-gather/life_mpi.c:177-179)
// as a plan: every rank exports its block in one of three frame formats
// (DENSE 1 B per cell, VTK 2 B, BITS = LIFEBITS packed rows), the root (rank
// world-1) places its own block first, then receives the others in rank order
// into two alternating staging slots (block k+1 arrives while block k is copied
// out).  Pure arithmetic on life_layout_query, shared by the device gather
// (life_dev.hip gather_impl) and the CPU tests.
enum GatherFormat { kGatherDense = 0, kGatherVtk = 1, kGatherBits = 2 };
struct GatherPiece {
    int32_t rank;         // the block's global rank
    int32_t slot;         // staging slot at the root: -1 = its own export, else 0 / 1
    int64_t bytes;        // message size = row_bytes * rows
    int64_t row_bytes;    // bytes per exported row
    int64_t rows;         // block rows
    int64_t dst;          // byte offset of its first row in the frame
    int32_t shared_first; // BITS: its first byte of every row is shared with the block on its left (OR-ed)
    int32_t shared_last;  // BITS: its last byte of every row is shared with the block on its right
};
int64_t gather_frame_row_bytes(int64_t nx, int fmt);
// Fills pieces[0 .. world) (the root's own first, then ranks 0 .. world-2 in
// receive order); *slot_bytes = the largest piece (one staging slot).
// Returns world, or LIFE_EINVAL.
int gather_plan(int64_t nx, int64_t ny, int dims0, int dims1, int kernel, int fmt, GatherPiece *pieces, int max,
                int64_t *slot_bytes);

// Launch-tail plan of one bit-tile launch over a full-width region (tile
// rows [ty0, ty1) of T owned rows each, the region ending at owned row
// yend): the first F tile rows stay full tiles, the rest become n2 tile rows
// of half-height tiles (T2 owned rows), banded in the last tile column like
// the full ones, dispatched last, so that the launch's last round is short
// items filling the slots the full tiles leave (life_kernels.hip
// launch_tstep).  Items of r tile rows: (ntx - 1) r + ceil(r
// / B) with bands of B tile rows (B > 1), else ntx r.  mode 1: round 4's rule
// (the fewest bottom rows whose half tiles fill one round, when the last
// round is under half full); mode 2: the split with the smallest makespan of
// a list schedule (items dealt in launch order to the earliest free of
// `slots` resident workgroups; full tiles last 1, half tiles c + (1 - c) /
// 2, c the fixed share of a tile: window load, stores, turnover).  F == ty1:
// no split.  Cached per argument set (a launch repeats its shape).
struct TailPlan {
    int64_t F = 0, n2 = 0;
    double makespan = 0.0;  // model tile-times (full tile = 1)
};
// items of `rows` tile rows `ntx` tile columns wide (the last column banded
// in items of B tile rows when B > 1)
inline int64_t tail_row_items(int64_t ntx, int64_t B, int64_t rows) {
    return rows <= 0 ? 0 : B > 1 ? (ntx - 1) * rows + (rows + B - 1) / B : ntx * rows;
}
// the list schedule's makespan of `pre` full items of another launch
// dispatched first (the ring beside an interior), F_rows full tile rows, then
// n2 half rows
double tail_makespan2(int64_t ntx, int64_t B, int64_t F_rows, int64_t n2, int64_t slots, double c, int64_t pre = 0);
TailPlan tail_plan(int64_t ntx, int64_t B, int64_t ty0, int64_t ty1, int64_t yend, int64_t T, int64_t T2,
                   int64_t slots, int mode, double c, int64_t pre = 0);

}  // namespace life
