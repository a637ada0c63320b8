// life_kernels.h -- host-side launchers of the gfx950 Game-of-Life kernels.
//
// All launchers are asynchronous on `s` and return the hipError_t of the
// launch.  Buffers are the padded shard layout of life_layout (see
// include/life_mi355x.h and DESIGN.md "Data layout in HBM").
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "life_host.h"
#include "life_mi355x.h"

namespace life {

// Region of owned cells a stencil launch updates: 16-byte units [u0,u1) of
// every padded row, owned rows [r0,r1) (0-based, padded row = r + 1).
struct Region {
    int64_t u0, u1, r0, r1;
};

// Kernel arguments of one stencil launch (by value).
struct StepArgs {
    const uint8_t *in;
    uint8_t *out;
    uint8_t *sink;  // >= 1 KiB scratch: stores of lanes outside the region land here
    int64_t pitch, xoff, units, w, h, ya;
    int64_t u0, u1, r0, r1, nbx;
    int32_t wrapy;
    int32_t xcd;  // 1: blocks renumbered into per-XCD row-major runs (step_kernel)
};

// Wrap flags: a periodic axis that lies entirely inside the shard (dims[d]
// == 1) is wrapped by the stencil itself (no apron, no fill kernel); the
// apron of a partitioned axis must hold the neighbours' cells.
struct Wrap {
    bool x, y;
};

// One generation over `reg`: reads `in`, writes `out`.
hipError_t launch_step(const life_layout &L, const uint8_t *in, uint8_t *out, uint8_t *sink,
                       const Region &reg, Wrap wrap, hipStream_t s);

// Tuning knobs of the stencil (rows per lane, rows of loads in flight);
// defaults chosen by measurement, overridable by LIFE_STEP_ROWS / LIFE_STEP_DEPTH.
struct StepTuning {
    int rows, depth;
};
StepTuning step_tuning(bool bit);
void set_step_tuning(int kernel, int rows, int depth);  // kernel -1: both

// Temporally blocked stencil (layouts with generations_per_exchange = K > 1,
// either encoding): tiles of 62 lane columns (bit: 64-cell interleaved pairs;
// byte: 32-cell words) x `rows` rows (one workgroup each), m <= min(K, 32)
// generations per launch from `in` to `out`; a bit tile's window holds m
// ghost rows above and below (byte: K), so the tile height depends on m:
// tile_geom(L, m).
constexpr int kMaxRegions = 4;  // regions one temporal launch may hold
struct TileRegion {
    int64_t tx0, tx1, ty0, ty1;
};
struct TileGeom {
    int64_t lanes;  // owned lane columns per tile (62)
    int64_t cells;  // cells per lane column: 64 (bit pairs) or 32 (byte words)
    int64_t rows, ntx, nty;
    int gsh;       // < 6: tile column bcol runs as bands of 2^gsh lanes (64 >> gsh tile rows per workgroup)
    int64_t bcol;  // the banded column (ntx - 1), -1 without banding
};
TileGeom tile_geom(const life_layout &L, int m);
// workgroups (items) one launch of region r takes: its full tiles, plus its
// banded items when it holds the banded column
int64_t region_items(const TileGeom &g, const TileRegion &r);
int tile_ghost(const life_layout &L, int m);  // ghost rows per window end: m (bit), K or 1 (byte, m = 1)
// Rows a temporally blocked buffer is allocated beyond its layout's `rows`:
// the last tile's window (<= 8 waves x 96 byte rows, 16 x 24 bit rows) may
// read past the bottom apron without clamping.
constexpr int64_t kTemporalSlackRows = 8 * 96;
// Dataflow form of the tiles (tflow_kernel): `passes` launches of m
// generations over a single shard whose axes both wrap inside it, as ONE
// persistent launch (no drain between passes).  `head` (2 words: the queue
// head, then an error word the caller zeroes once and reads: 1 + an item
// whose dependency wait timed out, 0 if none) and `done`
// (ntx * nty words, tile_geom(L, m)) are device scratch the launch zeroes;
// flow 1: write-through (`sc1`) stores, 2: plain stores + release fence.
// Pass p reads `in` for even p and `out` for odd p: after it, the result is
// in `out` when passes is odd, else in `in`.
bool flow_ok(const life_layout &L, int m);
// work items of one dataflow pass (tiles, or tiles + banded items of a banded
// last column; the queue also holds no-op items that pad the last group of
// banded rows unless work_only)
int64_t flow_items_per_pass(const life_layout &L, int m, bool work_only = false);
int flow_slots(const life_layout &L);  // resident workgroups of L's dataflow kernel on this device
int tile_slots(const life_layout &L);  // resident workgroups of L's per-launch tile kernel on this device
// ev0 / ev1 (optional): events stamped with the kernel dispatch's own start
// and end (hipExtLaunchKernel) -- no event packets between launches.
// One empty launch of the dataflow instance launch_tflow(L, m, flow) would use
// (and its occupancy query): the first launch of a kernel in a process costs
// ~140 us, which a device pays here at creation instead of inside its first
// dataflow step call.  `head`: the caller's scratch (2 words).
hipError_t prewarm_tflow(const life_layout &L, int m, int flow, unsigned int *head, hipStream_t s);
hipError_t launch_tflow(const life_layout &L, const uint8_t *in, uint8_t *out, int m, int64_t passes,
                        unsigned int *head, unsigned int *done, Wrap wrap, int flow, hipStream_t s,
                        hipEvent_t ev0 = nullptr, hipEvent_t ev1 = nullptr);
// Deep-halo passes (bit tiles, partitioned axes): the pass also advances the
// apron cells that stay valid for the next pass -- y rows [-y, 0) and
// [h, h + y) (the tile grid then spans h + 2y rows from owned row -y; the
// windows read at most y + m <= yapron rows above), and with x the apron
// pairs -1 and W are stored by the tile lanes that hold them.  A K-deep halo
// then feeds K generations (several passes) instead of one pass.
struct Extend {
    int64_t y = 0;
    bool x = false;
};
// Up to 4 disjoint tile regions in one launch; *valu_lane_ops (optional):
// the modelled VALU lane-ops of the launch as tiled (tstep_valu_per_tile_lane).
// Regions are in tile coordinates of tile_geom(extended_layout(L, ext), m).
// `concurrent`: items of another tile launch dispatched just before this one
// and running beside it (an exchange pass's ring beside its interior); the
// launch-tail plan of a one-region launch counts them as occupying slots
// (< 0: no launch-tail split).
hipError_t launch_tstep(const life_layout &L, const uint8_t *in, uint8_t *out, const TileRegion *r, int nreg,
                        int m, Wrap wrap, hipStream_t s,
                        double *valu_lane_ops = nullptr, hipEvent_t ev0 = nullptr, hipEvent_t ev1 = nullptr,
                        Extend ext = Extend{}, int64_t concurrent = 0);
// Computes (and caches) the launch-tail plans launch_tstep will use for the
// whole-shard launches of layout L at m = 1 .. mmax generations (with
// ext_y: also every deep-halo extension 0 .. K - m), so that a step call
// does not pay the planner's search (~50 us per new shape) before its first
// launch.
void prewarm_tail_plans(const life_layout &L, int mmax, bool ext_y);
// The layout a deep-halo pass tiles: h + 2 ext.y rows starting ext.y rows
// into the top apron.
life_layout extended_layout(const life_layout &L, const Extend &ext);
int temporal_rows(bool bit);      // register rows per wave: bit pair rows 16/24, byte word rows 32/48
int tile_waves(bool bit);         // waves per tile workgroup: 8
// VALU instructions the lanes at one lane position of a tile's waves issue
// for m generations (the op-count model of life_kernels.hip tstep_kernel,
// checked against the SQ_INSTS_VALU counter in profiles/); x 64 lanes x tiles.
double tstep_valu_per_tile_lane(int m, bool byte);
void set_temporal_rows(int kernel, int nr);  // kernel -1: both encodings (values valid for each)

// LDS-resident path for small single-shard grids: all `gens` generations in
// one single-workgroup launch (in -> out; in may equal out).  Usable when
// small_lds_bytes(L) <= kSmallMaxLds.
constexpr int64_t kSmallMaxLds = 160 * 1024;
int64_t small_lds_bytes(const life_layout &L);
hipError_t launch_small(const life_layout &L, const uint8_t *in, uint8_t *out, int64_t gens, hipStream_t s);
// Register-resident variant (one 1024-lane workgroup, the grid in VGPRs):
// usable when reg_small_rows(L) > 0 (at most 64 words per row and a strip
// height R from its instance list dividing h with h/R strips fitting the
// workgroup's lane groups); in != out.
int reg_small_rows(const life_layout &L);
hipError_t launch_reg_small(const life_layout &L, const uint8_t *in, uint8_t *out, int64_t gens,
                            hipStream_t s);
// Windowed register-resident variant over several CUs: ceil(h / own)
// workgroups, each holding own + 2K rows (strip height R) in VGPRs for at
// most K generations per launch; in != out.  reg_win_plan returns blocks == 0
// when the shape does not allow it.
struct RegWinPlan {
    int R, K, ns, own, blocks;
};
RegWinPlan reg_win_plan(const life_layout &L, int R, int K);
// nat_in / nat_out: the launch reads / writes natural 32-cell words instead
// of the shard's encoding (the launches inside one call; ignored, for every
// launch alike, when a row cannot hold them)
hipError_t launch_reg_win(const life_layout &L, const RegWinPlan &p, const uint8_t *in, uint8_t *out, int gens,
                          hipStream_t s, bool nat_in, bool nat_out);

// Column halo staging: pack writes the last xapron columns to slot 0 and the
// first xapron columns to slot 1 (h rows each: 1 byte 0/1 per row for a cell
// column, one 8-B pair per row for a bit-encoded 64-cell column, 32 bytes per
// row for a byte-encoded 32-cell column); unpack writes slot 0 into x in
// [-xapron, 0) and slot 1 into [w, w + xapron).
inline int64_t column_bytes_per_row(const life_layout &L) {
    if (L.xapron == 1) return 1;
    return L.kernel == LIFE_KERNEL_BIT ? 8 : 32;
}
// corners (the fused one-phase plan, life_halo_plan): also the four K x
// xapron corner blocks behind the two columns, K = yapron rows each.  Send
// slots 2h + cK + r, c in the plan's direction order SE, SW, NE, NW: my
// bottom-right, bottom-left, top-right, top-left K rows; receive slots in the
// same order: my top-left, top-right, bottom-left, bottom-right apron corner.
hipError_t launch_pack_columns(const life_layout &L, const uint8_t *buf, uint8_t *stage,
                               hipStream_t s, bool corners = false);
hipError_t launch_unpack_columns(const life_layout &L, uint8_t *buf, const uint8_t *stage,
                                 hipStream_t s, bool corners = false);
// staging bytes of one direction (send or receive) of a shard's exchange
inline int64_t column_stage_bytes(const life_layout &L) {
    return (2 * L.h + (L.xapron > 1 ? 4 * L.yapron : 0)) * column_bytes_per_row(L);
}
// Temporal layouts: a periodic x axis inside one shard is wrapped by the
// stencil (whole lane columns) when w is a multiple of the x-apron (64 bit
// cells, 32 byte cells); otherwise the shard fills its own aprons from its own
// columns (launch_wrap_columns, needs w >= xapron).
inline bool self_wrap_x(const life_layout &L, int dims0) {
    return L.xapron > 1 && dims0 == 1 && L.w % L.xapron != 0;
}
hipError_t launch_wrap_columns(const life_layout &L, uint8_t *buf, hipStream_t s);

// Dense w*h byte block (row pitch w) <-> padded encoded buffer.
hipError_t launch_import_block(const life_layout &L, const uint8_t *dense, uint8_t *buf,
                               hipStream_t s);
hipError_t launch_export_block(const life_layout &L, const uint8_t *buf, uint8_t *dense,
                               hipStream_t s);

// The block's VTK cell data: '0'/'1' + '\n' per owned cell, rows of 2w bytes.
hipError_t launch_vtk_block(const life_layout &L, const uint8_t *buf, uint8_t *out, hipStream_t s);
// Packed rows (LIFEBITS: bit x & 7 of byte x >> 3) of a block starting at
// global column x0: bits_row_bytes(L) bytes per row, the block's cells from
// bit x0 & 7 of its first byte on.
inline int64_t bits_row_bytes(const life_layout &L) { return ((L.x0 & 7) + L.w + 7) / 8; }
hipError_t launch_bits_block(const life_layout &L, const uint8_t *buf, uint8_t *out, hipStream_t s);

// Counter-based synthetic init of the owned cells (global indices).
hipError_t launch_fill_random(const life_layout &L, int64_t nx, uint64_t key, uint32_t thr32,
                              uint8_t *buf, hipStream_t s);

// Adds the live owned cells' count to out[0] and their checksum
// (sum of mix64(global y*nx + x + 1), mod 2^64) to out[1].
hipError_t launch_census(const life_layout &L, int64_t nx, const uint8_t *buf, unsigned long long *out,
                         hipStream_t s);

// Copy-ceiling probe: out[0, bytes) = in[0, bytes), bytes a multiple of 16.
hipError_t launch_copy(const void *in, void *out, int64_t bytes, hipStream_t s);

}  // namespace life
