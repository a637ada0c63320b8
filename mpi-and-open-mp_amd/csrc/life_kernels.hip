// life_kernels.hip -- gfx950 (CDNA4) kernels of the Game-of-Life hot path.
//
// Replaces the reference's life_step (6-cartesian/life_cart.c:189-215, the
// same body as 3-life/life2d.c:104-130): B3/S23 on a periodic grid.  The
// reference reads 9 ints through a modulo-wrapping ind() per cell; here every
// shard is a padded block whose one-cell apron holds the periodic / remote
// neighbours (filled by the halo phase), so the stencil is branch-free.
//
// Stencil mapping (both encodings): one lane owns a 16-byte unit of a row and
// walks R consecutive rows down, keeping the horizontal 3-sums of rows y-1,
// y, y+1 in registers (vertical reuse in registers, no LDS round trip).  The
// horizontal neighbours of a unit's edge cells come from lanes +-1 by DPP
// wave shifts (v_mov_b32_dpp wave_shr/wave_shl); lane 0 / lane 63 fetch the
// one dword beyond the wave's span themselves.  HBM traffic is one read and
// one write of each cell's encoding plus 2/R of re-read halo rows.
//
//  * ByteEnc: 1 byte per cell.  SWAR on 4 cells per dword: horizontal sum via
//    v_alignbyte, 9-cell sum n9 <= 9 per byte, rule ((n9 - c) | c) == 3.
//  * BitEnc: 1 bit per cell in 64-cell interleaved pairs (E = even cells,
//    O = odd cells, life_bitops.h).  Horizontal (L,C,R) full adder -> 2-bit
//    sum per row; three rows add to n9 = u0 + 2*S; alive' = (n9 == 3) |
//    (alive & n9 == 4).  Every boolean step is one v_bitop3_b32 (per pair:
//    2 funnel shifts + 4 ops for the two rows sums, 2 x 8 for the rule).
#include "life_kernels.h"
#include "life_bitops.h"
#include "life_diag.h"

#include <hip/hip_ext.h>

#include <algorithm>
#include <stdint.h>
#include <stdlib.h>

namespace life {
namespace {

constexpr int kBlock = 256;  // 4 waves of 64

__device__ __forceinline__ uint32_t from_left(uint32_t old, uint32_t v) {
    // lane i <- lane i-1 (wave_shr:1); lane 0 keeps `old`.
    return (uint32_t)__builtin_amdgcn_update_dpp((int)old, (int)v, 0x138, 0xf, 0xf, false);
}
__device__ __forceinline__ uint32_t from_right(uint32_t old, uint32_t v) {
    // lane i <- lane i+1 (wave_shl:1); lane 63 keeps `old`.
    return (uint32_t)__builtin_amdgcn_update_dpp((int)old, (int)v, 0x130, 0xf, 0xf, false);
}

// ------------------------------------------------------------------ encodings
struct ByteEnc {
    static constexpr int64_t kCellsPerUnit = 16;
    static constexpr uint32_t kCell0 = 0xFFu;  // cell 0 of a dword
    static __device__ __forceinline__ int64_t dword_of(int64_t x) { return x >> 2; }
    static __device__ __forceinline__ uint32_t pos_in_dword(int64_t x) { return 8u * (uint32_t)(x & 3); }
    static __device__ __forceinline__ uint32_t top_shift(int64_t x) { return 24u - pos_in_dword(x); }
    struct H {
        uint32_t v[4];
    };
    // Horizontal 3-sum (x-1, x, x+1) of 16 byte cells; l / r: dword left of
    // d.x and dword right of d.w.
    static __device__ __forceinline__ H hsum(uint4 d, uint32_t l, uint32_t r) {
        H h;
        h.v[0] = d.x + __builtin_amdgcn_alignbyte(d.x, l, 3) + __builtin_amdgcn_alignbyte(d.y, d.x, 1);
        h.v[1] = d.y + __builtin_amdgcn_alignbyte(d.y, d.x, 3) + __builtin_amdgcn_alignbyte(d.z, d.y, 1);
        h.v[2] = d.z + __builtin_amdgcn_alignbyte(d.z, d.y, 3) + __builtin_amdgcn_alignbyte(d.w, d.z, 1);
        h.v[3] = d.w + __builtin_amdgcn_alignbyte(d.w, d.z, 3) + __builtin_amdgcn_alignbyte(r, d.w, 1);
        return h;
    }
    static __device__ __forceinline__ uint32_t rule1(uint32_t n9, uint32_t c) {
        const uint32_t m = (n9 - c) | c;                          // n8 | alive, per byte <= 9
        const uint32_t t = m ^ 0x03030303u;                       // 0 where m == 3
        const uint32_t nz = (t + 0x7F7F7F7Fu) & 0x80808080u;      // 0x80 where t != 0
        return (nz ^ 0x80808080u) >> 7;
    }
    static __device__ __forceinline__ uint4 rule(const H &a, const H &b, const H &c, uint4 v) {
        uint4 o;
        o.x = rule1(a.v[0] + b.v[0] + c.v[0], v.x);
        o.y = rule1(a.v[1] + b.v[1] + c.v[1], v.y);
        o.z = rule1(a.v[2] + b.v[2] + c.v[2], v.z);
        o.w = rule1(a.v[3] + b.v[3] + c.v[3], v.w);
        return o;
    }
};


// ------------------------------------------------------------------ stencil
// Per-lane constants of one stencil launch.  Every load is unconditional (a
// lane right of the row reads a clamped, in-pitch unit) and every store
// goes somewhere (a lane that must not write redirects to `sink` with row
// stride 0), so a lane's whole strip is ONE basic block and the prefetch ring
// below really keeps D rows of loads in flight.
struct Lane {
    const uint8_t *in;
    int64_t pitch, h, ya;
    int64_t off;        // byte offset of the (clamped) unit in a padded row
    int64_t exoff;      // extra dword: left (lane 0), right (lane 63), wrap-left (unit 0)
    uint32_t exshift;   // wrap-left: move cell w-1 to the top position of the dword
    int64_t xoff;       // word 0 of a row (wrap-right source)
    uint4 pmask;        // wrap-right: where cell w sits inside this unit (last unit only)
    uint32_t pshift;    //   ... its bit/byte position within that dword
    bool pright;        // wrap-right: cell w is the right extra (w % cells_per_unit == 0)
    bool needex;        // lanes 0 / 63 and the wrap-left unit: the extra dword is read
    bool wrapy;
};

__device__ __forceinline__ const uint8_t *row_ptr(const Lane &c, int64_t y) {
    // owned row y in [-1, h]; with a periodic y axis inside the shard the
    // apron rows are the opposite owned rows (ind() wrap, life_cart.c:11).
    if (c.wrapy) y = y < 0 ? y + c.h : (y >= c.h ? y - c.h : y);
    return c.in + (y + c.ya) * c.pitch;
}

struct RowData {
    uint4 d;
    uint32_t ex, e0;
};

// A dword every lane reads at the same address, through the VECTOR memory
// path: the opaque zero offset keeps the compiler from turning a
// wave-uniform address into a scalar (constant-cache) load of grid data
// another kernel wrote.
__device__ __forceinline__ uint32_t load_u32_vec(const uint8_t *p) {
    uint32_t z;
    asm volatile("v_mov_b32 %0, 0" : "=v"(z));
    return *reinterpret_cast<const uint32_t *>(p + z);
}

template <bool WRAPX>
__device__ __forceinline__ RowData load_row(const Lane &c, int64_t y) {
    const uint8_t *row = row_ptr(c, y);
    RowData r;
    r.d = *reinterpret_cast<const uint4 *>(row + c.off);
    // only the lanes whose neighbour dword lies outside the wave (0, 63, the
    // wrap-left unit) load it: one memory instruction per row instead of two
    // for the other 62 lanes (their ex is never read: DPP takes lanes +-1)
    r.ex = c.needex ? *reinterpret_cast<const uint32_t *>(row + c.exoff) : 0u;
    r.e0 = WRAPX ? load_u32_vec(row + c.xoff) : 0u;  // one address per wave
    return r;
}

template <class E, bool WRAPX>
__device__ __forceinline__ typename E::H row_sum(const Lane &c, RowData &r) {
    uint32_t ex = r.ex << c.exshift;
    uint32_t right = from_right(ex, r.d.x);
    if (WRAPX) {
        // the cell right of w-1 is cell 0 of the row (periodic x inside the shard)
        const uint32_t c0 = (r.e0 & E::kCell0) << c.pshift;
        r.d.x = (r.d.x & ~c.pmask.x) | (c0 & c.pmask.x);
        r.d.y = (r.d.y & ~c.pmask.y) | (c0 & c.pmask.y);
        r.d.z = (r.d.z & ~c.pmask.z) | (c0 & c.pmask.z);
        r.d.w = (r.d.w & ~c.pmask.w) | (c0 & c.pmask.w);
        right = c.pright ? r.e0 : right;
    }
    return E::hsum(r.d, from_left(ex, r.d.w), right);
}

// N output rows starting at owned row ys (owned rows ys-1 .. ys+N are read),
// D rows of loads kept in flight.
template <class E, int N, int D, bool WRAPX>
__device__ __forceinline__ void strip_full(const Lane &c, int64_t ys, uint8_t *dst, int64_t spitch) {
    static_assert(D <= N + 2, "prefetch deeper than the strip");
    RowData q[D];
#pragma unroll
    for (int k = 0; k < D; ++k) q[k] = load_row<WRAPX>(c, ys - 1 + k);
    typename E::H hp, hc;
    uint4 cc;
#pragma unroll
    for (int k = 0; k < N + 2; ++k) {
        RowData r = q[k % D];
        if (k + D < N + 2) q[k % D] = load_row<WRAPX>(c, ys - 1 + k + D);
        const typename E::H hn = row_sum<E, WRAPX>(c, r);
        if (k == 0) {
            hp = hn;
        } else if (k == 1) {
            hc = hn;
            cc = r.d;
        } else {
            *reinterpret_cast<uint4 *>(dst) = E::rule(hp, hc, hn, cc);
            dst += spitch;
            hp = hc;
            hc = hn;
            cc = r.d;
        }
    }
}

template <class E, bool WRAPX>
__device__ __forceinline__ void strip_tail(const Lane &c, int64_t ys, int n, uint8_t *dst, int64_t spitch) {
    RowData r = load_row<WRAPX>(c, ys - 1);
    typename E::H hp = row_sum<E, WRAPX>(c, r);
    r = load_row<WRAPX>(c, ys);
    typename E::H hc = row_sum<E, WRAPX>(c, r);
    uint4 cc = r.d;
#pragma unroll 1
    for (int i = 0; i < n; ++i) {
        r = load_row<WRAPX>(c, ys + 1 + i);
        const typename E::H hn = row_sum<E, WRAPX>(c, r);
        *reinterpret_cast<uint4 *>(dst) = E::rule(hp, hc, hn, cc);
        dst += spitch;
        hp = hc;
        hc = hn;
        cc = r.d;
    }
}

template <class E, int R, int D, bool WRAPX>
__global__ __launch_bounds__(kBlock) void step_kernel(StepArgs a) {
    int64_t b = blockIdx.x;
    if (a.xcd) {
        // blocks b, b + 8, ... share an XCD: give each XCD a contiguous
        // row-major run of strips, so the strips beside and below a strip
        // (the extra dwords of lanes 0 / 63, the two halo rows) hit its L2
        const int64_t n = (int64_t)gridDim.x, x = b & 7, k = b >> 3, per = n >> 3, rem = n & 7;
        b = (x < rem ? x * (per + 1) : rem * (per + 1) + (x - rem) * per) + k;
    }
    const int64_t bx = b % a.nbx, by = b / a.nbx;
    const int lane = threadIdx.x & 63;
    const int64_t wbase = a.u0 + (bx * (kBlock / 64) + __builtin_amdgcn_readfirstlane(threadIdx.x >> 6)) * 64;
    if (wbase >= a.u1) return;  // the whole wave is right of the region
    const int64_t ys = a.r0 + by * R;
    const int64_t u = wbase + lane;
    const int64_t uc = u < a.units ? u : a.units;  // unit `units` is in-pitch: right-neighbour provider
    Lane c;
    c.in = a.in;
    c.pitch = a.pitch;
    c.h = a.h;
    c.ya = a.ya;
    c.wrapy = a.wrapy != 0;
    c.xoff = a.xoff;
    c.off = a.xoff + 16 * uc;
    c.exoff = c.off;
    c.exshift = 0;
    if (lane == 0) c.exoff = c.off - 4;
    if (lane == 63 && u < a.units) c.exoff = c.off + 16;
    c.needex = lane == 0 || lane == 63;
    c.pmask = make_uint4(0u, 0u, 0u, 0u);
    c.pshift = 0;
    c.pright = false;
    if (WRAPX) {
        if (u == 0) {  // left of cell 0 is cell w-1
            const int64_t wl = a.w - 1;
            c.exoff = a.xoff + E::dword_of(wl) * 4;
            c.exshift = E::top_shift(wl);
            c.needex = true;
        }
        if (u == a.units - 1) {  // right of cell w-1 is cell 0
            const int64_t q = a.w - (a.units - 1) * E::kCellsPerUnit;  // 1 .. kCellsPerUnit
            if (q == E::kCellsPerUnit) {
                c.pright = true;
            } else {
                const int comp = (int)E::dword_of(q);
                const uint32_t m = E::kCell0 << E::pos_in_dword(q);
                c.pshift = E::pos_in_dword(q);
                c.pmask.x = comp == 0 ? m : 0u;
                c.pmask.y = comp == 1 ? m : 0u;
                c.pmask.z = comp == 2 ? m : 0u;
                c.pmask.w = comp == 3 ? m : 0u;
            }
        }
    }
    const bool st = u < a.u1;
    uint8_t *dst = st ? a.out + (ys + a.ya) * a.pitch + a.xoff + 16 * u : a.sink + 16 * lane;
    const int64_t spitch = st ? a.pitch : 0;
    const int64_t n = a.r1 - ys < R ? a.r1 - ys : R;
    if (n == R)
        strip_full<E, R, D, WRAPX>(c, ys, dst, spitch);
    else
        strip_tail<E, WRAPX>(c, ys, (int)n, dst, spitch);
}

// ------------------------------------------------------------------ temporal
// Temporally blocked stencils (layouts with generations_per_exchange = K
// > 1): m <= K generations per launch, each cell read once from and written
// once to HBM per pass (plus the ghost rows of its window).  A tile is one
// workgroup of NW vertically stacked waves holding a window of NW*R rows x 64
// lane columns in registers, all m generations with one barrier each; lanes 0
// and 63 are the tile's x-apron, so a tile owns 62 lane columns.  A lane
// column is one interleaved pair (64 cells) for the bit encoding
// (tile_body_bit) and one 32-cell word, packed from 32 byte cells on load,
// for the byte encoding (tile_body_byte).  Two launch forms:
//
//  * tstep_kernel: one launch per pass, up to 4 tile regions (the boundary
//    ring of a partitioned shard, or the whole shard);
//  * tflow_kernel (bit): every pass of a step call on a single wrapped shard
//    in one persistent launch, tiles handed from pass to pass (LIFE_OPT_FLOW).

constexpr int kStackWaves = 8;  // waves per byte tile workgroup (2 per SIMD; 12 measured slower, profiles/r02/r2w)
struct TArgs {
    const uint8_t *in;
    uint8_t *out;
    int64_t pitch, xoff, W, h, ya;  // W = lane columns per owned row: pairs (bit) or 32-cell words (byte)
    // up to kMaxRegions tile regions in one launch (the boundary ring of a
    // partitioned shard); workgroup b belongs to the region with first[k] <= b
    int64_t tx0[kMaxRegions], tx1[kMaxRegions], ty0[kMaxRegions], ty1[kMaxRegions], first[kMaxRegions + 1];
    int32_t nreg, m;  // generations of the launch = ghost rows at each end of a window (bit)
    // banded tile column (bit; tile_geom): gsh < 6 cuts the tiles of column
    // bcol into bands of G = 2^gsh lanes, 64 / G tile rows per workgroup; a
    // region whose tx1 == bcol + 1 lists its full tiles first, then its
    // ceil((ty1 - ty0) / (64 / G)) banded items
    int32_t gsh;
    int64_t bcol;
    // tail split (bit, a launch of one region; launch_tstep): with tail_ntx
    // > 0, workgroups >= tail_first run half-height tiles (R / 2 rows per
    // wave) over owned rows [tail_y, tail_yend), tile columns [tail_tx0,
    // tail_tx0 + tail_ntx) per tile row, the last one banded like the full
    // tiles when it is the banded column (tail_band), so the last round of a
    // launch is made of half-length items
    int64_t tail_first, tail_y, tail_yend, tail_ntx, tail_tx0;
    int32_t tail_band;
    // XCD-aware order (bit, LIFE_XCD_ORDER): workgroups [0, xcd_n) are
    // renumbered so that each XCD (blocks b, b + 8, ... share one) walks a
    // contiguous row-major run of items; 0: dispatch order
    int64_t xcd_n;
    // deep-halo pass (Extend::x, bit): the lanes holding the apron pairs -1
    // and W store them too
    int32_t xext;
};

template <int NW>
using Xch = uint32_t[2][NW][4][64];  // byte tiles: [parity][wave][top s0/s1, bottom s0/s1][lane]
// bit tiles: [parity][1 + wave][top e0 e1 o0 o1, bottom ...][lane]; slots 0
// and NW + 1 stay zero (the dead rows beyond the window): no branch on the
// wave index in the generation loop
template <int NW>
using XchP = uint32_t[2][NW + 2][8][64];
template <int NW>
struct XchB {
    XchP<NW> s;
};

// Bit tiles over interleaved pairs.  Lane l of a tile holds pair column
// 62 tx + l - 1 of R consecutive window rows as (E, O) register pairs; wave
// i holds window rows [iR, (i+1)R) of a window that starts m rows above the
// tile, T = NW*R - 2m owned rows per tile.  Per generation and row: the
// neighbour dwords of the lanes on either side by two ds_bpermute (the LDS
// pipe; measured 4 % faster than a DPP move for the left one,
// profiles/r03/ubench_pair.txt), 2 v_alignbit, 2 full adders (4 v_bitop3) for
// the even and odd cells' horizontal sums, and the rule (8 v_bitop3) per
// dword: 22 VALU + 2 LDS per pair-row, 11 VALU per 32 cells (the natural
// one-word layout: 13).  Each generation a wave publishes the sums of its
// first and last row in LDS (8 dwords per lane), one barrier, and takes its
// neighbours'; the window's top and bottom m rows and the edge lanes absorb
// the wrong values that enter from outside (m rows / m <= 32 cells after m
// generations), so rows [m, NW*R - m) of lanes 1..62 are exact and stored.
//
// FLOW (tflow_kernel): the window is loaded with agent-scope (`sc1`,
// L1-bypassing) 8-B atomic-form loads, and stored with `sc1` write-through
// stores (FLOW 1) or plain stores (FLOW 2, the kernel releases them with a
// fence): the rows are another workgroup's output of the same launch.
//
// Banded tiles: a tile column that owns o <= 30 pairs (the last one: W =
// 62 (ntx - 1) + o) wastes most of a 64-lane tile.  With gsh < 6 the wave is
// cut into groups of G = 2^gsh lanes (1 ghost + o owned + ghost pairs), group
// g holding tile row ty + g of that column: one workgroup carries nb <= 64 /
// G tile rows ("bands").  The neighbour dwords a group's edge lanes fetch
// come from the adjacent group: garbage, exactly as a tile's lanes 0 / 63
// read beyond the tile, absorbed by the ghost lanes.  Only the loads and
// stores differ (per-lane rows); the generation loop is the tile's.  gsh = 6:
// an ordinary tile (nb = 1).
// LIFE_FLOW_BP_AHEAD (default 1): the dataflow tiles' generation loop issues
// each row's two neighbour permutes that many rows ahead of their use, rows
// fenced in program order.  Left to itself the compiler scheduled that loop
// (more live state around it than in tstep_bit_kernel's) with every permute
// right before its wait: mean permute -> wait distance 1.8 instructions
// against 7.6-9.8 in the per-launch tiles (tests/test_isa.py), the
// scheduling loss round 4 measured at 8 % there.  (Forcing the same in the
// per-launch tiles, whose own schedule is good, cost 1-3.5 %: off there.)
#ifndef LIFE_FLOW_BP_AHEAD
#define LIFE_FLOW_BP_AHEAD 1
#endif
// LIFE_FAST_WRAP: a tile's wrapped pair column and first row by one
// conditional add / subtract instead of a 64-bit remainder (per lane for the
// column) when the axis is long enough for the index to be at most one
// period out; the remainder stays for short axes.  Driver-shaped launch
// 0.4346 vs 0.4400 ms mean over three ABAB pairs on one box (-1.2 %, noisy),
// byte flat; parity + golden modules green (profiles/r04/fastwrap_ad).
#ifndef LIFE_FAST_WRAP
#define LIFE_FAST_WRAP 1
#endif

template <int R, bool WRAPX, bool WRAPY, int FLOW, int NW, bool BAND = false>
__device__ __forceinline__ void tile_body_bit(const TArgs &a, const uint8_t *in, uint8_t *out, int64_t tx,
                                              int64_t ty, XchB<NW> &xb, int gsh = 6, int nb = 1,
                                              int64_t ybase = 0, int64_t yend = -1) {
    XchP<NW> &xch = xb.s;
    static_assert(R >= 3, "window");
    const int K = a.m;  // ghost rows per window end
    const int T = NW * R - 2 * K;
    const int lane = threadIdx.x & 63;
    const int laddr = ((lane - 1) & 63) << 2, raddr = ((lane + 1) & 63) << 2;
    // wave index: uniform, so every row address below is scalar (SALU) math
    const int wi = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int gl = BAND ? lane >> gsh : 0;                  // this lane's band (tile row ty + gl)
    const int pin = BAND ? lane & ((1 << gsh) - 1) : lane;  // lane within its group
    const int64_t j = tx * 62 + pin - 1;                    // pair column of this lane
    int64_t jl;
    if (WRAPX) {
        // j lies in [-1, W + 62): one conditional add / subtract when W >= 64
        // (a 64-bit remainder per lane otherwise, ~100 VALU per tile)
        if (LIFE_FAST_WRAP && a.W >= 64) {
            jl = j < 0 ? j + a.W : (j >= a.W ? j - a.W : j);
        } else {
            jl = j % a.W;
            if (jl < 0) jl += a.W;
        }
    } else {
        jl = j > a.W ? a.W : j;  // pairs -1 .. W hold cells / apron; beyond: clamp (never stored)
    }
    const uint32_t voff = (uint32_t)(a.xoff + 8 * jl);
    const int64_t y0 = ybase + ty * T - K + (int64_t)wi * R;  // owned row of register row 0 (>= -K)
    // Row pointers are walked: with a periodic y axis the walk wraps at h;
    // with an apron the last tile's window may run past the apron row h+K-1
    // into the allocation slack below the buffer (kTemporalSlackRows; those
    // rows are never stored).
    const uint8_t *row0 = in + a.ya * a.pitch;  // owned row 0
    uint32_t ve[R], vo[R];
    {
        int64_t y = y0 + (BAND ? (int64_t)(gl < nb ? gl : nb - 1) * T : 0);  // bands: per-lane rows
        if (WRAPY) {
            // y lies in [-K, h + 16 T + NW R) (a band lane adds gl T, gl < 16):
            // one conditional add / subtract when h exceeds that margin with
            // room to spare (a 64-bit remainder otherwise)
            if (LIFE_FAST_WRAP && a.h > 65 * (int64_t)(NW * R)) {
                y = y < 0 ? y + a.h : (y >= a.h ? y - a.h : y);
            } else {
                y %= a.h;
                if (y < 0) y += a.h;
            }
        }
        const uint8_t *p = row0 + y * a.pitch;
#pragma unroll
        for (int r = 0; r < R; ++r) {
            uint64_t q;
            if (FLOW)
                q = __hip_atomic_load(reinterpret_cast<uint64_t *>(const_cast<uint8_t *>(p) + voff),
                                      __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            else
                q = *reinterpret_cast<const uint64_t *>(p + voff);
            ve[r] = (uint32_t)q;
            vo[r] = (uint32_t)(q >> 32);
            ++y;
            if (WRAPY && y == a.h) {
                y = 0;
                p = row0;
            } else {
                p += a.pitch;
            }
        }
    }
    auto hsum = [&](uint32_t e, uint32_t o, uint32_t &e0, uint32_t &e1, uint32_t &o0, uint32_t &o1) {
        BitEnc::pair_sums(e, o, bperm(laddr, o), bperm(raddr, e), e0, e1, o0, o1);
    };
    // Register budget (80 VGPRs at 3 tiles per CU, R = 24: 48 hold the
    // window): only the rolling sums of three rows stay live across the
    // loop.  Row 0 is updated first (its upper neighbour's sums come from LDS
    // right after the barrier), the bottom row's own sums and the row below
    // the wave are read back from LDS when row R-1 is reached.  No branch on
    // the wave index inside the loop (the zero slots stand for the dead rows
    // beyond the window): a branch there split the loop body into blocks and
    // the every row's ds_bpermute was hoisted above it, their 2R results
    // spilling (46-83 VGPRs at R = 24).
    if (wi == 0 || wi == NW - 1)  // the dead slots (ordered by the first barrier below)
        for (int q = 0; q < 16; ++q) xch[q >> 3][wi == 0 ? 0 : NW + 1][q & 7][lane] = 0u;
    for (int g = 0; g < a.m; ++g) {
        const int par = g & 1;
        uint32_t pe0, pe1, po0, po1, ce0, ce1, co0, co1;
        {
            uint32_t be0, be1, bo0, bo1;
            hsum(ve[R - 1], vo[R - 1], be0, be1, bo0, bo1);
            xch[par][wi + 1][4][lane] = be0;
            xch[par][wi + 1][5][lane] = be1;
            xch[par][wi + 1][6][lane] = bo0;
            xch[par][wi + 1][7][lane] = bo1;
        }
        hsum(ve[0], vo[0], pe0, pe1, po0, po1);
        xch[par][wi + 1][0][lane] = pe0;
        xch[par][wi + 1][1][lane] = pe1;
        xch[par][wi + 1][2][lane] = po0;
        xch[par][wi + 1][3][lane] = po1;
        __syncthreads();
        hsum(ve[1], vo[1], ce0, ce1, co0, co1);
        {
            // the wave above (slot 0 above the window: zero, dead ghost rows)
            const uint32_t ae0 = xch[par][wi][4][lane], ae1 = xch[par][wi][5][lane];
            const uint32_t ao0 = xch[par][wi][6][lane], ao1 = xch[par][wi][7][lane];
            ve[0] = BitEnc::rule1(ae0, ae1, pe0, pe1, ce0, ce1, ve[0]);
            vo[0] = BitEnc::rule1(ao0, ao1, po0, po1, co0, co1, vo[0]);
        }
        constexpr int BAH = FLOW ? LIFE_FLOW_BP_AHEAD : 0;  // permutes ahead (dataflow tiles only)
        uint32_t bl[BAH > 0 ? BAH : 1], br[BAH > 0 ? BAH : 1];
#pragma unroll
        for (int k = 0; k < BAH; ++k)
            if (2 + k < R - 1) {
                bl[k] = bperm(laddr, vo[2 + k]);
                br[k] = bperm(raddr, ve[2 + k]);
            }
#pragma unroll
        for (int r = 1; r < R - 1; ++r) {
            uint32_t ne0, ne1, no0, no1;
            if (r + 1 == R - 1) {  // published before the barrier
                ne0 = xch[par][wi + 1][4][lane];
                ne1 = xch[par][wi + 1][5][lane];
                no0 = xch[par][wi + 1][6][lane];
                no1 = xch[par][wi + 1][7][lane];
            } else if (BAH > 0) {
                const uint32_t l = bl[0], rr = br[0];
#pragma unroll
                for (int k = 0; k + 1 < BAH; ++k) {
                    bl[k] = bl[k + 1];
                    br[k] = br[k + 1];
                }
                if (r + 1 + BAH < R - 1) {
                    bl[BAH - 1] = bperm(laddr, vo[r + 1 + BAH]);
                    br[BAH - 1] = bperm(raddr, ve[r + 1 + BAH]);
                }
                __builtin_amdgcn_sched_barrier(0);
                BitEnc::pair_sums(ve[r + 1], vo[r + 1], l, rr, ne0, ne1, no0, no1);
            } else {
                hsum(ve[r + 1], vo[r + 1], ne0, ne1, no0, no1);
            }
            ve[r] = BitEnc::rule1(pe0, pe1, ce0, ce1, ne0, ne1, ve[r]);
            vo[r] = BitEnc::rule1(po0, po1, co0, co1, no0, no1, vo[r]);
            pe0 = ce0;
            pe1 = ce1;
            po0 = co0;
            po1 = co1;
            ce0 = ne0;
            ce1 = ne1;
            co0 = no0;
            co1 = no1;
        }
        {
            // the wave below (slot NW + 1 below the window: zero)
            const uint32_t de0 = xch[par][wi + 2][0][lane], de1 = xch[par][wi + 2][1][lane];
            const uint32_t do0 = xch[par][wi + 2][2][lane], do1 = xch[par][wi + 2][3][lane];
            ve[R - 1] = BitEnc::rule1(pe0, pe1, ce0, ce1, de0, de1, ve[R - 1]);
            vo[R - 1] = BitEnc::rule1(po0, po1, co0, co1, do0, do1, vo[R - 1]);
        }
    }
    // window rows [K, NW*R - K) are the tile's owned rows [ty*T, ty*T + T);
    // this wave's share of them (a half-height tile's ghost rows may span more
    // than one wave: K > R)
    const int r0 = min(max(K - wi * R, 0), R), r1 = min(max(NW * R - K - wi * R, 0), R);
    // Which lanes store, recomputed here from the lane id (the empty asm
    // makes it a fresh value): nothing per-lane but voff and the window lives
    // across the generation loop.  Extra live state there (the deep-halo
    // apron-pair test kept the 64-bit column index alive) made the compiler
    // issue each row's ds_bpermute right before its use and cost 2-8 % of the
    // launch (tests/test_isa.py).  The apron pairs of a
    // deep-halo pass (Extend::x) exist only on a partitioned x axis.
    int lane2 = (int)(threadIdx.x & 63);
    asm volatile("" : "+v"(lane2));
    const int gl2 = BAND ? lane2 >> gsh : 0;
    const int pin2 = BAND ? lane2 & ((1 << gsh) - 1) : lane2;
    const int64_t j2 = tx * 62 + pin2 - 1;
    const bool st = (BAND ? (pin2 >= 1 && pin2 <= (1 << gsh) - 2 && j2 < a.W && gl2 < nb)
                          : (lane2 >= 1 && lane2 <= 62 && j2 < a.W)) ||
                    (!WRAPX && a.xext && (!BAND || gl2 < nb) && (j2 == -1 || j2 == a.W));
    const int64_t yb = y0 + (BAND ? (int64_t)(gl2 < nb ? gl2 : 0) * T : 0);  // this lane's band
    const int64_t ylim = yend >= 0 ? yend : a.h;  // half tiles of a region stop at its last row
    uint8_t *q = out + (a.ya + yb + r0) * a.pitch + voff;
#pragma unroll
    for (int r = 0; r < R; ++r) {
        if (r < r0 || r >= r1) continue;
        if (st && yb + r < ylim) {
            const uint64_t v = (uint64_t)ve[r] | ((uint64_t)vo[r] << 32);
            if (FLOW == 1)
                __hip_atomic_store(reinterpret_cast<uint64_t *>(q), v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            else
                *reinterpret_cast<uint64_t *>(q) = v;
        }
        q += a.pitch;
    }
}

// Waves per SIMD the byte tiles are compiled for (LIFE_BYTE_WPE, compile
// time, A/B): 4 = 2 tiles of 8 waves per CU (up to 128 VGPRs), 6 = 3 tiles
// (80 VGPRs: the load / compute / store phases of three tiles overlap).
#ifndef LIFE_BYTE_WPE
#define LIFE_BYTE_WPE 4
#endif
#ifndef LIFE_BYTE_LOAD_CHUNK
#define LIFE_BYTE_LOAD_CHUNK 0
#endif
// LIFE_BYTE_BP_AHEAD: the generation loop's left-neighbour permutes are
// issued this many rows ahead of their use, the rows fenced in program order
// (LIFE_BYTE_BP_FENCE; unfenced, the compiler sinks every permute next to
// its use and waits for it).  A tile spends 33 us loading, 93 us in its
// generations, 4 us storing (scripts/wg_trace.py, profiles/r04/byte_ab):
// 2 ahead measured 2.29-2.30 against 2.33-2.36 ms per 32-generation launch
// (4 ahead 2.32, profiles/r04/byte_ab).
#ifndef LIFE_BYTE_BP_AHEAD
#define LIFE_BYTE_BP_AHEAD 2
#endif
#ifndef LIFE_BYTE_BP_FENCE
#define LIFE_BYTE_BP_FENCE 1
#endif
// Byte tiles: lane l of a tile holds word column 62 tx + l - 1 -- 32 byte
// cells, packed into one register word per row by v_dot4_u32_u8 on load
// (two 16-B loads) and unpacked on store -- in the drifting frame
// (bit_hsum_drift: left neighbour only, 12 VALU + 1 LDS per row and
// generation; +2 % over the centred frame for bytes,
// profiles/r01/drift_ab.jsonl).  GK ghost rows per window end, compile-time
// (a runtime depth measured 29 % slower here, profiles/r02/ghost_ab.txt).
// The same window / exchange / barrier scheme as the bit tiles.
template <int R, int GK, bool WRAPX, bool WRAPY, int NW>
__device__ __forceinline__ void tile_body_byte(const TArgs &a, const uint8_t *in, uint8_t *out, int64_t tx,
                                               int64_t ty, Xch<NW> &xch) {
    static_assert(R >= 3 && GK >= 1 && GK <= 32, "window");
    constexpr int K = GK;
    constexpr int T = NW * R - 2 * K;
    const int lane = threadIdx.x & 63;
    const int laddr = ((lane - 1) & 63) << 2;
    const int wi = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int64_t j = tx * 62 + lane - 1;  // word column of this lane
    int64_t jl;
    if (WRAPX) {
        if (LIFE_FAST_WRAP && a.W >= 64) {  // j in [-1, W + 62), as tile_body_bit
            jl = j < 0 ? j + a.W : (j >= a.W ? j - a.W : j);
        } else {
            jl = j % a.W;
            if (jl < 0) jl += a.W;
        }
    } else {
        jl = j > a.W ? a.W : j;
    }
    const uint32_t voff = (uint32_t)(a.xoff + 32 * jl);
    const int64_t y0 = ty * T - K + (int64_t)wi * R;
    const uint8_t *row0 = in + a.ya * a.pitch;
    uint32_t v[R];
    {
        int64_t y = y0;
        if (WRAPY) {
            if (LIFE_FAST_WRAP && a.h >= 2 * (int64_t)(NW * R) + 64) {  // y in [-K, h + T)
                y = y < 0 ? y + a.h : (y >= a.h ? y - a.h : y);
            } else {
                y %= a.h;
                if (y < 0) y += a.h;
            }
        }
        const uint8_t *p = row0 + y * a.pitch;
#pragma unroll
        for (int r = 0; r < R; ++r) {
            // LIFE_BYTE_LOAD_CHUNK rows of loads in flight at most: a
            // scheduling fence after every chunk keeps the load phase's
            // registers (8 per row in flight) inside the occupancy budget
            if (LIFE_BYTE_LOAD_CHUNK > 0 && r > 0 && r % (LIFE_BYTE_LOAD_CHUNK > 0 ? LIFE_BYTE_LOAD_CHUNK : 1) == 0)
                __builtin_amdgcn_sched_barrier(0);
            const uint4 *q = reinterpret_cast<const uint4 *>(p + voff);
            v[r] = pack32(q[0], q[1]);
            ++y;
            if (WRAPY && y == a.h) {
                y = 0;
                p = row0;
            } else {
                p += a.pitch;
            }
        }
    }
    for (int g = 0; g < a.m; ++g) {
        const int par = g & 1;
        uint32_t t0, t1, b0, b1, tL, bL;  // xL: the row's own cells in the drifting frame
        bit_hsum_drift(v[0], laddr, t0, t1, tL);
        bit_hsum_drift(v[R - 1], laddr, b0, b1, bL);
        xch[par][wi][0][lane] = t0;
        xch[par][wi][1][lane] = t1;
        xch[par][wi][2][lane] = b0;
        xch[par][wi][3][lane] = b1;
        __syncthreads();
        if (g == 0) wg_trace(1);  // window loaded, first generation's sums published
        uint32_t a0 = 0u, a1 = 0u, d0 = 0u, d1 = 0u;
        if (wi > 0) {
            a0 = xch[par][wi - 1][2][lane];
            a1 = xch[par][wi - 1][3][lane];
        }
        if (wi < NW - 1) {
            d0 = xch[par][wi + 1][0][lane];
            d1 = xch[par][wi + 1][1][lane];
        }
        uint32_t p0 = t0, p1 = t1, c0, c1, cL;
        bit_hsum_drift(v[1], laddr, c0, c1, cL);
        const uint32_t h10 = c0, h11 = c1;
        // LIFE_BYTE_BP_AHEAD rows' left-neighbour words in flight ahead of
        // their use (0: each fetched in its own row)
        constexpr int AH = LIFE_BYTE_BP_AHEAD;
        uint32_t ahead[AH > 0 ? AH : 1];
#pragma unroll
        for (int k = 0; k < AH; ++k)
            if (2 + k < R - 1) ahead[k] = bperm(laddr, v[2 + k]);
#pragma unroll
        for (int r = 1; r < R - 1; ++r) {
            uint32_t n0, n1, nL;
            if (r + 1 == R - 1) {
                n0 = b0;
                n1 = b1;
                nL = bL;
            } else if (AH > 0) {
                const uint32_t l = ahead[0];
#pragma unroll
                for (int k = 0; k + 1 < AH; ++k) ahead[k] = ahead[k + 1];
                if (r + 1 + AH < R - 1) ahead[AH - 1] = bperm(laddr, v[r + 1 + AH]);
                // rows stay in program order: the compiler would otherwise
                // sink every permute next to its use again
                if (LIFE_BYTE_BP_FENCE) __builtin_amdgcn_sched_barrier(0);
                nL = __builtin_amdgcn_alignbit(v[r + 1], l, 31);
                BitEnc::fa(__builtin_amdgcn_alignbit(v[r + 1], l, 30), nL, v[r + 1], n0, n1);
            } else {
                bit_hsum_drift(v[r + 1], laddr, n0, n1, nL);
            }
            v[r] = BitEnc::rule1(p0, p1, c0, c1, n0, n1, cL);
            cL = nL;
            p0 = c0;
            p1 = c1;
            c0 = n0;
            c1 = n1;
        }
        v[R - 1] = BitEnc::rule1(p0, p1, b0, b1, d0, d1, bL);
        v[0] = BitEnc::rule1(a0, a1, t0, t1, h10, h11, tL);
    }
    wg_trace(2);  // generations done
    const int r0 = min(max(K - wi * R, 0), R), r1 = min(max(NW * R - K - wi * R, 0), R);
    const bool st = lane >= 1 && lane <= 62 && j < a.W;
    uint8_t *q = out + (a.ya + y0 + r0) * a.pitch + voff;
#pragma unroll
    for (int r = 0; r < R; ++r) {
        if (r < r0 || r >= r1) continue;
        v[r] = drift_realign(v[r], a.m);  // every lane: the bpermute reads lane + 1
        if (st && y0 + r < a.h) {
            uint4 *o = reinterpret_cast<uint4 *>(q);
            o[0] = unpack_half(v[r], 0);
            o[1] = unpack_half(v[r], 1);
        }
        q += a.pitch;
    }
    wg_trace(3);  // stores issued
}

// Waves per SIMD the bit tiles are compiled for (the VGPR budget): 3 tiles
// of 8 waves or 2 of 12 per CU at <= 80 VGPRs; 16-wave tiles: 2 per CU at 64
// (R = 16) or 1 at 128.
constexpr int bit_wpe(int NW, int R) { return NW == 16 ? (R <= 16 ? 8 : 4) : (R <= 24 ? 6 : 4); }

// Item i of the tail (TArgs::tail_*): RS rows per wave, tile rows of TS =
// NW RS - 2m owned rows from owned row tail_y, the last one stopping at
// tail_yend; tail_ntx - 1 ordinary tiles per tile row from column tail_tx0,
// then the banded items of the last tile column (B = 64 >> gsh tile rows
// each), or tail_ntx tiles per row without it.  (Round 5's half tiles spanned
// the last column as full-width tiles; banded they take (64 - o - 2) / 64
// fewer lanes there.)
template <int RS, bool WRAPX, bool WRAPY, int NW>
__device__ __forceinline__ void tail_item(const TArgs &a, int64_t i, XchB<NW> &xch) {
    const int64_t TS = (int64_t)NW * RS - 2 * a.m, y0 = a.tail_y, yend = a.tail_yend;
    const int64_t rows = (yend - y0 + TS - 1) / TS;
    const bool band = a.tail_band != 0;
    const int64_t ntxs = a.tail_ntx - (band ? 1 : 0), nfull = ntxs * rows;
    if (i < nfull) {
        tile_body_bit<RS, WRAPX, WRAPY, 0, NW>(a, a.in, a.out, a.tail_tx0 + i % ntxs, i / ntxs, xch, 6, 1, y0,
                                              yend);
    } else {
        const int64_t B = 64 >> a.gsh, ty = (i - nfull) * B;
        const int nb = (int)(rows - ty < B ? rows - ty : B);
        tile_body_bit<RS, WRAPX, WRAPY, 0, NW, true>(a, a.in, a.out, a.bcol, ty, xch, a.gsh, nb, y0, yend);
    }
}

// One workgroup per tile (or banded item / partial-height tail tile).
template <int R, bool WRAPX, bool WRAPY, int NW>
__global__ __launch_bounds__(64 * NW, bit_wpe(NW, R)) void tstep_bit_kernel(TArgs a) {
    __shared__ XchB<NW> xch;
    wg_trace(0);
    int64_t wg = blockIdx.x;
    if (wg < a.xcd_n) {
        // the dispatcher deals blocks round-robin over the 8 XCDs: XCD x runs
        // blocks 8k + x, here items first_x + k, so the tiles beside and below
        // a tile share its XCD's L2 (their common ghost rows and boundary
        // lines are fetched once); a bijection of [0, xcd_n)
        const int64_t n = a.xcd_n, x = wg & 7, k = wg >> 3, per = n >> 3, rem = n & 7;
        wg = (x < rem ? x * (per + 1) : rem * (per + 1) + (x - rem) * per) + k;
    }
    if (a.tail_ntx > 0 && wg >= a.tail_first) {
        tail_item<R / 2, WRAPX, WRAPY, NW>(a, wg - a.tail_first, xch);
        wg_trace(1);
        return;
    }
    const int64_t nwg = a.first[a.nreg];
    if (wg >= nwg) return;  // whole workgroup
    int k = 0;
    while (k + 1 < a.nreg && wg >= a.first[k + 1]) ++k;
    const int64_t wr = wg - a.first[k];
    const bool bands = a.gsh < 6 && a.tx1[k] == a.bcol + 1;
    const int64_t ntx = a.tx1[k] - a.tx0[k] - (bands ? 1 : 0);
    const int64_t nfull = ntx * (a.ty1[k] - a.ty0[k]);
    if (wr < nfull) {
        const int64_t tx = a.tx0[k] + wr % ntx, ty = a.ty0[k] + wr / ntx;
        tile_body_bit<R, WRAPX, WRAPY, 0, NW>(a, a.in, a.out, tx, ty, xch);
    } else {
        const int64_t B = 64 >> a.gsh, ty = a.ty0[k] + (wr - nfull) * B;
        const int nb = (int)(a.ty1[k] - ty < B ? a.ty1[k] - ty : B);
        tile_body_bit<R, WRAPX, WRAPY, 0, NW, true>(a, a.in, a.out, a.bcol, ty, xch, a.gsh, nb);
    }
    wg_trace(1);
}

template <int R, int GK, bool WRAPX, bool WRAPY, int NW>
__global__ __launch_bounds__(64 * NW, LIFE_BYTE_WPE) void tstep_byte_kernel(TArgs a) {
    __shared__ Xch<NW> xch;
    wg_trace(0);
    int64_t wg = blockIdx.x;
    if (wg < a.xcd_n) {  // per-XCD row-major runs, as tstep_bit_kernel
        const int64_t n = a.xcd_n, x = wg & 7, k = wg >> 3, per = n >> 3, rem = n & 7;
        wg = (x < rem ? x * (per + 1) : rem * (per + 1) + (x - rem) * per) + k;
    }
    const int64_t nwg = a.first[a.nreg];
    if (wg >= nwg) return;
    int k = 0;
    while (k + 1 < a.nreg && wg >= a.first[k + 1]) ++k;
    const int64_t wr = wg - a.first[k];
    const int64_t ntx = a.tx1[k] - a.tx0[k];
    const int64_t tx = a.tx0[k] + wr % ntx, ty = a.ty0[k] + wr / ntx;
    tile_body_byte<R, GK, WRAPX, WRAPY, NW>(a, a.in, a.out, tx, ty, xch);
}

// tflow_kernel: `passes` launches of the bit tiles (m generations each, both
// axes periodic inside one shard) as ONE persistent launch.  Workgroups pull
// work items (pass p, tile) in order from a queue head; a tile of pass p > 0
// starts once every tile whose rows its window reads -- tile rows ty-2..ty+2
// (a short last tile row lets a window reach two rows over), columns
// tx-1..tx+1, periodic -- has finished pass p-1, which also guarantees that no
// reader of the rows it overwrites (pass p-1 of the same tiles) is still
// running.  Pass p walks the tile rows from row p (mod nty), so the rows a
// tile waits for were pulled about a whole pass earlier: no pass boundary
// drains the chip (the per-launch ramp and tail of tstep_kernel, ~48 us).
// Deadlock-free without co-residency: an item waits only on items pulled
// before it, and a pulled item is running on a resident workgroup.
// Hand-off (MI355X_MICROARCH.md, inter-workgroup visibility, row 1): the
// window rows are loaded `sc1`; every storing wave waits vmcnt(0), then a
// workgroup barrier, then one lane stores the tile's pass count `sc1`; the
// polling wave's lanes read the flags `sc1`, a barrier, then every wave loads.
struct FArgs {
    TArgs t;                         // geometry, m; t.in / t.out: buffers of pass 0
    int64_t ntx, nty, items;         // items = passes * per_pass
    // BAND: the last tile column (t.bcol) as banded items of B = 64 >> t.gsh
    // tile rows; a pass is ngroups groups of B tile rows, each (ntx - 1) * B
    // ordinary items then one banded item (tile rows past nty: no-op items)
    int64_t per_pass, ngroups, B;
    unsigned int *head;              // queue head (zeroed before the launch), then an error word: 1 + the
                                     // last item whose dependency wait timed out (0: none)
    unsigned int *done;              // per tile: passes completed (zeroed before the launch)
};

// BAND (a last tile column owning o <= 30 pairs: 32768^2's 16, 16384^2's
// 8): that column runs as banded items, as tstep_bit_kernel does, instead of
// full-width tiles that waste (64 - o - 2) / 64 of their lanes.  Without it
// the instance has no banded code in its loop (the banded items cost the
// ordinary tiles 2.5 % there, code size in the persistent loop;
// profiles/r02/r2x).
template <int R, bool WRAPX, bool WRAPY, int FLOW, int NW, bool BAND = false>
__global__ __launch_bounds__(64 * NW, bit_wpe(NW, R)) void tflow_kernel(FArgs f) {
    __shared__ XchB<NW> xch;
    __shared__ unsigned int item_sh;
    const TArgs &a = f.t;
    const int64_t tiles = f.ntx * f.nty;
    const int lane = threadIdx.x & 63;
    unsigned int *prev_flag = nullptr;  // wave 0, lanes < prev_n: the finished item's tile counters
    unsigned int prev_val = 0;
    int prev_n = 0;
    int traced = 0;  // diagnostics builds: items 0..3 stamp pulled / dependencies met / stored
    wg_trace(0);
    for (;;) {
        // ONE thread-0 region per iteration, behind the barrier that closes
        // the previous item: publish that item (its stores were drained by
        // every wave before the barrier), then pull the next.  (Two thread-0
        // regions on either side of the loop's back edge were merged by the
        // compiler into a region that lanes 1..63 of wave 0 never wait for:
        // the workgroup then re-ran its item forever.)
        if (!BAND && threadIdx.x == 0) {
            if (prev_flag) {
                if (FLOW == 2) {
                    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
                    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
                }
                __hip_atomic_store(prev_flag, prev_val, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            }
            item_sh = atomicAdd(f.head, 1u);
        }
        if (BAND && threadIdx.x < 64) {  // one wave-0 region: a banded item publishes its nb tiles
            if (prev_n > 0) {
                if (FLOW == 2) {
                    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
                    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
                }
                if (lane < prev_n)
                    __hip_atomic_store(prev_flag + (int64_t)lane * f.ntx, prev_val, __ATOMIC_RELAXED,
                                       __HIP_MEMORY_SCOPE_AGENT);
            }
            if (lane == 0) item_sh = atomicAdd(f.head, 1u);
        }
        __syncthreads();
        // uniform: scalar registers, scalar arithmetic
        const uint32_t item = __builtin_amdgcn_readfirstlane(item_sh);
        if ((int64_t)item >= f.items) return;  // the whole workgroup leaves
        if (LIFE_WG_TRACE && traced < 4) wg_trace(1 + 3 * traced);
        const uint32_t ntx = (uint32_t)f.ntx, nty = (uint32_t)f.nty;
        uint32_t p;
        int64_t tx, ty;
        int nb = 1;  // tile rows of this item (a banded item: up to B)
        if (!BAND) {
            p = item / (uint32_t)tiles;
            const uint32_t k = item - p * (uint32_t)tiles, kr = k / ntx;
            tx = k - kr * ntx;
            ty = (kr + p) % nty;
        } else {
            p = item / (uint32_t)f.per_pass;
            const uint32_t k = item - p * (uint32_t)f.per_pass;
            const uint32_t nfull = ntx - 1, G1 = nfull * (uint32_t)f.B + 1u;
            const uint32_t g = k / G1, off = k - g * G1;
            const int64_t ty0 = (int64_t)((g + p) % (uint32_t)f.ngroups) * f.B;  // groups rotate per pass
            if (off < nfull * (uint32_t)f.B) {
                tx = off % nfull;
                ty = ty0 + off / nfull;
            } else {
                tx = a.bcol;
                ty = ty0;
                nb = (int)(f.nty - ty0 < f.B ? f.nty - ty0 : f.B);
            }
            if (ty >= f.nty) {  // a padding item of the last group
                prev_n = 0;
                prev_flag = nullptr;
                __syncthreads();  // item_sh is rewritten by the next pull
                continue;
            }
        }
        if (p > 0 && threadIdx.x < 64) {
            // tile rows ty-2 .. ty+nb+1 x columns tx-1..tx+1 (one lane each)
            bool ok = true;
            const unsigned int *flag = nullptr;
            if (lane < 3 * (nb + 4)) {
                const int64_t dy = lane / 3 - 2, dx = lane % 3 - 1;
                int64_t yy = (ty + dy) % f.nty, xx = (tx + dx) % f.ntx;
                if (yy < 0) yy += f.nty;
                if (xx < 0) xx += f.ntx;
                flag = f.done + yy * f.ntx + xx;
            }
            // bounded: a wait of ~seconds means a broken invariant; record it
            // (the host reports it at the next sync) rather than hang the GPU
            for (uint32_t spin = 0;; ++spin) {
                if (flag)
                    ok = __hip_atomic_load(const_cast<unsigned int *>(flag), __ATOMIC_RELAXED,
                                           __HIP_MEMORY_SCOPE_AGENT) >= p;
                if (__all(ok)) break;
                if (spin == (1u << 20)) {
                    if (lane == 0) atomicMax(f.head + 1, item + 1);
                    break;
                }
                __builtin_amdgcn_s_sleep(2);
            }
            if (FLOW == 2) {  // plain producer stores: the valid form needs the acquire
                __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
                asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            }
        }
        __syncthreads();
        if (LIFE_WG_TRACE && traced < 4) wg_trace(2 + 3 * traced);
        const uint8_t *in = (p & 1) ? a.out : a.in;
        uint8_t *out = const_cast<uint8_t *>((p & 1) ? a.in : a.out);
        if (BAND && tx == a.bcol)
            tile_body_bit<R, WRAPX, WRAPY, FLOW, NW, true>(a, in, out, tx, ty, xch, a.gsh, nb);
        else
            tile_body_bit<R, WRAPX, WRAPY, FLOW, NW>(a, in, out, tx, ty, xch);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this wave's stores have left
        __syncthreads();
        if (LIFE_WG_TRACE && traced < 4) wg_trace(3 + 3 * traced++);
        prev_flag = f.done + ty * f.ntx + tx;
        prev_val = p + 1;
        prev_n = nb;
    }
}

// Natural 32-cell word j of a bit-encoded row (bit k = cell 32j + k) from
// the pair layout and back: the even / odd halves are 16-bit halves of the
// pair's E / O dwords.  Small-grid kernels work in natural words inside the
// CU and convert once per launch.
__device__ __forceinline__ uint32_t load_nat32(const uint8_t *row, int64_t j) {
    const uint16_t *h = reinterpret_cast<const uint16_t *>(row) + 4 * (j >> 1) + (j & 1);
    return nat32(h[0], h[2]);
}
__device__ __forceinline__ void store_nat32(uint8_t *row, int64_t j, uint32_t x) {
    uint16_t *h = reinterpret_cast<uint16_t *>(row) + 4 * (j >> 1) + (j & 1);
    h[0] = (uint16_t)compact16(x);
    h[2] = (uint16_t)compact16(x >> 1);
}

// ------------------------------------------------------------------ small grids
// LDS-resident stencil for a grid that fits one CU (configs[1]: p46gun_big,
// 500^2): one 1024-thread workgroup imports the shard into LDS as bits
// (W = ceil(w/32) words per row, two h x W buffers), runs G generations with
// one barrier each, and exports the result in the shard's own encoding.  No
// HBM traffic and no launch per generation: the per-generation cost is
// ~1-2k cycles of one CU instead of a full-chip launch.  Both axes wrap
// inside the shard (single-shard grids only); a width that is not a
// multiple of 32 is wrapped by the same patching as WRAPX.
constexpr int kSmallThreads = 1024;

struct SArgs {
    const uint8_t *in;
    uint8_t *out;
    int64_t pitch, xoff, ya;
    int32_t w, h, W, gens, bit;
};

__global__ __launch_bounds__(kSmallThreads) void small_kernel(SArgs a) {
    extern __shared__ __attribute__((aligned(16))) uint32_t lds[];
    const int W = a.W, h = a.h, w = a.w, n = W * h;
    uint32_t *A = lds, *B = lds + n;
    const int t = threadIdx.x;
    const int q = w - 32 * (W - 1);                   // valid bits in the last word: 1..32
    const uint32_t lastmask = q == 32 ? 0xFFFFFFFFu : ((1u << q) - 1u);
    // import: one word per thread-iteration
    for (int i = t; i < n; i += kSmallThreads) {
        const int y = i / W, j = i % W;
        const uint8_t *row = a.in + (int64_t)(y + a.ya) * a.pitch + a.xoff;
        uint32_t v = 0;
        if (a.bit) {
            v = load_nat32(row, j);
        } else {
            for (int k = 0; k < 32 && 32 * j + k < w; ++k) v |= (uint32_t)(row[32 * j + k] != 0) << k;
        }
        A[i] = j == W - 1 ? v & lastmask : v;
    }
    __syncthreads();
    // thread -> (word column j, rows [y0, y1))
    const int groups = kSmallThreads / W;  // W <= 1024 is checked on the host
    const int j = t % W, g = t / W;
    const int R = (h + groups - 1) / groups;
    const int y0 = g < groups ? g * R : h, y1 = min(h, y0 + R);
    const int jl = j == 0 ? W - 1 : j - 1, jr = j == W - 1 ? 0 : j + 1;
    const uint32_t lshift = j == 0 ? 31u - (uint32_t)((w - 1) & 31) : 0u;  // bit of cell w-1 -> bit 31
    const bool last = j == W - 1;
    for (int gen = 0; gen < a.gens; ++gen) {
        if (y0 < y1) {
            auto hsum = [&](int y, uint32_t &s0, uint32_t &s1, uint32_t &c) {
                y = y < 0 ? y + h : (y >= h ? y - h : y);
                const uint32_t *r = A + y * W;
                c = r[j];
                uint32_t lw = r[jl] << lshift;
                uint32_t rw = r[jr];
                uint32_t cc = c;
                if (last) {  // the cell right of w-1 is cell 0
                    if (q < 32)
                        cc = (cc & lastmask) | ((rw & 1u) << q);
                }
                const uint32_t L = __builtin_amdgcn_alignbit(cc, lw, 31);
                const uint32_t Rr = __builtin_amdgcn_alignbit(rw, cc, 1);
                BitEnc::fa(L, cc, Rr, s0, s1);
            };
            uint32_t p0, p1, c0, c1, n0, n1, cp, cc, cn;
            hsum(y0 - 1, p0, p1, cp);
            hsum(y0, c0, c1, cc);
            for (int y = y0; y < y1; ++y) {
                hsum(y + 1, n0, n1, cn);
                const uint32_t v = BitEnc::rule1(p0, p1, c0, c1, n0, n1, cc);
                B[y * W + j] = last ? v & lastmask : v;
                p0 = c0;
                p1 = c1;
                c0 = n0;
                c1 = n1;
                cc = cn;
            }
        }
        __syncthreads();
        uint32_t *tmp = A;
        A = B;
        B = tmp;
    }
    // export into the shard's encoding (owned cells only)
    for (int i = t; i < n; i += kSmallThreads) {
        const int y = i / W, jj = i % W;
        uint8_t *row = a.out + (int64_t)(y + a.ya) * a.pitch + a.xoff;
        const uint32_t v = A[i];
        if (a.bit) {
            store_nat32(row, jj, v);
        } else {
            for (int k = 0; k < 32 && 32 * jj + k < w; ++k) row[32 * jj + k] = (uint8_t)((v >> k) & 1u);
        }
    }
}

// ------------------------------------------------------- small grids, in VGPRs
// Register-resident variant of the small-grid path (configs[1] p46gun_big
// 500^2).  One 1024-lane workgroup holds the whole grid in VGPRs: a wave is
// split into 64/Wp lane groups (Wp = W rounded up to a power of two), each
// group owns a strip of R consecutive rows, one word column per lane; the
// grid is ns = h/R strips (R divides h, so every strip is full).  Per
// generation a lane computes the 2-bit horizontal sums of its R rows
// (neighbour words by ds_bpermute inside the group, periodic in x),
// publishes the sums of its first and last row in LDS, one barrier, reads the
// strip above's last / the strip below's first sums (periodic in y), and
// applies the rule to its R rows.  PATCH (w % 32 != 0): the x wrap crosses a
// partial word, so cell w-1 is moved to bit 31 of word 0's left word and
// cell 0 is put at bit q of the last word before the sums.
//
// WIN (windowed, several CUs): workgroup b owns rows [b*own, b*own + own) and
// holds the window of ns*R = own + 2K rows starting K rows above them (y
// periodic); the strips at the window's top and bottom take zeros from
// outside, so after m <= K generations rows [K, K + own) of the window are
// exact and only those are stored (in != out; the host runs ceil(gens / K)
// launches, swapping buffers).  ceil(h / own) workgroups instead of one.
constexpr int kRegThreads = 1024;
constexpr int kRegMaxW = 64;

struct RArgs {
    const uint8_t *in;
    uint8_t *out;
    int64_t pitch, xoff, ya;
    int32_t w, h, W, lgWp, gens, bit, ns;
    int32_t own, K;  // WIN: owned rows per workgroup, halo rows above/below
    // WIN, the launches of one call: 1 = the buffer holds natural 32-cell
    // words (bit k = cell 32j + k at row + xoff + 4j) instead of the shard's
    // encoding -- every launch but the first reads them, every launch but the
    // last writes them (no pair (de)interleave or byte (un)packing between
    // launches)
    int32_t nat_in, nat_out;
};

// ROT16 (W == Wp == 16, rows of 481..512 cells, e.g. p46gun_big): a lane
// group is exactly one 16-lane DPP row, so the periodic neighbour words come
// from DPP row rotates on the VALU instead of two ds_bpermute round trips
// through the LDS pipe per row and generation.
template <int R, bool PATCH, bool WIN, bool ROT16 = false>
__global__ __launch_bounds__(kRegThreads) void rsmall_kernel(RArgs a) {
    // [parity][top s0/s1, bottom s0/s1][thread]; WIN: 64 zero slots behind the
    // threads stand for the rows outside the window
    __shared__ uint32_t xch[2][4][kRegThreads + (WIN ? 64 : 0)];
    const int t = threadIdx.x;
    if (WIN && t < 64)
        for (int q = 0; q < 8; ++q) xch[q >> 2][q & 3][kRegThreads + t] = 0u;  // ordered by the first barrier
    const int Wp = 1 << a.lgWp, W = a.W;
    const int j = t & (Wp - 1);  // word column
    const int st = t >> a.lgWp;  // strip
    const bool active = st < a.ns && j < W;
    const int base = (t & 63) & ~(Wp - 1);  // first lane of this lane group
    const int jl = j == 0 ? W - 1 : j - 1, jr = j + 1 >= W ? 0 : j + 1;
    const int addr_l = (base + jl) << 2, addr_r = (base + jr) << 2;
    const int q = a.w - 32 * (W - 1);  // valid cells in the last word: 1..32
    const bool last = j == W - 1;
    const uint32_t keep = (last && q < 32) ? (1u << q) - 1u : 0xFFFFFFFFu;
    const uint32_t lsh = j == 0 ? (uint32_t)((32 - q) & 31) : 0u;  // cell w-1 -> bit 31
    const uint32_t qs = (uint32_t)(q & 31);
    const int sa = st == 0 ? a.ns - 1 : st - 1, sb = st + 1 >= a.ns ? 0 : st + 1;
    int ta = ((sa << a.lgWp) + j) & (kRegThreads - 1), tb = ((sb << a.lgWp) + j) & (kRegThreads - 1);
    if (WIN) {
        if (st == 0) ta = kRegThreads + (j & 63);
        if (st + 1 >= a.ns) tb = kRegThreads + (j & 63);
    }
    const int y0 = st * R;
    // WIN: owned row of window row 0 (may be negative: periodic in y)
    const int64_t wy = WIN ? (int64_t)blockIdx.x * a.own - a.K : 0;

    uint32_t v[R];
#pragma unroll
    for (int r = 0; r < R; ++r) {
        uint32_t x = 0;
        if (active) {
            int64_t gy = y0 + r;
            if (WIN) {
                gy = (wy + gy) % a.h;
                if (gy < 0) gy += a.h;
            }
            const uint8_t *row = a.in + (gy + a.ya) * a.pitch + a.xoff;
            if (WIN && a.nat_in) {
                x = reinterpret_cast<const uint32_t *>(row)[j];
            } else if (a.bit) {
                x = load_nat32(row, j);
            } else {
                for (int k = 0; k < 32 && 32 * j + k < a.w; ++k) x |= (uint32_t)(row[32 * j + k] != 0) << k;
            }
        }
        v[r] = x;
    }
    auto hsum = [&](uint32_t c, uint32_t &s0, uint32_t &s1) {
        uint32_t l;
        uint32_t rw;
        if (ROT16) {
            l = (uint32_t)__builtin_amdgcn_mov_dpp((int)c, 0x121, 0xf, 0xf, false);   // row_ror:1 -> lane j-1
            rw = (uint32_t)__builtin_amdgcn_mov_dpp((int)c, 0x12F, 0xf, 0xf, false);  // row_ror:15 -> lane j+1
        } else {
            l = bperm(addr_l, c);
            rw = bperm(addr_r, c);
        }
        if (PATCH) {
            l <<= lsh;
            // (c & keep) | (rw << qs & ~keep): the last word gets cell 0 at bit q (above it: don't-care)
            c = b3<((0xF0 & 0xCC) | (~0xCC & 0xAA)) & 0xFF>(c, keep, rw << qs);
        }
        BitEnc::fa(__builtin_amdgcn_alignbit(c, l, 31), c, __builtin_amdgcn_alignbit(rw, c, 1), s0, s1);
    };
    for (int g = 0; g < a.gens; ++g) {
        const int par = g & 1;
        uint32_t h0[R], h1[R];
        hsum(v[0], h0[0], h1[0]);
        if (R > 1) hsum(v[R - 1], h0[R - 1], h1[R - 1]);
        xch[par][0][t] = h0[0];
        xch[par][1][t] = h1[0];
        xch[par][2][t] = h0[R - 1];
        xch[par][3][t] = h1[R - 1];
        __syncthreads();
        const uint32_t a0 = xch[par][2][ta], a1 = xch[par][3][ta];
        const uint32_t d0 = xch[par][0][tb], d1 = xch[par][1][tb];
#pragma unroll
        for (int r = 1; r < R - 1; ++r) hsum(v[r], h0[r], h1[r]);
#pragma unroll
        for (int r = 1; r < R - 1; ++r)
            v[r] = BitEnc::rule1(h0[r - 1], h1[r - 1], h0[r], h1[r], h0[r + 1], h1[r + 1], v[r]);
        if (R == 1) {
            v[0] = BitEnc::rule1(a0, a1, h0[0], h1[0], d0, d1, v[0]);
        } else {
            v[0] = BitEnc::rule1(a0, a1, h0[0], h1[0], h0[1], h1[1], v[0]);
            v[R - 1] = BitEnc::rule1(h0[R - 2], h1[R - 2], h0[R - 1], h1[R - 1], d0, d1, v[R - 1]);
        }
    }
    if (!active) return;
#pragma unroll
    for (int r = 0; r < R; ++r) {
        int64_t gy = y0 + r;
        if (WIN) {
            // window rows [K, K + own) that exist
            if (gy < a.K || gy >= a.K + a.own || wy + gy >= a.h) continue;
            gy += wy;
        }
        uint8_t *row = a.out + (gy + a.ya) * a.pitch + a.xoff;
        const uint32_t x = v[r] & keep;
        if (WIN && a.nat_out) {
            reinterpret_cast<uint32_t *>(row)[j] = x;
        } else if (a.bit) {
            store_nat32(row, j, x);
        } else {
            for (int k = 0; k < 32 && 32 * j + k < a.w; ++k) row[32 * j + k] = (uint8_t)((x >> k) & 1u);
        }
    }
}

// Strip heights with a kernel instance: the smallest that divides h and
// gives at most kRegThreads / Wp strips is used.
constexpr int kRegRows[] = {1, 2, 3, 4, 5, 6, 8, 10, 12, 16, 20, 25, 32};

template <bool PATCH, bool WIN>
hipError_t launch_rs(const RArgs &a, int R, unsigned blocks, hipStream_t s) {
    // only the waves that own strips (the barrier counts the launched waves)
    const unsigned threads = (unsigned)((((int64_t)a.ns << a.lgWp) + 63) / 64 * 64);
    if (WIN && R == 1 && a.W == 16 && a.lgWp == 4) {  // the automatic window shape, 16-word rows
        rsmall_kernel<1, PATCH, WIN, true><<<blocks, threads, 0, s>>>(a);
        return hipGetLastError();
    }
    switch (R) {
#define LIFE_RS(N) \
    case N: rsmall_kernel<N, PATCH, WIN><<<blocks, threads, 0, s>>>(a); break;
        LIFE_RS(1) LIFE_RS(2) LIFE_RS(3) LIFE_RS(4) LIFE_RS(5) LIFE_RS(6) LIFE_RS(8) LIFE_RS(10) LIFE_RS(12)
        LIFE_RS(16) LIFE_RS(20) LIFE_RS(25) LIFE_RS(32)
#undef LIFE_RS
    default: return hipErrorInvalidValue;
    }
    return hipGetLastError();
}

// ------------------------------------------------------------------ cell access
// Byte: cell x of a padded row at row[xoff + x].  Bit: the pair layout
// (life_bitops.h): bit pair_bit(x) of dword pair_dword(x) counted from
// row + xoff (x may be negative: the left apron).
__device__ __forceinline__ uint32_t get_cell(const uint8_t *row, int64_t xoff, int64_t x, bool bit) {
    if (!bit) return row[xoff + x];
    const uint32_t *w = reinterpret_cast<const uint32_t *>(row + xoff);
    return (w[pair_dword(x)] >> pair_bit(x)) & 1u;
}
__device__ __forceinline__ void set_cell(uint8_t *row, int64_t xoff, int64_t x, uint32_t v, bool bit) {
    if (!bit) {
        row[xoff + x] = (uint8_t)v;
        return;
    }
    uint32_t *w = reinterpret_cast<uint32_t *>(row + xoff) + pair_dword(x);
    const uint32_t m = 1u << pair_bit(x);
    *w = (*w & ~m) | (v ? m : 0u);
}

// Column halo staging.  Cell columns (xapron == 1): one byte 0/1 per row.
// Temporal layouts: the bit encoding's x-apron is one pair (64 cells, 8 B
// per row and side, sent in pair form), the byte encoding's 32 byte cells.
// The left column (cells [0, 64)) is pair 0; the right one (cells [w-64,
// w)) and the right apron (cells [w, w+64)) straddle two pairs when w % 64 !=
// 0: they go through the natural 64-bit order (nat64 / pair_of), a funnel
// shift on the way out, a merge that keeps the owned cells on the way in.
__device__ __forceinline__ uint64_t pair_nat(const uint32_t *wd, int64_t p) { return nat64(wd[2 * p], wd[2 * p + 1]); }
__device__ __forceinline__ void put_pair(uint32_t *wd, int64_t p, uint64_t v) {
    const uint2 q = pair_of(v);
    wd[2 * p] = q.x;
    wd[2 * p + 1] = q.y;
}
__device__ __forceinline__ uint64_t right_column_bits(const uint32_t *wd, int64_t w) {  // cells [w-64, w), w >= 64
    const int64_t x = w - 64, p = x >> 6;
    const uint32_t s = (uint32_t)(x & 63);
    if (s == 0) return pair_nat(wd, p);
    return (pair_nat(wd, p) >> s) | (pair_nat(wd, p + 1) << (64 - s));
}
__device__ __forceinline__ void put_right_apron_bits(uint32_t *wd, int64_t w, uint64_t v) {  // cells [w, w+64)
    const int64_t p = w >> 6;
    const uint32_t s = (uint32_t)(w & 63);
    if (s == 0) {
        put_pair(wd, p, v);
        return;
    }
    const uint64_t keep = (1ull << s) - 1ull;  // the owned cells of the partial pair
    put_pair(wd, p, (pair_nat(wd, p) & keep) | (v << s));
    put_pair(wd, p + 1, v >> (64 - s));  // cells beyond w+63: never read as owned
}
__device__ __forceinline__ void copy32(uint8_t *dst, const uint8_t *src) {
    // byte-cell columns need not be 4-byte aligned (w % 4 != 0)
    for (int k = 0; k < 32; ++k) dst[k] = src[k];
}

// Threads [h, h + 4K) of a corner exchange (temporal layouts, K = ya): the
// owned row a send-slot corner c comes from -- c = 0, 1 (SE, SW): the bottom
// K rows; c = 2, 3 (NE, NW): the top K -- and whether it is the right
// column (c even) or pair 0 / the first 32 cells (c odd).  The receive slot
// c lands in apron row -K + r (c = 0, 1) or h + r (c = 2, 3), x-apron left
// (c even) or right (c odd).
__global__ void pack_columns_kernel(const uint8_t *buf, int64_t pitch, int64_t ya, int64_t xoff, int64_t w,
                                    int64_t h, int64_t xa, uint8_t *stage, bool bit, int64_t nc) {
    int64_t y = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (y >= h + nc) return;
    bool right = true, left = true;  // columns: both (slot y and slot h + y)
    int64_t out = y, lo = h + y;     // the stage entries of the right column and of pair 0 / cells [0, 32)
    if (y >= h) {                    // corner c, row r: one entry
        const int64_t c = (y - h) / ya, r = (y - h) % ya;
        out = lo = y + h;  // entries 2h + cK + r
        right = (c & 1) == 0;
        left = !right;
        y = c < 2 ? h - ya + r : r;
    }
    const uint8_t *row = buf + (y + ya) * pitch;
    if (xa == 64 && bit) {
        const uint32_t *wd = reinterpret_cast<const uint32_t *>(row + xoff);
        uint64_t *st = reinterpret_cast<uint64_t *>(stage);
        if (right) {
            const uint2 r = pair_of(right_column_bits(wd, w));
            st[out] = (uint64_t)r.x | ((uint64_t)r.y << 32);
        }
        if (left) st[lo] = *reinterpret_cast<const uint64_t *>(wd);  // pair 0
        return;
    }
    if (xa == 32) {  // 32 byte cells per row and side
        if (right) copy32(stage + 32 * out, row + xoff + w - 32);
        if (left) {
            const uint4 *l = reinterpret_cast<const uint4 *>(row + xoff);
            uint4 *st = reinterpret_cast<uint4 *>(stage + 32 * lo);
            st[0] = l[0];
            st[1] = l[1];
        }
        return;
    }
    stage[y] = (uint8_t)get_cell(row, xoff, w - 1, bit);
    stage[h + y] = (uint8_t)get_cell(row, xoff, 0, bit);
}

__global__ void unpack_columns_kernel(uint8_t *buf, int64_t pitch, int64_t ya, int64_t xoff, int64_t w,
                                      int64_t h, int64_t xa, const uint8_t *stage, bool bit, int64_t nc) {
    int64_t y = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (y >= h + nc) return;
    bool left = true, right = true;  // columns: slot y -> left apron, slot h + y -> right apron
    int64_t in = y, ri = h + y;
    if (y >= h) {  // corner c, row r: apron rows -K + r (c < 2) or h + r, left apron for even c
        const int64_t c = (y - h) / ya, r = (y - h) % ya;
        in = ri = y + h;
        left = (c & 1) == 0;
        right = !left;
        y = c < 2 ? r - ya : h + r;
    }
    uint8_t *row = buf + (y + ya) * pitch;
    if (xa == 64 && bit) {
        uint32_t *wd = reinterpret_cast<uint32_t *>(row + xoff);
        const uint64_t *st = reinterpret_cast<const uint64_t *>(stage);
        if (left) reinterpret_cast<uint64_t *>(wd)[-1] = st[in];  // pair -1 = cells [-64, 0)
        if (right) {
            const uint64_t r = st[ri];
            put_right_apron_bits(wd, w, nat64((uint32_t)r, (uint32_t)(r >> 32)));
        }
        return;
    }
    if (xa == 32) {
        if (left) {
            uint4 *l = reinterpret_cast<uint4 *>(row + xoff - 32);
            const uint4 *st = reinterpret_cast<const uint4 *>(stage + 32 * in);
            l[0] = st[0];
            l[1] = st[1];
        }
        if (right) copy32(row + xoff + w, stage + 32 * ri);
        return;
    }
    set_cell(row, xoff, -1, stage[y] ? 1u : 0u, bit);
    set_cell(row, xoff, w, stage[h + y] ? 1u : 0u, bit);
}

// Periodic x inside one shard of a temporal layout whose width is not a
// multiple of the lane column (64 bit cells / 32 byte cells; the tiles' WRAPX
// reads whole lane columns): the shard is its own left and right neighbour,
// so the aprons are filled from its own columns.
__global__ void wrap_columns_kernel(uint8_t *buf, int64_t pitch, int64_t ya, int64_t xoff, int64_t w, int64_t h,
                                    bool bit) {
    const int64_t y = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (y >= h) return;
    uint8_t *row = buf + (y + ya) * pitch;
    if (bit) {
        uint32_t *wd = reinterpret_cast<uint32_t *>(row + xoff);
        const uint64_t l = pair_nat(wd, 0), r = right_column_bits(wd, w);
        put_pair(wd, -1, r);
        put_right_apron_bits(wd, w, l);
        return;
    }
    copy32(row + xoff - 32, row + xoff + w - 32);
    copy32(row + xoff + w, row + xoff);
}

// One thread per 16-byte unit of an owned row: dense (row pitch w) -> padded.
template <int CPU>  // cells per unit: 16 (byte) or 128 (bit)
__global__ void import_kernel(const uint8_t *dense, uint8_t *buf, int64_t pitch, int64_t ya, int64_t xoff,
                              int64_t w, int64_t h, int64_t units) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= units * h) return;
    const int64_t u = i % units, y = i / units;
    const uint8_t *in = dense + y * w;
    uint32_t word[4] = {0u, 0u, 0u, 0u};
    const int64_t x0 = u * CPU;
    for (int k = 0; k < CPU; ++k) {
        const int64_t x = x0 + k;
        if (x >= w) break;
        const uint32_t v = in[x] != 0;
        if (CPU == 16)
            word[k >> 2] |= v << (8 * (k & 3));
        else
            word[pair_dword(k)] |= v << pair_bit(k);  // a unit = two interleaved pairs
    }
    *reinterpret_cast<uint4 *>(buf + (y + ya) * pitch + xoff + 16 * u) =
        make_uint4(word[0], word[1], word[2], word[3]);
}

template <int CPU>
__global__ void export_kernel(const uint8_t *buf, uint8_t *dense, int64_t pitch, int64_t ya, int64_t xoff,
                              int64_t w, int64_t h, int64_t units) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= units * h) return;
    const int64_t u = i % units, y = i / units;
    const uint4 q = *reinterpret_cast<const uint4 *>(buf + (y + ya) * pitch + xoff + 16 * u);
    const uint32_t word[4] = {q.x, q.y, q.z, q.w};
    uint8_t *o = dense + y * w;
    const int64_t x0 = u * CPU;
    for (int k = 0; k < CPU; ++k) {
        const int64_t x = x0 + k;
        if (x >= w) break;
        o[x] = CPU == 16 ? (uint8_t)((word[k >> 2] >> (8 * (k & 3))) & 0xFFu)
                         : (uint8_t)((word[pair_dword(k)] >> pair_bit(k)) & 1u);
    }
}

// VTK CELL_DATA body of a block (life_save_vtk, life_cart.c:181-185: "%d\n"
// per cell, x fastest): 2 bytes per cell, '0'/'1' then '\n', row pitch 2w.
// One thread per 8 cells of a row (16 output bytes); 2-D grid, y strides rows.
__device__ __forceinline__ uint64_t vtk4(uint32_t cells4) {  // 4 cells, bit k -> ASCII pair k
    uint64_t v = 0;
#pragma unroll
    for (int k = 0; k < 4; ++k) v |= (uint64_t)(0x0A30u | ((cells4 >> k) & 1u)) << (16 * k);
    return v;
}
template <bool BIT>
__global__ void vtk_kernel(const uint8_t *buf, int64_t pitch, int64_t ya, int64_t xoff, int64_t w, int64_t h,
                           uint8_t *out) {
    const int64_t x0 = 8 * ((int64_t)blockIdx.x * blockDim.x + threadIdx.x);
    if (x0 >= w) return;
    const int n = w - x0 < 8 ? (int)(w - x0) : 8;
    const bool vec = (w & 7) == 0;  // 16-B aligned output rows
    for (int64_t y = blockIdx.y; y < h; y += gridDim.y) {
        const uint8_t *row = buf + (y + ya) * pitch + xoff;
        uint32_t c;  // cell k at bit k
        if (BIT) {
            // x0 is a multiple of 8: four even cells from E, four odd from O
            const uint32_t *wd = reinterpret_cast<const uint32_t *>(row) + 2 * (x0 >> 6);
            const uint32_t sh = (uint32_t)((x0 & 63) >> 1);
            c = nat32((wd[0] >> sh) & 15u, (wd[1] >> sh) & 15u);
        } else {
            c = 0;
            for (int k = 0; k < n; ++k) c |= (uint32_t)(row[x0 + k] & 1u) << k;
        }
        uint8_t *o = out + y * 2 * w + 2 * x0;
        if (vec && n == 8) {
            *reinterpret_cast<uint4 *>(o) = make_uint4((uint32_t)vtk4(c), (uint32_t)(vtk4(c) >> 32),
                                                       (uint32_t)vtk4(c >> 4), (uint32_t)(vtk4(c >> 4) >> 32));
        } else {
            for (int k = 0; k < n; ++k) {
                o[2 * k] = (uint8_t)('0' + ((c >> k) & 1u));
                o[2 * k + 1] = '\n';
            }
        }
    }
}

// Packed frame rows of a block (the driver's LIFEBITS checkpoint format:
// cell x of a row at bit (x & 7) of byte (x >> 3)).  The block starts at
// global column x0; with s = x0 & 7 its cells land at bits s.. of its first
// output byte, so output byte j holds block cells 8j - s .. 8j - s + 7 (those
// outside [0, w) are 0: the host ORs the bytes two blocks share).  One thread
// per output byte; 2-D grid, y strides rows.  Bit encoding: the pair(s)
// holding the byte's cells in natural order (nat64), then a funnel shift.
template <bool BIT>
__global__ void bits_kernel(const uint8_t *buf, int64_t pitch, int64_t ya, int64_t xoff, int64_t w, int64_t h,
                            int s, uint8_t *out, int64_t rb) {
    const int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (j >= rb) return;
    const int64_t c0 = 8 * j - s;  // block cell of bit 0 of this byte (>= -7)
    const uint32_t lo = c0 < 0 ? (uint32_t)(-c0) : 0u;                     // bits below: none
    const uint32_t hi = w - c0 >= 8 ? 8u : (uint32_t)(w - c0);            // bits at and above: none
    const uint32_t keep = ((1u << hi) - 1u) & ~((1u << lo) - 1u);
    for (int64_t y = blockIdx.y; y < h; y += gridDim.y) {
        const uint8_t *row = buf + (y + ya) * pitch + xoff;
        uint32_t v;
        if (BIT) {
            const uint32_t *wd = reinterpret_cast<const uint32_t *>(row);
            if (c0 < 0) {
                v = (uint32_t)pair_nat(wd, 0) << lo;
            } else {
                // the next pair is owned or x-apron / pitch padding: in-row
                const int64_t pp = c0 >> 6;
                const uint32_t sh = (uint32_t)(c0 & 63);
                uint64_t n = pair_nat(wd, pp) >> sh;
                if (sh > 56) n |= pair_nat(wd, pp + 1) << (64 - sh);
                v = (uint32_t)n;
            }
        } else {
            v = 0;
            for (uint32_t b = lo; b < hi; ++b) v |= (uint32_t)(row[c0 + b] & 1u) << b;
        }
        out[y * rb + j] = (uint8_t)(v & keep);
    }
}

__device__ __forceinline__ uint64_t splitmix64(uint64_t z) {
    z += 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

template <int CPU>
__global__ void fill_random_kernel(uint8_t *buf, int64_t pitch, int64_t ya, int64_t xoff, int64_t w, int64_t h,
                                   int64_t units, int64_t gx0, int64_t gy0, int64_t nx, uint64_t key,
                                   uint32_t thr) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= units * h) return;
    const int64_t u = i % units, y = i / units;
    uint32_t word[4] = {0u, 0u, 0u, 0u};
    const int64_t x0 = u * CPU;
    const uint64_t base = (uint64_t)((gy0 + y) * nx + gx0);
    for (int k = 0; k < CPU; ++k) {
        const int64_t x = x0 + k;
        if (x >= w) break;
        const uint32_t v = (uint32_t)(splitmix64(key ^ (base + (uint64_t)x)) >> 32) < thr;
        if (CPU == 16)
            word[k >> 2] |= v << (8 * (k & 3));
        else
            word[pair_dword(k)] |= v << pair_bit(k);
    }
    *reinterpret_cast<uint4 *>(buf + (y + ya) * pitch + xoff + 16 * u) =
        make_uint4(word[0], word[1], word[2], word[3]);
}

// Census of the owned cells: live count and the position-weighted checksum
// sum over live (x, y) of mix64(y*nx + x + 1), both mod 2^64 -- independent
// of the cell encoding and of the partition, so the 1-GPU and N-shard runs of
// one grid, and the byte and bit kernels, can be compared at sizes no host
// copy or CPU oracle reaches.  2-D grid: x over 16-B units, y strides rows.
__device__ __forceinline__ uint64_t cell_mix(uint64_t v) {
    v *= 0x9E3779B97F4A7C15ull;
    return v ^ (v >> 29);
}

template <int CPU>
__global__ void census_kernel(const uint8_t *buf, int64_t pitch, int64_t ya, int64_t xoff, int64_t w, int64_t h,
                              int64_t units, int64_t gx0, int64_t gy0, int64_t nx, unsigned long long *out) {
    const int64_t u = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    unsigned long long c = 0, sum = 0;
    constexpr int kPerWord = CPU / 4;  // cells per dword
    if (u < units) {
        const int64_t valid = w - u * CPU;  // cells of this unit inside the block
        uint32_t m[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            if (CPU == 16) {
                const int64_t left = valid - k * kPerWord;
                m[k] = left <= 0 ? 0u : left >= kPerWord ? 0xFFFFFFFFu : (0xFFFFFFFFu >> (32 - 8 * left));
            } else {  // dword k: cells 64 (k >> 1) + 2i + (k & 1), i < 32
                const int64_t n = (valid - 64 * (k >> 1) - (k & 1) + 1) >> 1;  // valid bits (floor; may be < 0)
                m[k] = n <= 0 ? 0u : n >= 32 ? 0xFFFFFFFFu : (0xFFFFFFFFu >> (32 - n));
            }
        }
        for (int64_t y = blockIdx.y; y < h; y += gridDim.y) {
            const uint4 q = *reinterpret_cast<const uint4 *>(buf + (y + ya) * pitch + xoff + 16 * u);
            const uint32_t word[4] = {q.x, q.y, q.z, q.w};
            const uint64_t base = (uint64_t)((gy0 + y) * nx + gx0 + u * CPU) + 1u;
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                uint32_t bits = word[k] & m[k];  // byte cells are 0/1: bit 8j = cell j of the dword
                c += __popc(bits);
                while (bits) {
                    const int b = __ffs(bits) - 1;
                    bits &= bits - 1u;
                    sum += cell_mix(base + (uint64_t)(CPU == 16 ? k * kPerWord + (b >> 3)
                                                                : 64 * (k >> 1) + 2 * b + (k & 1)));
                }
            }
        }
    }
    for (int s = 32; s > 0; s >>= 1) {
        c += __shfl_xor(c, s);
        sum += __shfl_xor(sum, s);
    }
    if ((threadIdx.x & 63) == 0) {
        if (c) atomicAdd(out, c);
        if (sum) atomicAdd(out + 1, sum);
    }
}

inline bool is_bit(const life_layout &L) { return L.kernel == LIFE_KERNEL_BIT; }
inline unsigned blocks_for(int64_t n, int b) { return (unsigned)((n + b - 1) / b); }

}  // namespace

namespace {
// Measured on MI355X at 65536^2 (scripts/tune.py, profiles/): byte R16/D8 the
// fastest of {16,32,64} x {2,4,8} once the strips are dealt to the XCDs in
// row-major runs (1.497 ms against 1.647 for the former R64/D2,
// profiles/r03/r5j tune_byte1.log); bit R16 with the whole strip in flight
// (D18) 1.7 % ahead of D8 (profiles/r03/r5b tune_bit1.log).
struct Tunings {
    StepTuning t[2];  // [0] byte, [1] bit
    // temporal tiles: register rows per wave, per encoding [byte (32-cell
    // words), bit (64-cell pairs)], and waves per bit tile workgroup
    // (window = waves x rows, tile = window - 2 ghost rows per end)
    int nr[2] = {48, 24};
    int nw_bit = 8;
    Tunings() : t{{16, 8}, {16, 18}} {
        for (StepTuning &v : t) {
            if (const char *e = getenv("LIFE_STEP_ROWS")) v.rows = atoi(e);
            if (const char *e = getenv("LIFE_STEP_DEPTH")) v.depth = atoi(e);
        }
        if (const char *e = getenv("LIFE_TEMPORAL_ROWS")) nr[1] = atoi(e);
        if (const char *e = getenv("LIFE_TEMPORAL_ROWS_BYTE")) nr[0] = atoi(e);
        if (const char *e = getenv("LIFE_TILE_WAVES")) nw_bit = atoi(e);
    }
};
Tunings &tunings() {
    static Tunings t;
    return t;
}
// Tile heights with a kernel instance.  Round 5 kept the shipped shapes and
// one alternative each: every other shape measured slower at 65536^2
// (profiles/r02/r2w, r03/r4g) and at 32768^2 (bit 32x8, 24x12, 16x16:
// 0.96-0.99 of 24x8, profiles/r05/a).
// (byte 64-row tiles, round 5: 61.3 vs 60.5 T at 65536^2, 48.1 vs 50.0 T at
// 32768^2 -- flat, removed; profiles/r05/g)
bool temporal_rows_ok(bool bit, int nr) { return bit ? (nr == 16 || nr == 24) : (nr == 32 || nr == 48); }
// bit tile shapes with a kernel instance (pair rows R x waves NW)
bool bit_shape_ok(int R, int NW) { return NW == 8 && (R == 16 || R == 24); }
}  // namespace

StepTuning step_tuning(bool bit) { return tunings().t[bit ? 1 : 0]; }

int temporal_rows(bool bit) {
    const int nr = tunings().nr[bit ? 1 : 0];
    if (!temporal_rows_ok(bit, nr)) return bit ? 24 : 48;
    if (bit && !bit_shape_ok(nr, tunings().nw_bit)) return 24;
    return nr;
}

int tile_waves(bool bit) {
    return bit && bit_shape_ok(temporal_rows(true), tunings().nw_bit) ? tunings().nw_bit : kStackWaves;
}

// VALU instructions per lane position of a tile for m generations.  Bit, per
// pair row and generation: 2 v_alignbit + 2 full adders (4 v_bitop3) + the
// rule for both dwords (16 v_bitop3) = 22 (+ 2 ds_bpermute on the LDS pipe);
// byte, per word row: the drifting frame (12) plus pack (8 v_dot4 + 3
// shifts) and unpack (8 x bfe/mul24/and) once per row and launch.
double tstep_valu_per_tile_lane(int m, bool byte) {
    if (byte) return (double)kStackWaves * (double)temporal_rows(false) * (12.0 * (double)m + 35.0);
    return (double)tile_waves(true) * (double)temporal_rows(true) * 22.0 * (double)m;
}

void set_temporal_rows(int kernel, int nr) {
    for (int k = 0; k < 2; k++)
        if ((kernel < 0 || kernel == k) && temporal_rows_ok(k == 1, nr)) tunings().nr[k] = nr;
}

void set_step_tuning(int kernel, int rows, int depth) {
    for (int k = 0; k < 2; k++) {
        if (kernel >= 0 && kernel != k) continue;
        if (rows == 16 || rows == 32 || rows == 64) tunings().t[k].rows = rows;
        if (depth == 2 || depth == 4 || depth == 8 || depth == 18) tunings().t[k].depth = depth;
    }
}

namespace {
template <class E, int R, int D>
hipError_t launch_rd(const StepArgs &a, bool wrapx, unsigned grid, hipStream_t s) {
    if (wrapx)
        step_kernel<E, R, D, true><<<grid, kBlock, 0, s>>>(a);
    else
        step_kernel<E, R, D, false><<<grid, kBlock, 0, s>>>(a);
    return hipGetLastError();
}

template <class E, int R>
hipError_t launch_r(const StepArgs &a, int depth, bool wrapx, unsigned grid, hipStream_t s) {
    switch (depth) {
    case 2: return launch_rd<E, R, 2>(a, wrapx, grid, s);
    case 8: return launch_rd<E, R, 8>(a, wrapx, grid, s);
    case 18:  // R = 16 only: the lane's whole strip (16 + 2 rows) loaded before any row is computed
        if constexpr (R == 16) return launch_rd<E, 16, 18>(a, wrapx, grid, s);
        return launch_rd<E, R, 4>(a, wrapx, grid, s);
    default: return launch_rd<E, R, 4>(a, wrapx, grid, s);
    }
}

template <class E>
hipError_t launch_e(const StepArgs &a, const StepTuning &t, bool wrapx, unsigned grid, hipStream_t s) {
    switch (t.rows) {
    case 16: return launch_r<E, 16>(a, t.depth, wrapx, grid, s);
    case 64: return launch_r<E, 64>(a, t.depth, wrapx, grid, s);
    default: return launch_r<E, 32>(a, t.depth, wrapx, grid, s);
    }
}
}  // namespace

// Per-XCD runs of one-generation strips (StepArgs::xcd).  Measured at
// 65536^2 (profiles/r03/r5f): byte 1.872 -> 1.730 ms (0.73 -> 0.79 of the copy
// ceiling), bit 0.1998 -> 0.2012 ms (within noise, off): on for the byte
// encoding.  LIFE_XCD_ORDER_ONEGEN=0/1 forces it for both.
static bool onegen_xcd_enabled(bool bit) {
    static const int v = [] {
        const char *e = getenv("LIFE_XCD_ORDER_ONEGEN");
        return e ? (atoi(e) != 0 ? 1 : 0) : -1;
    }();
    return v >= 0 ? v == 1 : !bit;
}

hipError_t launch_step(const life_layout &L, const uint8_t *in, uint8_t *out, uint8_t *sink,
                       const Region &reg, Wrap wrap, hipStream_t s) {
    if (reg.u1 <= reg.u0 || reg.r1 <= reg.r0) return hipSuccess;
    StepTuning t = step_tuning(is_bit(L));
    if (t.rows != 16 && t.rows != 64) t.rows = 32;
    StepArgs a;
    a.in = in;
    a.out = out;
    a.sink = sink;
    a.pitch = L.pitch;
    a.xoff = L.xoff;
    a.units = L.units;
    a.w = L.w;
    a.h = L.h;
    a.ya = L.yapron;
    a.u0 = reg.u0;
    a.u1 = reg.u1;
    a.r0 = reg.r0;
    a.r1 = reg.r1;
    a.nbx = (reg.u1 - reg.u0 + kBlock - 1) / kBlock;
    a.wrapy = wrap.y ? 1 : 0;
    a.xcd = onegen_xcd_enabled(is_bit(L)) ? 1 : 0;
    const int64_t nby = (reg.r1 - reg.r0 + t.rows - 1) / t.rows;
    const unsigned grid = (unsigned)(a.nbx * nby);
    return is_bit(L) ? launch_e<BitEnc>(a, t, wrap.x, grid, s) : launch_e<ByteEnc>(a, t, wrap.x, grid, s);
}

namespace {
// One launch; with events (timing on) through hipExtLaunchKernel, which
// stamps them with the dispatch's own start and end: no event packets
// between back-to-back launches (each cost a ~5 us bubble and ~6 us of host
// time before the first launch, profiles/r03/r4d trace).
hipError_t launch_fn(const void *fn, unsigned grid, unsigned threads, void *arg, hipStream_t s, hipEvent_t ev0,
                     hipEvent_t ev1) {
    void *args[] = {arg};
    if (ev0 || ev1) return hipExtLaunchKernel(fn, dim3(grid), dim3(threads), args, 0, s, ev0, ev1, 0);
    return hipLaunchKernel(fn, dim3(grid), dim3(threads), args, 0, s);
}

template <int R, int GK>
const void *byte_fn(Wrap wrap) {
    constexpr int NW = kStackWaves;
    if (wrap.x && wrap.y) return (const void *)tstep_byte_kernel<R, GK, true, true, NW>;
    if (wrap.x) return (const void *)tstep_byte_kernel<R, GK, true, false, NW>;
    if (wrap.y) return (const void *)tstep_byte_kernel<R, GK, false, true, NW>;
    return (const void *)tstep_byte_kernel<R, GK, false, false, NW>;
}

template <int GK>
const void *byte_k(Wrap wrap) {
    switch (temporal_rows(false)) {
    case 32: return byte_fn<32, GK>(wrap);
    default: return byte_fn<48, GK>(wrap);
    }
}

template <int R, int NW>
const void *bit_fn(Wrap wrap) {
    if (wrap.x && wrap.y) return (const void *)tstep_bit_kernel<R, true, true, NW>;
    if (wrap.x) return (const void *)tstep_bit_kernel<R, true, false, NW>;
    if (wrap.y) return (const void *)tstep_bit_kernel<R, false, true, NW>;
    return (const void *)tstep_bit_kernel<R, false, false, NW>;
}

// the bit tile shape's instances: per-launch tiles and the occupancy probe
#define LIFE_BIT_SHAPES(X) X(24, 8) X(16, 8)
const void *bit_k(Wrap wrap) {
    const int R = temporal_rows(true), NW = tile_waves(true);
#define LIFE_BIT_CASE(r, nw) \
    if (R == r && NW == nw) return bit_fn<r, nw>(wrap);
    LIFE_BIT_SHAPES(LIFE_BIT_CASE)
#undef LIFE_BIT_CASE
    return nullptr;
}
const void *tstep_bit_fn() { return bit_k(Wrap{true, true}); }
}  // namespace

// Byte tiles are compiled for a fixed ghost depth (a runtime depth measured
// 29 % slower, profiles/r02/ghost_ab.txt): K (16 / 32), and 1 for the
// one-generation launches of step(1) calls at the default tile height (a
// 384-row window then re-reads 2 rows instead of 64)
// (LIFE_BYTE_ONE_GHOST=0: K ghost rows for them too; A/B knob)
static bool byte_one_ghost(const life_layout &L, int m) {
    static const bool on = [] {
        const char *e = getenv("LIFE_BYTE_ONE_GHOST");
        return e ? atoi(e) != 0 : true;
    }();
    return on && !is_bit(L) && m == 1 && temporal_rows(false) == 48;
}
int tile_ghost(const life_layout &L, int m) {
    return is_bit(L) ? m : byte_one_ghost(L, m) ? 1 : L.generations_per_exchange;
}

// LIFE_BANDS=0: no banded tile column (A/B knob)
static bool bands_enabled() {
    static const bool on = [] {
        const char *e = getenv("LIFE_BANDS");
        return e ? atoi(e) != 0 : true;
    }();
    return on;
}

TileGeom tile_geom(const life_layout &L, int m) {
    TileGeom g;
    const bool bit = is_bit(L);
    g.lanes = 62;
    g.cells = bit ? 64 : 32;
    g.rows = (int64_t)tile_waves(bit) * temporal_rows(bit) - 2 * (int64_t)tile_ghost(L, m);
    const int64_t W = (L.w + g.cells - 1) / g.cells;  // lane columns (pairs / words) per row
    g.ntx = (W + g.lanes - 1) / g.lanes;
    g.nty = (L.h + g.rows - 1) / g.rows;
    // the last tile column owns o lane columns: bands of G >= o + 2 lanes when
    // G <= 32 (65536^2: 1024 pairs, o = 32, no bands; 32768^2: o = 16, G = 32)
    const int64_t o = W - g.lanes * (g.ntx - 1);
    int gsh = 2;
    while ((1 << gsh) < o + 2) ++gsh;
    g.gsh = bit && bands_enabled() && gsh <= 5 ? gsh : 6;
    g.bcol = g.gsh < 6 ? g.ntx - 1 : -1;
    return g;
}

// LIFE_XCD_ORDER=0: dispatch-order bit tiles instead of per-XCD row-major
// runs (TArgs::xcd_n).  Measured at the driver's 65536^2 call (profiles/r03/
// r5a): FETCH_SIZE x2 0.758 -> 0.572 GB per launch, WRITE_SIZE 0.554 -> 0.539
// GB (1.22x -> 1.035x compulsory), time within the run-to-run spread (+1 %)
static bool xcd_order_enabled() {
    static const bool on = [] {
        const char *e = getenv("LIFE_XCD_ORDER");
        return e ? atoi(e) != 0 : true;
    }();
    return on;
}
// LIFE_XCD_ORDER_BYTE=0: dispatch order for the byte tiles.  The per-XCD
// order measured (profiles/r03/r5b, 65536^2): 64.4-65.7 -> 66.9-67.0 T,
// FETCH_SIZE x2 5.81 -> 5.41 GB per 32-generation launch, WRITE unchanged.
// Walking each XCD's run in strips of 4 / 8 / 16 tile columns instead (so the
// tile below, sharing 64 ghost rows, is in flight beside each tile) fetched
// 1-3 % less and ran 12 / 5 / 0 % slower (r5l): a 768 KB window per tile
// leaves no L2 reuse to find
static bool xcd_order_byte_enabled() {
    static const bool on = [] {
        const char *e = getenv("LIFE_XCD_ORDER_BYTE");
        return e ? atoi(e) != 0 : true;
    }();
    return on;
}

// LIFE_TAIL_SPLIT: 0 no half-height tail tiles, 1 the round-4 rule (the
// fewest bottom tile rows whose half tiles fill one round, when the last
// round is under half full), 2 (default) the split a list-scheduling model
// of the launch says ends first (life::tail_plan, life_plan.cpp).  (Round 6
// measured a third tier, 3/4-height tiles, chosen by the same model: 5-7 %
// slower at the small blocks, profiles/r06/c -- removed.)
static int tail_split_mode() {
    static const int v = [] {
        const char *e = getenv("LIFE_TAIL_SPLIT");
        const int m = e ? atoi(e) : 2;
        return m >= 0 && m <= 2 ? m : 2;
    }();
    return v;
}
// LIFE_TAIL_C (measurement knob, default 0.06): the fixed share of a tile's
// duration (window load, stores, workgroup turnover) in the tail model's
// item durations (life::tail_plan).
static double tail_c() {
    static const double v = [] {
        const char *e = getenv("LIFE_TAIL_C");
        const double c = e ? atof(e) : 0.06;
        return c >= 0.0 && c < 1.0 ? c : 0.06;
    }();
    return v;
}
// resident workgroups of a kernel on this device (occupancy)
static int slots_of(const void *fn, int threads) {
    int dev = 0, cus = 0, per = 0;
    if (!fn || hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess ||
        hipOccupancyMaxActiveBlocksPerMultiprocessor(&per, fn, threads, 0) != hipSuccess)
        return 0;
    return cus * per;
}
// the bit tiles of the current shape (cached per shape)
static int tstep_bit_slots() {
    static int cached = 0, key = -1;
    const int k = temporal_rows(true) * 64 + tile_waves(true);
    if (k != key) {
        cached = slots_of(tstep_bit_fn(), 64 * tile_waves(true));
        key = k;
    }
    return cached;
}

int tile_slots(const life_layout &L) {
    if (is_bit(L)) return tstep_bit_slots();
    static int cached = 0, key = -1;
    const int k = temporal_rows(false);
    if (k != key) {
        cached = slots_of(byte_k<32>(Wrap{true, true}), 64 * kStackWaves);
        key = k;
    }
    return cached;
}

int64_t region_items(const TileGeom &g, const TileRegion &r) {
    if (r.tx1 <= r.tx0 || r.ty1 <= r.ty0) return 0;
    if (g.gsh >= 6 || r.tx1 != g.bcol + 1) return (r.tx1 - r.tx0) * (r.ty1 - r.ty0);
    const int64_t B = 64 >> g.gsh;
    return (r.tx1 - r.tx0 - 1) * (r.ty1 - r.ty0) + (r.ty1 - r.ty0 + B - 1) / B;
}

life_layout extended_layout(const life_layout &L, const Extend &ext) {
    life_layout V = L;
    V.h += 2 * ext.y;
    V.yapron -= ext.y;
    V.rows = V.h + 2 * V.yapron;
    return V;
}

// Bands of the tile columns [tx0, tx1): B tile rows per banded item when
// the region holds the banded last column, else 1 (no bands).
static int64_t region_bands(const TileGeom &g, int64_t tx1) { return g.gsh < 6 && tx1 == g.bcol + 1 ? 64 >> g.gsh : 1; }

// The tail plan of a bit launch over tile columns [tx0, tx1) x rows [ty0,
// ty1) of tile_geom(L, m), beside `pre` items of another launch dispatched
// just before it (launch_tstep; cached by life::tail_plan).
static TailPlan tail_plan_for(const life_layout &L, const TileGeom &g, int m, int64_t tx0, int64_t tx1, int64_t ty0,
                              int64_t ty1, int64_t pre) {
    const int64_t T2 = (int64_t)tile_waves(true) * (temporal_rows(true) / 2) - 2 * (int64_t)tile_ghost(L, m);
    const int64_t yend = std::min(ty1 * g.rows, L.h);
    return tail_plan(tx1 - tx0, region_bands(g, tx1), ty0, ty1, yend, g.rows, T2, tstep_bit_slots(),
                     tail_split_mode(), tail_c(), pre);
}

void prewarm_tail_plans(const life_layout &L, int mmax, bool ext_y) {
    if (!is_bit(L) || L.generations_per_exchange < 2 || tail_split_mode() == 0) return;
    const int K = L.generations_per_exchange;
    for (int m = 1; m <= std::min(mmax, K); ++m)
        for (int e = 0; e <= (ext_y ? K - m : 0); ++e) {
            Extend x;
            x.y = e;
            const life_layout V = extended_layout(L, x);
            const TileGeom g = tile_geom(V, m);
            if (g.rows >= 1) (void)tail_plan_for(V, g, m, 0, g.ntx, 0, g.nty, 0);
        }
}

hipError_t launch_tstep(const life_layout &Lin, const uint8_t *in, uint8_t *out, const TileRegion *r, int nreg,
                        int m, Wrap wrap, hipStream_t s, double *valu_lane_ops, hipEvent_t ev0, hipEvent_t ev1,
                        Extend ext, int64_t concurrent) {
    const int K = Lin.generations_per_exchange;
    const bool bit = is_bit(Lin);
    // m <= 32: the tile's edge lanes absorb at most 32 wrong cells; m <= the
    // apron depth a partitioned axis provides.  Deep-halo passes: bit only
    // (the byte windows hold K ghost rows whatever m is), the window's top
    // ghost rows inside the apron (y + m <= yapron), no wrapped axis extended.
    if (nreg < 0 || nreg > kMaxRegions || m > K || m > 32 || K < 2 || Lin.yapron != K || ext.y < 0 ||
        ((ext.y > 0 || ext.x) && (!bit || ext.y + m > K || (ext.y > 0 && wrap.y) || (ext.x && wrap.x))) ||
        tile_waves(bit) * temporal_rows(bit) - 2 * tile_ghost(Lin, m) < 1 || (!bit && K != 16 && K != 32))
        return hipErrorInvalidValue;
    const life_layout L = extended_layout(Lin, ext);
    const TileGeom g = tile_geom(L, m);
    TArgs a;
    a.in = in;
    a.out = out;
    a.pitch = L.pitch;
    a.xoff = L.xoff;
    a.W = (L.w + g.cells - 1) / g.cells;  // the last lane column may be partial: its upper cells are the right apron
    a.h = L.h;
    a.ya = L.yapron;
    a.m = m;
    a.xext = ext.x ? 1 : 0;
    a.nreg = 0;
    a.first[0] = 0;
    a.gsh = (int32_t)g.gsh;
    a.bcol = g.bcol;
    for (int k = 0; k < nreg; k++) {
        if (r[k].tx1 <= r[k].tx0 || r[k].ty1 <= r[k].ty0) continue;
        const int n = a.nreg++;
        a.tx0[n] = r[k].tx0;
        a.tx1[n] = r[k].tx1;
        a.ty0[n] = r[k].ty0;
        a.ty1[n] = r[k].ty1;
        a.first[n + 1] = a.first[n] + region_items(g, r[k]);
    }
    if (a.nreg == 0 || m <= 0) return hipSuccess;
    int64_t items = a.first[a.nreg];  // one workgroup per tile (or banded item)
    a.tail_first = a.tail_y = a.tail_yend = a.tail_ntx = a.tail_tx0 = 0;
    a.tail_band = 0;
    const int64_t T2 = (int64_t)tile_waves(bit) * (temporal_rows(bit) / 2) - 2 * (int64_t)tile_ghost(L, m);
    if (bit && T2 >= 1 && a.nreg == 1 && tail_split_mode() > 0 && concurrent >= 0) {
        // One region: the whole shard, a deep-halo pass over the extended
        // shard, a row strip's interior, or (round 6) the interior of an
        // exchange pass beside its ring (`concurrent` = the ring's items,
        // dispatched just before it on another stream).  The launch runs
        // items / slots rounds of equal tiles; a last round under full leaves
        // CUs idle for up to a whole tile time.  The bottom tile rows are
        // re-tiled as half-height tiles (banded in the last column like the
        // full tiles, round 6), dispatched last, so the final round is
        // half-length items on every slot (life::tail_plan).  The byte tiles
        // (2 per CU, 32 ghost rows: a third of a half tile) lost 3-4 % with
        // half tiles (profiles/r02/r2z) and keep whole tiles.
        const int64_t tx0 = a.tx0[0], tx1 = a.tx1[0], ty0 = a.ty0[0], ty1 = a.ty1[0];
        const int64_t yend = std::min(ty1 * g.rows, L.h), B = region_bands(g, tx1);
        const TailPlan p = tail_plan_for(L, g, m, tx0, tx1, ty0, ty1, concurrent);
        if (p.F < ty1 && p.F >= ty0) {
            a.ty1[0] = p.F;
            a.first[1] = region_items(g, TileRegion{tx0, tx1, ty0, p.F});
            a.tail_first = a.first[1];
            a.tail_y = p.F * g.rows;
            a.tail_yend = yend;
            a.tail_ntx = tx1 - tx0;
            a.tail_tx0 = tx0;
            a.tail_band = B > 1 ? 1 : 0;
            items = a.tail_first + tail_row_items(tx1 - tx0, B, p.n2);
        }
    }
    const bool split = a.tail_ntx > 0;
    a.xcd_n = (bit ? xcd_order_enabled() : xcd_order_byte_enabled()) ? (split ? a.tail_first : items) : 0;
    if (valu_lane_ops) {
        const double lane = 64.0 * tstep_valu_per_tile_lane(m, !bit);
        *valu_lane_ops = (double)(split ? a.tail_first : items) * lane;
        if (split)  // half tiles: R / 2 register rows per wave
            *valu_lane_ops += (double)(items - a.tail_first) * lane * 0.5;
    }
    const void *fn = bit                      ? bit_k(wrap)
                     : byte_one_ghost(L, m) ? byte_fn<48, 1>(wrap)
                     : K == 16              ? byte_k<16>(wrap)
                                            : byte_k<32>(wrap);
    if (!fn) return hipErrorInvalidValue;
    return launch_fn(fn, (unsigned)items, 64u * (unsigned)tile_waves(bit), &a, s, ev0, ev1);
}

namespace {
// Instances of the dataflow tiles (bit, both axes wrapped): one per tile shape
// and hand-off form.
// (LIFE_FLOW_BANDS=0: full-width tiles in the last column; A/B knob)
bool flow_bands_enabled() {
    static const bool on = [] {
        const char *e = getenv("LIFE_FLOW_BANDS");
        return e ? atoi(e) != 0 : true;
    }();
    return on;
}
const void *flow_kernel_of(const life_layout &L, int flow, bool band = false) {
    if (!is_bit(L)) return nullptr;
    const int R = temporal_rows(true), NW = tile_waves(true);
#define LIFE_BIT_CASE(r, nw)                                                                     \
    if (R == r && NW == nw) {                                                                    \
        if (band)                                                                                \
            return flow == 2 ? (const void *)tflow_kernel<r, true, true, 2, nw, true>            \
                             : (const void *)tflow_kernel<r, true, true, 1, nw, true>;           \
        return flow == 2 ? (const void *)tflow_kernel<r, true, true, 2, nw>                      \
                         : (const void *)tflow_kernel<r, true, true, 1, nw>;                     \
    }
    LIFE_BIT_SHAPES(LIFE_BIT_CASE)
#undef LIFE_BIT_CASE
    return nullptr;
}
// the banded form for this geometry: a banded last column (tile_geom)
bool flow_band(const TileGeom &g) { return g.gsh < 6 && flow_bands_enabled(); }
}  // namespace

int64_t flow_items_per_pass(const life_layout &L, int m, bool work_only) {
    const TileGeom g = tile_geom(L, m);
    if (!flow_band(g)) return g.ntx * g.nty;
    const int64_t B = 64 >> g.gsh, ngroups = (g.nty + B - 1) / B;
    // work_only: without the no-op padding items of the last group
    return work_only ? (g.ntx - 1) * g.nty + ngroups : ngroups * ((g.ntx - 1) * B + 1);
}

bool flow_ok(const life_layout &L, int m) {
    // an instance for this encoding / tile shape, and the dependency rule
    // reads tile rows ty-2..ty+2: a window may reach at most one tile row
    // beyond its neighbours (ghost rows <= T)
    if (!flow_kernel_of(L, 1) || m < 1) return false;
    const TileGeom g = tile_geom(L, m);
    return g.rows >= tile_ghost(L, m);
}

int flow_slots(const life_layout &L) {
    static int cached = 0, key = -1;
    const int k = is_bit(L) ? temporal_rows(true) * 64 + tile_waves(true) : -2;
    if (k != key) {
        cached = slots_of(flow_kernel_of(L, 1), 64 * tile_waves(is_bit(L)));
        key = k;
    }
    return cached;
}

hipError_t prewarm_tflow(const life_layout &L, int m, int flow, unsigned int *head, hipStream_t s) {
    const TileGeom g = tile_geom(L, m);
    const void *fn = flow_kernel_of(L, flow, flow_band(g));
    if (!fn || !flow_ok(L, m) || flow_slots(L) <= 0) return hipErrorInvalidValue;  // (caches the slot count)
    FArgs f{};  // no items: the one workgroup pulls item 0 and leaves
    f.head = head;
    const hipError_t e = hipMemsetAsync(head, 0, sizeof(unsigned int), s);
    if (e != hipSuccess) return e;
    return launch_fn(fn, 1u, 64u * (unsigned)tile_waves(true), &f, s, nullptr, nullptr);
}

hipError_t launch_tflow(const life_layout &L, const uint8_t *in, uint8_t *out, int m, int64_t passes,
                        unsigned int *head, unsigned int *done, Wrap wrap, int flow, hipStream_t s, hipEvent_t ev0,
                        hipEvent_t ev1) {
    const void *fn = flow_kernel_of(L, flow);
    if (!fn || !wrap.x || !wrap.y || m < 1 || m > 32 || m > L.generations_per_exchange || passes < 1 ||
        !flow_ok(L, m))
        return hipErrorInvalidValue;
    const TileGeom g = tile_geom(L, m);
    FArgs f{};
    f.t.in = in;
    f.t.out = out;
    f.t.pitch = L.pitch;
    f.t.xoff = L.xoff;
    f.t.W = (L.w + g.cells - 1) / g.cells;
    f.t.h = L.h;
    f.t.ya = L.yapron;
    f.t.m = m;
    const bool band = flow_band(g);
    if (band) fn = flow_kernel_of(L, flow, true);
    f.t.gsh = band ? (int32_t)g.gsh : 6;
    f.t.bcol = band ? g.bcol : -1;
    f.ntx = g.ntx;
    f.nty = g.nty;
    f.B = band ? 64 >> g.gsh : 1;
    f.ngroups = (g.nty + f.B - 1) / f.B;
    f.per_pass = flow_items_per_pass(L, m);
    f.items = passes * f.per_pass;
    f.head = head;
    f.done = done;
    hipError_t e = hipMemsetAsync(head, 0, sizeof(unsigned int), s);  // the error word is the caller's
    if (e == hipSuccess) e = hipMemsetAsync(done, 0, sizeof(unsigned int) * (size_t)(g.ntx * g.nty), s);
    if (e != hipSuccess) return e;
    const int n = flow_slots(L);  // resident workgroups
    if (n <= 0) return hipErrorInvalidValue;
    const unsigned grid = (unsigned)std::min<int64_t>(f.items, n);
    // every workgroup pulls one item past the last: the 32-bit head must not wrap
    if (f.items + (int64_t)grid > kFlowMaxHead) return hipErrorInvalidValue;
    return launch_fn(fn, grid, 64u * (unsigned)tile_waves(true), &f, s, ev0, ev1);
}

int reg_small_rows(const life_layout &L) {
    const int64_t W = (L.w + 31) / 32;
    if (W > kRegMaxW || L.h <= 0) return 0;
    int64_t Wp = 1;
    while (Wp < W) Wp <<= 1;
    const int64_t strips = kRegThreads / Wp;
    for (int R : kRegRows)
        if (L.h % R == 0 && L.h / R <= strips) return R;
    return 0;
}

hipError_t launch_reg_small(const life_layout &L, const uint8_t *in, uint8_t *out, int64_t gens,
                            hipStream_t s) {
    const int R = reg_small_rows(L);
    if (R == 0 || gens <= 0 || gens > INT32_MAX) return hipErrorInvalidValue;
    RArgs a;
    a.in = in;
    a.out = out;
    a.pitch = L.pitch;
    a.xoff = L.xoff;
    a.ya = L.yapron;
    a.w = (int32_t)L.w;
    a.h = (int32_t)L.h;
    a.W = (int32_t)((L.w + 31) / 32);
    a.lgWp = 0;
    while ((1 << a.lgWp) < a.W) ++a.lgWp;
    a.gens = (int32_t)gens;
    a.bit = is_bit(L) ? 1 : 0;
    a.ns = (int32_t)(L.h / R);
    a.own = a.h;
    a.K = 0;
    a.nat_in = a.nat_out = 0;
    return L.w % 32 ? launch_rs<true, false>(a, R, 1, s) : launch_rs<false, false>(a, R, 1, s);
}

// Windowed plan: strip height R, halo K, strips per window ns (ns*R = own +
// 2K), owned rows per workgroup.  Zero when the grid is not a VGPR shape, or
// too short for one window to leave owned rows to more than one workgroup.
// R = 0: automatic, R = 1 and K = min(30, (ns - 4) / 2), i.e. 4 owned rows per
// workgroup -- the p46gun_big sweep (profiles/r01/p46_window_*.jsonl): R = 1
// beats R >= 2 at every K, and the rate rises with K up to 30 (a
// generation costs one barrier's latency whatever the window holds, so
// deeper halos mean fewer launches).
RegWinPlan reg_win_plan(const life_layout &L, int R, int K) {
    RegWinPlan p{};
    const int64_t W = (L.w + 31) / 32;
    if (W > kRegMaxW || L.h <= 0) return p;
    int64_t Wp = 1;
    while (Wp < W) Wp <<= 1;
    const int64_t ns = kRegThreads / Wp;
    if (R == 0) {
        R = 1;
        K = (int)std::min<int64_t>(30, (ns - 4) / 2);
        if (K < 8) return p;
    }
    if (K < 1 || (R != 1 && R != 2 && R != 3 && R != 4 && R != 5 && R != 6 && R != 8)) return p;
    const int64_t own = ns * R - 2 * K;
    if (own < 1 || own >= L.h) return p;
    p.R = R;
    p.K = K;
    p.ns = (int)ns;
    p.own = (int)own;
    p.blocks = (int)((L.h + own - 1) / own);
    return p;
}

hipError_t launch_reg_win(const life_layout &L, const RegWinPlan &p, const uint8_t *in, uint8_t *out, int gens,
                          hipStream_t s, bool nat_in, bool nat_out) {
    if (p.blocks < 1 || gens < 1 || gens > p.K || in == out) return hipErrorInvalidValue;
    RArgs a;
    a.in = in;
    a.out = out;
    a.pitch = L.pitch;
    a.xoff = L.xoff;
    a.ya = L.yapron;
    a.w = (int32_t)L.w;
    a.h = (int32_t)L.h;
    a.W = (int32_t)((L.w + 31) / 32);
    a.lgWp = 0;
    while ((1 << a.lgWp) < a.W) ++a.lgWp;
    a.gens = gens;
    a.bit = is_bit(L) ? 1 : 0;
    a.ns = p.ns;
    a.own = p.own;
    a.K = p.K;
    const bool fits = L.xoff + 4 * (int64_t)a.W <= L.pitch;  // natural words inside the padded row
    a.nat_in = nat_in && fits ? 1 : 0;
    a.nat_out = nat_out && fits ? 1 : 0;
    const unsigned b = (unsigned)p.blocks;
    return L.w % 32 ? launch_rs<true, true>(a, p.R, b, s) : launch_rs<false, true>(a, p.R, b, s);
}

int64_t small_lds_bytes(const life_layout &L) {
    const int64_t W = (L.w + 31) / 32;
    return W > kSmallThreads ? INT64_MAX : 2 * W * L.h * 4;
}

hipError_t launch_small(const life_layout &L, const uint8_t *in, uint8_t *out, int64_t gens, hipStream_t s) {
    const int64_t bytes = small_lds_bytes(L);
    if (bytes > kSmallMaxLds || gens <= 0 || gens > INT32_MAX) return hipErrorInvalidValue;
    static bool attr_set = false;  // opt in to more than 64 KiB of dynamic LDS
    if (!attr_set) {
        const hipError_t e = hipFuncSetAttribute((const void *)small_kernel,
                                                 hipFuncAttributeMaxDynamicSharedMemorySize, (int)kSmallMaxLds);
        if (e != hipSuccess) return e;
        attr_set = true;
    }
    SArgs a;
    a.in = in;
    a.out = out;
    a.pitch = L.pitch;
    a.xoff = L.xoff;
    a.ya = L.yapron;
    a.w = (int32_t)L.w;
    a.h = (int32_t)L.h;
    a.W = (int32_t)((L.w + 31) / 32);
    a.gens = (int32_t)gens;
    a.bit = is_bit(L) ? 1 : 0;
    small_kernel<<<1, kSmallThreads, (size_t)bytes, s>>>(a);
    return hipGetLastError();
}

hipError_t launch_pack_columns(const life_layout &L, const uint8_t *buf, uint8_t *stage, hipStream_t s,
                               bool corners) {
    if (corners && L.xapron < 32) return hipErrorInvalidValue;
    const int64_t nc = corners ? 4 * L.yapron : 0;
    pack_columns_kernel<<<blocks_for(L.h + nc, 256), 256, 0, s>>>(buf, L.pitch, L.yapron, L.xoff, L.w, L.h, L.xapron,
                                                                   stage, is_bit(L), nc);
    return hipGetLastError();
}

hipError_t launch_wrap_columns(const life_layout &L, uint8_t *buf, hipStream_t s) {
    if (L.xapron < 32 || L.w < L.xapron) return hipErrorInvalidValue;
    wrap_columns_kernel<<<blocks_for(L.h, 256), 256, 0, s>>>(buf, L.pitch, L.yapron, L.xoff, L.w, L.h, is_bit(L));
    return hipGetLastError();
}

hipError_t launch_unpack_columns(const life_layout &L, uint8_t *buf, const uint8_t *stage, hipStream_t s,
                                 bool corners) {
    if (corners && L.xapron < 32) return hipErrorInvalidValue;
    const int64_t nc = corners ? 4 * L.yapron : 0;
    unpack_columns_kernel<<<blocks_for(L.h + nc, 256), 256, 0, s>>>(buf, L.pitch, L.yapron, L.xoff, L.w, L.h,
                                                                     L.xapron, stage, is_bit(L), nc);
    return hipGetLastError();
}

hipError_t launch_import_block(const life_layout &L, const uint8_t *dense, uint8_t *buf, hipStream_t s) {
    const unsigned g = blocks_for(L.units * L.h, 256);
    if (is_bit(L))
        import_kernel<128><<<g, 256, 0, s>>>(dense, buf, L.pitch, L.yapron, L.xoff, L.w, L.h, L.units);
    else
        import_kernel<16><<<g, 256, 0, s>>>(dense, buf, L.pitch, L.yapron, L.xoff, L.w, L.h, L.units);
    return hipGetLastError();
}

hipError_t launch_export_block(const life_layout &L, const uint8_t *buf, uint8_t *dense, hipStream_t s) {
    const unsigned g = blocks_for(L.units * L.h, 256);
    if (is_bit(L))
        export_kernel<128><<<g, 256, 0, s>>>(buf, dense, L.pitch, L.yapron, L.xoff, L.w, L.h, L.units);
    else
        export_kernel<16><<<g, 256, 0, s>>>(buf, dense, L.pitch, L.yapron, L.xoff, L.w, L.h, L.units);
    return hipGetLastError();
}

hipError_t launch_fill_random(const life_layout &L, int64_t nx, uint64_t key, uint32_t thr32, uint8_t *buf,
                              hipStream_t s) {
    const unsigned g = blocks_for(L.units * L.h, 256);
    if (is_bit(L))
        fill_random_kernel<128><<<g, 256, 0, s>>>(buf, L.pitch, L.yapron, L.xoff, L.w, L.h, L.units, L.x0, L.y0, nx,
                                                  key, thr32);
    else
        fill_random_kernel<16><<<g, 256, 0, s>>>(buf, L.pitch, L.yapron, L.xoff, L.w, L.h, L.units, L.x0, L.y0, nx,
                                                 key, thr32);
    return hipGetLastError();
}

hipError_t launch_vtk_block(const life_layout &L, const uint8_t *buf, uint8_t *out, hipStream_t s) {
    const dim3 grid(blocks_for((L.w + 7) / 8, 256), (unsigned)(L.h < 8192 ? L.h : 8192));
    if (is_bit(L))
        vtk_kernel<true><<<grid, 256, 0, s>>>(buf, L.pitch, L.yapron, L.xoff, L.w, L.h, out);
    else
        vtk_kernel<false><<<grid, 256, 0, s>>>(buf, L.pitch, L.yapron, L.xoff, L.w, L.h, out);
    return hipGetLastError();
}

hipError_t launch_bits_block(const life_layout &L, const uint8_t *buf, uint8_t *out, hipStream_t s) {
    const int sh = (int)(L.x0 & 7);
    const int64_t rb = bits_row_bytes(L);
    const dim3 grid(blocks_for(rb, 256), (unsigned)(L.h < 8192 ? L.h : 8192));
    if (is_bit(L))
        bits_kernel<true><<<grid, 256, 0, s>>>(buf, L.pitch, L.yapron, L.xoff, L.w, L.h, sh, out, rb);
    else
        bits_kernel<false><<<grid, 256, 0, s>>>(buf, L.pitch, L.yapron, L.xoff, L.w, L.h, sh, out, rb);
    return hipGetLastError();
}

namespace {
// Copy ceiling: one 16-B load + store per lane, one wave-instruction each,
// a workgroup per 4 KiB.  Measured against grid-stride, unrolled and
// nontemporal variants (scripts/ubench_copy.hip, profiles/r01/ubench_copy.txt):
// this shape is the fastest, 6.30 TB/s on 2 GiB.
__global__ __launch_bounds__(256) void copy_kernel(const uint4 *__restrict__ in, uint4 *__restrict__ out,
                                                   int64_t n) {
    const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (i < n) out[i] = in[i];
}
}  // namespace

hipError_t launch_copy(const void *in, void *out, int64_t bytes, hipStream_t s) {
    const int64_t n = bytes / 16;
    copy_kernel<<<(unsigned)((n + 255) / 256), 256, 0, s>>>(reinterpret_cast<const uint4 *>(in),
                                                            reinterpret_cast<uint4 *>(out), n);
    return hipGetLastError();
}

hipError_t launch_census(const life_layout &L, int64_t nx, const uint8_t *buf, unsigned long long *out,
                         hipStream_t s) {
    const dim3 grid(blocks_for(L.units, 256), (unsigned)(L.h < 4096 ? L.h : 4096));
    if (is_bit(L))
        census_kernel<128><<<grid, 256, 0, s>>>(buf, L.pitch, L.yapron, L.xoff, L.w, L.h, L.units, L.x0, L.y0, nx,
                                                 out);
    else
        census_kernel<16><<<grid, 256, 0, s>>>(buf, L.pitch, L.yapron, L.xoff, L.w, L.h, L.units, L.x0, L.y0, nx,
                                                out);
    return hipGetLastError();
}

}  // namespace life
