// life_bitops.h -- bit-sliced Game-of-Life building blocks shared by the
// gfx950 kernels (life_kernels.hip).  Device code only.
//
// BIT encoding layout (HBM and registers): cells come in 64-cell PAIRS of
// dwords, bit-interleaved -- pair p of a row holds cells [64p, 64p + 64) as
// E (dword 2p: bit i = cell 64p + 2i, the even cells) and O (dword 2p + 1:
// bit i = cell 64p + 2i + 1, the odd cells).  The horizontal neighbours of an
// even cell are the odd cells at the same bit of O and one bit below, of an
// odd cell the even cells at the same bit of E and one bit above: a row's
// 3-cell sums need ONE funnel shift per dword (v_alignbit, issued at half the
// rate of v_bitop3 on gfx950: profiles/r01/ubench_valu.txt) instead of two
// plus a DPP move for the natural layout -- 12.9 vs 16.4 ns per word and
// generation in registers (profiles/r03/ubench_pair.txt).
//
// A row's horizontal 3-sums are a 2-bit number per cell (full adder of the
// cell and its two neighbours); three rows' sums give n9 = u0 + 2*S, and the
// B3/S23 rule of life_cart.c:202-208 / life2d.c:117-123 becomes 8
// v_bitop3_b32 (a 3-gate tail is impossible: exhaustive search,
// profiles/r03/rule_search.txt).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace life {

// v_bitop3_b32 (gfx950): any 3-input bitwise function in one VALU op.  The
// truth table is indexed by {S0,S1,S2} with S0 the most significant bit, so
// the immediate of f is f(0xF0, 0xCC, 0xAA).
template <uint32_t IMM>
__device__ __forceinline__ uint32_t b3(uint32_t a, uint32_t b, uint32_t c) {
    return __builtin_amdgcn_bitop3_b32(a, b, c, IMM);
}
constexpr uint32_t kXor3 = 0xF0 ^ 0xCC ^ 0xAA;                          // a ^ b ^ c
constexpr uint32_t kMaj = (0xF0 & 0xCC) | (0xF0 & 0xAA) | (0xCC & 0xAA);  // majority
constexpr uint32_t kEq1 = ((0xF0 ^ 0xCC) & ~0xAA) & 0xFF;                // (v0^k0) & ~v1
constexpr uint32_t kEq2 = (~(0xF0 ^ 0xCC) & (0xAA ^ (0xF0 & 0xCC))) & 0xFF;  // ~(v0^k0) & (v1^(v0&k0))
constexpr uint32_t kMux = ((0xF0 & 0xCC) | (~0xF0 & 0xAA)) & 0xFF;       // a ? b : c
constexpr uint32_t kAndOr = (0xF0 & (0xCC | 0xAA)) & 0xFF;               // a & (b | c)

// Pair layout of a cell x (x may be negative: aprons; arithmetic shifts give
// floor division): dword index relative to the row's cell 0 and bit.
__host__ __device__ __forceinline__ int64_t pair_dword(int64_t x) { return ((x >> 6) << 1) | (x & 1); }
__host__ __device__ __forceinline__ uint32_t pair_bit(int64_t x) { return (uint32_t)((x & 63) >> 1); }

// Bit (de)interleaving between a pair (E, O) and the natural 64-bit order
// (bit j = cell j): helper kernels only (halo columns, frames, small grids).
__device__ __forceinline__ uint32_t spread16(uint32_t x) {  // bit i -> bit 2i, i < 16
    x &= 0xFFFFu;
    x = (x | (x << 8)) & 0x00FF00FFu;
    x = (x | (x << 4)) & 0x0F0F0F0Fu;
    x = (x | (x << 2)) & 0x33333333u;
    return (x | (x << 1)) & 0x55555555u;
}
__device__ __forceinline__ uint32_t compact16(uint32_t x) {  // bit 2i -> bit i
    x &= 0x55555555u;
    x = (x | (x >> 1)) & 0x33333333u;
    x = (x | (x >> 2)) & 0x0F0F0F0Fu;
    x = (x | (x >> 4)) & 0x00FF00FFu;
    return (x | (x >> 8)) & 0x0000FFFFu;
}
// 32 natural cells (bit k = cell k) from 16 even / 16 odd cells, and back
__device__ __forceinline__ uint32_t nat32(uint32_t e16, uint32_t o16) { return spread16(e16) | (spread16(o16) << 1); }
__device__ __forceinline__ uint64_t nat64(uint32_t e, uint32_t o) {
    return (uint64_t)nat32(e, o) | ((uint64_t)nat32(e >> 16, o >> 16) << 32);
}
__device__ __forceinline__ uint2 pair_of(uint64_t v) {
    const uint32_t lo = (uint32_t)v, hi = (uint32_t)(v >> 32);
    return make_uint2(compact16(lo) | (compact16(hi) << 16), compact16(lo >> 1) | (compact16(hi >> 1) << 16));
}

struct BitEnc {
    static constexpr int64_t kCellsPerUnit = 128;  // a 16-B unit = two pairs (E0, O0, E1, O1)
    static constexpr uint32_t kCell0 = 1u;
    static __device__ __forceinline__ int64_t dword_of(int64_t x) { return pair_dword(x); }
    static __device__ __forceinline__ uint32_t pos_in_dword(int64_t x) { return pair_bit(x); }
    static __device__ __forceinline__ uint32_t top_shift(int64_t x) { return 31u - pos_in_dword(x); }
    struct H {
        uint32_t s0[4], s1[4];
    };
    // full adder: L + C + R = s0 + 2*s1
    static __device__ __forceinline__ void fa(uint32_t L, uint32_t C, uint32_t R, uint32_t &s0,
                                              uint32_t &s1) {
        s0 = b3<kXor3>(L, C, R);
        s1 = b3<kMaj>(L, C, R);
    }
    // Horizontal sums of one pair: even cells 2i take O[i-1] + E[i] + O[i]
    // (op: the O dword of the pair on the left, its bit 31 = cell 2i - 1 at
    // i = 0), odd cells 2i+1 take E[i] + O[i] + E[i+1] (en: the E dword of
    // the pair on the right, bit 0 = the cell after 2i + 1 at i = 31).
    static __device__ __forceinline__ void pair_sums(uint32_t e, uint32_t o, uint32_t op, uint32_t en,
                                                     uint32_t &e0, uint32_t &e1, uint32_t &o0, uint32_t &o1) {
        fa(__builtin_amdgcn_alignbit(o, op, 31), e, o, e0, e1);
        fa(e, o, __builtin_amdgcn_alignbit(en, e, 1), o0, o1);
    }
    // The 128 cells of a 16-B unit (two pairs); l: the O dword left of the
    // unit, r: the E dword right of it.
    static __device__ __forceinline__ H hsum(uint4 d, uint32_t l, uint32_t r) {
        H h;
        pair_sums(d.x, d.y, l, d.z, h.s0[0], h.s1[0], h.s0[1], h.s1[1]);
        pair_sums(d.z, d.w, d.y, r, h.s0[2], h.s1[2], h.s0[3], h.s1[3]);
        return h;
    }
    // Rows a, b, c (2-bit horizontal sums) -> next state of the centre row.
    // n9 = (a0+b0+c0) + 2(a1+b1+c1) = u0 + 2*S with S = v0 + k0 + 2*v1;
    // alive' = (n9 == 3) | (alive & n9 == 4) = u0 ? S==1 : (alive & S==2).
    static __device__ __forceinline__ uint32_t rule1(uint32_t a0, uint32_t a1, uint32_t b0, uint32_t b1,
                                                     uint32_t c0, uint32_t c1, uint32_t alive) {
        const uint32_t u0 = b3<kXor3>(a0, b0, c0), k0 = b3<kMaj>(a0, b0, c0);
        const uint32_t v0 = b3<kXor3>(a1, b1, c1), v1 = b3<kMaj>(a1, b1, c1);
        const uint32_t eq1 = b3<kEq1>(v0, k0, v1);  // S == 1
        const uint32_t eq2 = b3<kEq2>(v0, k0, v1);  // S == 2
        const uint32_t e = b3<kMux>(u0, eq1, eq2);
        return b3<kAndOr>(e, u0, alive);  // u0 ? eq1 : (alive & eq2)
    }
    static __device__ __forceinline__ uint4 rule(const H &a, const H &b, const H &c, uint4 v) {
        uint4 o;
        o.x = rule1(a.s0[0], a.s1[0], b.s0[0], b.s1[0], c.s0[0], c.s1[0], v.x);
        o.y = rule1(a.s0[1], a.s1[1], b.s0[1], b.s1[1], c.s0[1], c.s1[1], v.y);
        o.z = rule1(a.s0[2], a.s1[2], b.s0[2], b.s1[2], c.s0[2], c.s1[2], v.z);
        o.w = rule1(a.s0[3], a.s1[3], b.s0[3], b.s1[3], c.s0[3], c.s1[3], v.w);
        return o;
    }
};

__device__ __forceinline__ uint32_t bperm(int addr, uint32_t v) {
    return (uint32_t)__builtin_amdgcn_ds_bpermute(addr, (int)v);
}

// BYTE tiles (natural 32-cell words per lane, packed from bytes on load):
// drifting frame: the next state of cell x-1 is computed at the bit that held
// cell x, so a row's sums need only the LEFT neighbour word: with P the row's
// bits, hsum at p = P[p-2] + P[p-1] + P[p] = LL + L + v (L = v << 1 | l >> 31,
// LL = v << 2 | l >> 30, l by ds_bpermute), and the cell's own state is L.
// The frame moves one bit left per generation for every row alike; after m
// generations bit p holds cell p - m and the store realigns once per launch.
// Light cone: after m <= 32 generations window positions [2m, 2048) are exact,
// i.e. cells [m, 2048 - m) after realignment.  12 VALU (2 v_alignbit, 10
// v_bitop3) + 1 ds_bpermute per row and generation.
__device__ __forceinline__ void bit_hsum_drift(uint32_t v, int laddr, uint32_t &s0, uint32_t &s1, uint32_t &L) {
    const uint32_t l = bperm(laddr, v);
    L = __builtin_amdgcn_alignbit(v, l, 31);
    const uint32_t LL = __builtin_amdgcn_alignbit(v, l, 30);
    BitEnc::fa(LL, L, v, s0, s1);
}
// after m generations in the drifting frame: the aligned word of this lane's
// column (bits m..31 of this lane, 0..m-1 of the right lane)
__device__ __forceinline__ uint32_t drift_realign(uint32_t v, int m) {
    const uint32_t r = bperm((((int)__lane_id() + 1) & 63) << 2, v);
    if (m == 0) return v;
    return m >= 32 ? r : __builtin_amdgcn_alignbit(r, v, (uint32_t)m);
}

// BYTE encoding through the same lanes: a lane's word column is 32 byte cells
// (two 16-B loads per row), packed into one word on load (v_dot4_u32_u8
// weights 1..128 per byte pair) and unpacked on store (nibble x 0x204081).
__device__ __forceinline__ uint32_t pack32(uint4 lo, uint4 hi) {
    constexpr uint32_t W0 = 0x08040201u, W1 = 0x80402010u;  // bit weights of cells 0-3 / 4-7
    const uint32_t b3 = __builtin_amdgcn_udot4(hi.z, W0, __builtin_amdgcn_udot4(hi.w, W1, 0u, false), false);
    const uint32_t b2 = __builtin_amdgcn_udot4(hi.x, W0, __builtin_amdgcn_udot4(hi.y, W1, b3 << 8, false), false);
    const uint32_t b1 = __builtin_amdgcn_udot4(lo.z, W0, __builtin_amdgcn_udot4(lo.w, W1, b2 << 8, false), false);
    return __builtin_amdgcn_udot4(lo.x, W0, __builtin_amdgcn_udot4(lo.y, W1, b1 << 8, false), false);
}
// 16 byte cells (one 16-B load) -> 16 bits, cell k at bit k
__device__ __forceinline__ uint32_t pack16(uint4 c) {
    constexpr uint32_t W0 = 0x08040201u, W1 = 0x80402010u;
    const uint32_t b1 = __builtin_amdgcn_udot4(c.z, W0, __builtin_amdgcn_udot4(c.w, W1, 0u, false), false);
    return __builtin_amdgcn_udot4(c.x, W0, __builtin_amdgcn_udot4(c.y, W1, b1 << 8, false), false);
}
__device__ __forceinline__ uint32_t unpack_nibble(uint32_t w, int k) {
    // cells 4k..4k+3 -> bytes 0..3 (bit j of the nibble lands on bit 8j)
    return __umul24(__builtin_amdgcn_ubfe(w, 4 * k, 4), 0x204081u) & 0x01010101u;
}
__device__ __forceinline__ uint4 unpack_half(uint32_t w, int half) {  // cells 16*half .. +15
    return make_uint4(unpack_nibble(w, 4 * half), unpack_nibble(w, 4 * half + 1), unpack_nibble(w, 4 * half + 2),
                      unpack_nibble(w, 4 * half + 3));
}

}  // namespace life
