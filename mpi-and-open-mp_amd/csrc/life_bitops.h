// life_bitops.h -- bit-sliced Game-of-Life building blocks shared by the
// gfx950 kernels (life_kernels.hip, life_sweep.hip).  Device code only.
//
// One 32-cell word per lane, cell x at bit x.  A row's horizontal 3-sums are
// a 2-bit number per cell (full adder of the cell and its two neighbours);
// three rows' sums give n9 = u0 + 2*S, and the B3/S23 rule of
// life_cart.c:202-208 / life2d.c:117-123 becomes 8 v_bitop3_b32.
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

struct BitEnc {
    static constexpr int64_t kCellsPerUnit = 128;
    static constexpr uint32_t kCell0 = 1u;
    static __device__ __forceinline__ int64_t dword_of(int64_t x) { return x >> 5; }
    static __device__ __forceinline__ uint32_t pos_in_dword(int64_t x) { return (uint32_t)(x & 31); }
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
    static __device__ __forceinline__ H hsum(uint4 d, uint32_t l, uint32_t r) {
        H h;
        fa(__builtin_amdgcn_alignbit(d.x, l, 31), d.x, __builtin_amdgcn_alignbit(d.y, d.x, 1), h.s0[0], h.s1[0]);
        fa(__builtin_amdgcn_alignbit(d.y, d.x, 31), d.y, __builtin_amdgcn_alignbit(d.z, d.y, 1), h.s0[1], h.s1[1]);
        fa(__builtin_amdgcn_alignbit(d.z, d.y, 31), d.z, __builtin_amdgcn_alignbit(d.w, d.z, 1), h.s0[2], h.s1[2]);
        fa(__builtin_amdgcn_alignbit(d.w, d.z, 31), d.w, __builtin_amdgcn_alignbit(r, d.w, 1), h.s0[3], h.s1[3]);
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

// Drifting frame: the next state of cell x-1 is computed at the bit that held
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
