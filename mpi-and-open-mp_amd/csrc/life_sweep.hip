// life_sweep.hip -- the sweep stencil: the default temporally blocked
// Game-of-Life kernel for gfx950 (replaces life_step + life_exchange of
// 6-cartesian/life_cart.c:73-74 for m <= K generations per launch).
//
// sweep_kernel<BYTE, M>: M generations per launch, one wave per (column
// strip, row segment), the generations pipelined down the segment.
//
// A wave's 64 lanes hold one 2048-cell window of a row, one 32-cell word per
// lane.  Stage g (g = 1..M, all in the wave's registers) turns rows of
// generation g-1 into rows of generation g: it keeps the horizontal sums of
// the last two rows it received and the cells of the newer one; each step it
// takes the next row, computes its sums (bit_hsum_drift), applies the rule
// to the row above and hands the result (generation g of that row) to stage
// g+1.  Stage 1 takes rows loaded from HBM, stage M's output is stored.  Stage
// g works two rows above stage g-1 (it consumes what g-1 produced the step
// BEFORE), so the M stages of one step are independent instruction streams:
// their M ds_bpermute round trips overlap, and the wave needs no LDS array
// and no barrier.
//
// Ghost work.  In x, the window's light cone: after m <= edge generations the
// cells [edge, 2048 - edge) of the window are exact; strips are placed every
// sw = 64 - edge/16 words (edge 16: 63 words, the two edge lanes own half a
// word each; edge 32: 62 words, lanes 0 and 63 own nothing).  In y: a segment
// of S owned rows reads S + 2m rows, and stage g runs only while its rows can
// still reach an owned row of stage m: m (S + m + 1) stage-steps for m S
// owned row-generations.  The launch is sized to one round of resident waves.
//
// VALU per stage-step: 12 (bit_hsum_drift 4 + rule 8, 2 of them v_alignbit);
// per step the store's realignment (1 + 1 ds_bpermute); BYTE adds pack (11)
// per loaded row and unpack (24) per stored row.
#include <stdlib.h>

#include <algorithm>

#include "life_bitops.h"
#include "life_kernels.h"

namespace life {
namespace {

struct WArgs {
    const uint8_t *in;
    uint8_t *out;
    int64_t pitch, xoff, W, h, ya;
    int64_t lo, hi;  // owned cells of a row, whole words (periodic x: shifted by edge - 32)
    int64_t seg;     // owned rows per segment
    int32_t sw, edge, wrapx, wrapy, nreg;
    // up to kMaxRegions regions of strips [sx0, sx1) x segments [q0, q1);
    // wave v belongs to the region with first[k] <= v
    int64_t sx0[kMaxRegions], sx1[kMaxRegions], q0[kMaxRegions], q1[kMaxRegions], first[kMaxRegions + 1];
};

// Build-time variants (scripts/build_variants.sh; defaults by measurement):
// LIFE_SWEEP_LEFT 0: the left neighbour word by ds_bpermute (LDS pipe), 1: by
// a DPP wave_shr move (VALU); LIFE_SWEEP_GROUP: stages whose instructions are
// interleaved op by op (instruction-level parallelism inside one wave);
// LIFE_SWEEP_OCC: resident waves per SIMD the registers are sized for (0:
// by stage count).
#ifndef LIFE_SWEEP_LEFT
#define LIFE_SWEEP_LEFT 1
#endif
#ifndef LIFE_SWEEP_GROUP
#define LIFE_SWEEP_GROUP 1
#endif
#ifndef LIFE_SWEEP_OCC
#define LIFE_SWEEP_OCC 0
#endif
// LIFE_SWEEP_PIPE 1: software-pipelined stages (the rule of stage g issued
// interleaved with the row sums of stage g-1, two independent chains).
#ifndef LIFE_SWEEP_PIPE
#define LIFE_SWEEP_PIPE 0
#endif

// Resident waves per SIMD a stage count is built for.
template <int M>
constexpr int sweep_waves_per_simd() {
    return LIFE_SWEEP_OCC > 0 ? LIFE_SWEEP_OCC : (M <= 8 ? 4 : (M <= 16 ? 3 : 2));
}

__device__ __forceinline__ uint32_t right_word(int raddr, uint32_t v) {
#if LIFE_SWEEP_LEFT == 1
    (void)raddr;
    return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x130, 0xf, 0xf, true);  // wave_shl:1, lane 63 <- 0
#else
    return bperm(raddr, v);
#endif
}
__device__ __forceinline__ uint32_t left_word(int laddr, uint32_t v) {
#if LIFE_SWEEP_LEFT == 1
    (void)laddr;
    return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x138, 0xf, 0xf, true);  // wave_shr:1, lane 0 <- 0
#else
    return bperm(laddr, v);
#endif
}

// Per-wave state.  Every array index below is a compile-time constant
// (fully unrolled stage loop, step phase T6 = t mod 6 a template argument),
// so all of it lives in VGPRs, and each value keeps its slot from step to
// step: the horizontal sums of a stage's rows rotate through 3 slots (prev,
// cur, new), the rule's own-cell words through 2.
// Buffer resource of a raw byte buffer at p (gfx9 descriptor word 3).  Loads
// and stores address a row as the resource base + this lane's constant 32-bit
// offset + a scalar row offset, so no VALU instruction computes an address.
// Records: 2^31 bytes; a lane offset of kOob is out of range, so the hardware
// drops that lane's store (and a load returns 0): every step issues the same
// unconditional memory instructions, with no exec-mask branches, and the
// waits for the prefetched rows count exactly.
constexpr uint32_t kOob = 0x80000000u;
__device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc(const void *p) {
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<void *>(p), (short)0, (int)0x7FFFFFFF, 0x00020000);
}
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

template <bool BYTE, int M>
struct Sweep {
    const uint8_t *row0;         // padded row of owned row 0 (input)
    __amdgpu_buffer_rsrc_t rin;  // loads: rows from the current base
    __amdgpu_buffer_rsrc_t rout;  // stores: from the segment's first owned row
    int32_t lsoff, ssoff;        // scalar row offsets of the next load / store
    int32_t pitch;
    int32_t n_in, S;             // window rows, owned rows
    int32_t wrapin;              // loads left before the periodic y wrap (INT32_MAX: none)
    int32_t hrows;               // periodic y: rows between wraps (h)
    uint32_t voff;               // byte offset of this lane's word in a row
    uint32_t fo;                 // store offset of the whole word (kOob: the lane does not own it)
    uint32_t ho;                 // store offset of the owned half word (kOob: none)
    uint32_t hsh;                // half-word lanes: shift that brings the owned half to bit 0
    bool halves;                 // the layout has half-word lanes (edge 16; uniform)
    int laddr, raddr;
    uint32_t hs0[3][M + 1], hs1[3][M + 1], ls[2][M + 1], o[M + 1], ring[3];

    // Loads window row `next` (live = false: past the window, the lanes read
    // nothing and get 0).
    __device__ __forceinline__ uint32_t load(bool live) {
        const int off = live ? (int)voff : (int)kOob;
        uint32_t v;
        if (BYTE) {
            const u32x4 a = __builtin_amdgcn_raw_buffer_load_b128(rin, off, lsoff, 0);
            const u32x4 b = __builtin_amdgcn_raw_buffer_load_b128(rin, live ? off + 16 : off, lsoff, 0);
            v = pack32(make_uint4(a.x, a.y, a.z, a.w), make_uint4(b.x, b.y, b.z, b.w));
        } else {
            v = __builtin_amdgcn_raw_buffer_load_b32(rin, off, lsoff, 0);
        }
        lsoff += pitch;
        if (--wrapin == 0) {  // periodic y: back to owned row 0
            rin = rsrc(row0);
            lsoff = 0;
            wrapin = hrows;
        }
        return v;
    }
    __device__ __forceinline__ void store8(uint32_t a, uint32_t b, int off, int add, bool live) {
        typedef unsigned int u32x2 __attribute__((ext_vector_type(2)));
        __builtin_amdgcn_raw_buffer_store_b64(u32x2{a, b}, rout, live ? off + add : off, ssoff, 0);
    }
    // Stores stage M's output row (live = false: not an owned row, every lane
    // is dropped).
    __device__ __forceinline__ void store(uint32_t v, bool live) {
        // after M generations of the drifting frame bit p holds cell p - M
        const uint32_t r = right_word(raddr, v);
        v = M >= 32 ? r : __builtin_amdgcn_alignbit(r, v, (uint32_t)M);
        const int f = live ? (int)fo : (int)kOob, h = live ? (int)ho : (int)kOob;
        if (BYTE) {
            // 8-byte pieces: a VALU write to the data VGPRs of a wider store
            // issued just before it corrupts the stored data on gfx950 (seen
            // here: the compiler reused the first data VGPR of a dwordx4 store
            // one instruction later and the first 4 cells came out wrong)
            const uint4 lo = unpack_half(v, 0), hi = unpack_half(v, 1);
            store8(lo.x, lo.y, f, 0, live);
            store8(lo.z, lo.w, f, 8, live);
            store8(hi.x, hi.y, f, 16, live);
            store8(hi.z, hi.w, f, 24, live);
            if (halves) {
                const uint4 e = unpack_half(v >> hsh, 0);
                store8(e.x, e.y, h, 0, live);
                store8(e.z, e.w, h, 8, live);
            }
        } else {
            __builtin_amdgcn_raw_buffer_store_b32(v, rout, f, ssoff, 0);
            if (halves) __builtin_amdgcn_raw_buffer_store_b16((unsigned short)(v >> hsh), rout, h, ssoff, 0);
        }
        if (live) ssoff += pitch;
    }
    // Step t (T6 = t mod 6): stage g turns window row t - 2g + 1 of
    // generation g-1 into row t - 2g of generation g; it is active for t in
    // [3g - 2, n_in + g).  Descending g: stage g reads o[g-1] before stage g-1
    // overwrites it.  Slots: sums of the stage's rows r-1, r, r+1 in
    // hs[T6 % 3], hs[(T6+1) % 3], hs[(T6+2) % 3]; own cells of row r in
    // ls[T6 % 2], of row r+1 in ls[(T6+1) % 2]; stage 1's input row t-1 in
    // ring[(T6+2) % 3], the slot the load of row t+2 then refills.  STEADY:
    // every stage active, a row stored and a row loaded (the loop bounds
    // guarantee it), so the step has no branch and the waits for the
    // prefetched loads are exact.
    template <int T6, bool STEADY>
    __device__ __forceinline__ void step(int32_t t) {
        constexpr int P = T6 % 3, C = (T6 + 1) % 3, N = (T6 + 2) % 3, LC = T6 % 2, LN = (T6 + 1) % 2;
#if LIFE_SWEEP_PIPE
        if (true) {
            // a(g): stage g's row sums; b(g): its rule.  Order a(M), [b(M) | a(M-1)],
            // ..., [b(2) | a(1)], b(1): the same reads-before-writes as stage order.
            uint32_t pin = 0u, pl = 0u;  // a(g) in flight: input word, left word
            auto a_begin = [&](int g) {
                pin = g == 1 ? ring[N] : o[g - 1];
                pl = left_word(laddr, pin);
            };
            auto a_end = [&](int g) {
                const uint32_t L = __builtin_amdgcn_alignbit(pin, pl, 31), LL = __builtin_amdgcn_alignbit(pin, pl, 30);
                hs0[N][g] = b3<kXor3>(LL, L, pin);
                hs1[N][g] = b3<kMaj>(LL, L, pin);
                ls[LN][g] = L;
            };
            auto act = [&](int g) { return g >= 1 && (STEADY || (t >= 3 * g - 2 && t < n_in + g)); };
            if (act(M)) {
                a_begin(M);
                a_end(M);
            }
#pragma unroll
            for (int g = M; g >= 1; --g) {
                const bool an = act(g - 1), bn = act(g);
                if (an) a_begin(g - 1);
                uint32_t u0 = 0, k0 = 0, v0 = 0, v1 = 0;
                if (bn) {
                    u0 = b3<kXor3>(hs0[P][g], hs0[C][g], hs0[N][g]);
                    k0 = b3<kMaj>(hs0[P][g], hs0[C][g], hs0[N][g]);
                    v0 = b3<kXor3>(hs1[P][g], hs1[C][g], hs1[N][g]);
                    v1 = b3<kMaj>(hs1[P][g], hs1[C][g], hs1[N][g]);
                }
                if (an) a_end(g - 1);
                if (bn) {
                    const uint32_t e1 = b3<kEq1>(v0, k0, v1), e2 = b3<kEq2>(v0, k0, v1);
                    o[g] = b3<kAndOr>(b3<kMux>(u0, e1, e2), u0, ls[LC][g]);
                }
            }
        } else
#endif
        {
        constexpr int G = LIFE_SWEEP_GROUP;
        // stages in groups of G, descending; inside a group every operation
        // runs for all its stages before the next (all inputs are read before
        // any output is written, so stage g still reads o[g-1] first)
#pragma unroll
        for (int g0 = M; g0 >= 1; g0 -= G) {
            bool act[G];
            uint32_t in[G], l[G], L[G], LL[G];
#pragma unroll
            for (int i = 0; i < G; ++i) {
                const int g = g0 - i;
                act[i] = g >= 1 && (STEADY || (t >= 3 * g - 2 && t < n_in + g));
                in[i] = g < 1 ? 0u : (g == 1 ? ring[N] : o[g - 1]);
            }
#pragma unroll
            for (int i = 0; i < G; ++i)
                if (act[i]) l[i] = left_word(laddr, in[i]);
#pragma unroll
            for (int i = 0; i < G; ++i)
                if (act[i]) {
                    L[i] = __builtin_amdgcn_alignbit(in[i], l[i], 31);
                    LL[i] = __builtin_amdgcn_alignbit(in[i], l[i], 30);
                }
#pragma unroll
            for (int i = 0; i < G; ++i)
                if (act[i]) {
                    const int g = g0 - i;
                    hs0[N][g] = b3<kXor3>(LL[i], L[i], in[i]);
                    hs1[N][g] = b3<kMaj>(LL[i], L[i], in[i]);
                    ls[LN][g] = L[i];
                }
            uint32_t u0[G], k0[G], v0[G], v1[G], e1[G], e2[G];
#pragma unroll
            for (int i = 0; i < G; ++i)
                if (act[i]) {
                    const int g = g0 - i;
                    u0[i] = b3<kXor3>(hs0[P][g], hs0[C][g], hs0[N][g]);
                    k0[i] = b3<kMaj>(hs0[P][g], hs0[C][g], hs0[N][g]);
                }
#pragma unroll
            for (int i = 0; i < G; ++i)
                if (act[i]) {
                    const int g = g0 - i;
                    v0[i] = b3<kXor3>(hs1[P][g], hs1[C][g], hs1[N][g]);
                    v1[i] = b3<kMaj>(hs1[P][g], hs1[C][g], hs1[N][g]);
                }
#pragma unroll
            for (int i = 0; i < G; ++i)
                if (act[i]) {
                    e1[i] = b3<kEq1>(v0[i], k0[i], v1[i]);
                    e2[i] = b3<kEq2>(v0[i], k0[i], v1[i]);
                }
#pragma unroll
            for (int i = 0; i < G; ++i)
                if (act[i]) {
                    const int g = g0 - i;
                    o[g] = b3<kAndOr>(b3<kMux>(u0[i], e1[i], e2[i]), u0[i], ls[LC][g]);
                }
        }
        }
        const int32_t r = t - 2 * M;  // window row stage M produced
        store(o[M], STEADY || (r >= M && r < M + S));
        ring[N] = load(STEADY || t + 2 < n_in);
    }
    template <bool STEADY>
    __device__ __forceinline__ void six(int32_t t) {
        step<0, STEADY>(t);
        step<1, STEADY>(t + 1);
        step<2, STEADY>(t + 2);
        step<3, STEADY>(t + 3);
        step<4, STEADY>(t + 4);
        step<5, STEADY>(t + 5);
    }
};

template <bool BYTE, int M>
__global__ __launch_bounds__(256, sweep_waves_per_simd<M>()) void sweep_kernel(WArgs a) {
    static_assert(M >= 1 && M <= 32, "stages");
    const int lane = threadIdx.x & 63;
    const int64_t wv = (int64_t)blockIdx.x * 4 + __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    if (wv >= a.first[a.nreg]) return;  // whole wave (no barrier in this kernel)
    int k = 0;
    while (k + 1 < a.nreg && wv >= a.first[k + 1]) ++k;
    // the waves of a workgroup are vertically adjacent segments of one strip
    // (their ghost rows meet in one XCD's L2)
    const int64_t rr = wv - a.first[k], nq = a.q1[k] - a.q0[k];
    const int64_t s = a.sx0[k] + rr / nq, q = a.q0[k] + rr % nq;
    const int64_t y0 = q * a.seg;
    const int64_t S = a.h - y0 < a.seg ? a.h - y0 : a.seg;  // owned rows [y0, y0 + S)
    if (S <= 0) return;
    const int64_t B = s * a.sw - 1;  // word of lane 0
    const int64_t j = B + lane;
    int64_t jl = j;
    if (a.wrapx) {
        jl %= a.W;
        if (jl < 0) jl += a.W;
    } else {
        jl = j > a.W ? a.W : j;  // words -1 .. W hold cells / apron; beyond: clamp (never stored)
    }
    Sweep<BYTE, M> w;
    w.voff = (uint32_t)(a.xoff + (BYTE ? 32 : 4) * jl);
    w.laddr = ((lane - 1) & 63) << 2;
    w.raddr = ((lane + 1) & 63) << 2;
    {
        // owned cells of this lane's word: the window's exact cells inside
        // the row's owned range (a whole word, one half of it, or nothing)
        const int64_t clo = 32 * B + a.edge > a.lo ? 32 * B + a.edge : a.lo;
        const int64_t chi = 32 * B + 2048 - a.edge < a.hi ? 32 * B + 2048 - a.edge : a.hi;
        const int64_t ca = 32 * j > clo ? 32 * j : clo, cb = 32 * j + 32 < chi ? 32 * j + 32 : chi;
        const bool upper = ca != 32 * j;
        w.fo = cb - ca == 32 ? w.voff : kOob;
        w.ho = cb - ca == 16 ? w.voff + (upper ? (BYTE ? 16u : 2u) : 0u) : kOob;
        w.hsh = upper ? 16u : 0u;
        w.halves = a.edge == 16;
    }
    w.pitch = (int32_t)a.pitch;
    w.S = (int32_t)S;
    w.n_in = (int32_t)(S + 2 * M);
    w.row0 = a.in + a.ya * a.pitch;
    int64_t yl = y0 - M;  // first window row
    w.wrapin = w.hrows = INT32_MAX;
    if (a.wrapy) {
        yl %= a.h;
        if (yl < 0) yl += a.h;
        w.wrapin = (int32_t)(a.h - yl);
        w.hrows = (int32_t)a.h;
    }
    w.rin = rsrc(w.row0 + yl * a.pitch);
    w.rout = rsrc(a.out + (a.ya + y0) * a.pitch);
    w.lsoff = w.ssoff = 0;
#pragma unroll
    for (int g = 0; g <= M; ++g) {
        w.o[g] = 0u;
#pragma unroll
        for (int i = 0; i < 3; ++i) w.hs0[i][g] = w.hs1[i][g] = 0u;
        w.ls[0][g] = w.ls[1][g] = 0u;
    }
    w.ring[2] = 0u;
    w.ring[0] = w.load(true);
    w.ring[1] = w.load(true);  // n_in >= 3
    // Three loops, each starting on a multiple of 6 so the slots line up:
    // ramp up, the steady state (every stage active, a row stored and one
    // loaded each step: t in [3M, n_in - 2)), ramp down.
    const int32_t tend = w.n_in + M;
    const int32_t s0 = (3 * M + 5) / 6 * 6;
    const int32_t s1 = w.n_in - 2 - s0 >= 6 ? s0 + (w.n_in - 2 - s0) / 6 * 6 : s0;
    int32_t t = 0;
    for (; t < s0 && t < tend; t += 6) w.template six<false>(t);
    for (; t < s1; t += 6) w.template six<true>(t);
    for (; t < tend; t += 6) w.template six<false>(t);
}

int device_cus() {
    static int cus[64] = {0};
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return 256;
    if (!cus[dev]) {
        int n = 0;
        if (hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n <= 0) n = 256;
        cus[dev] = n;
    }
    return cus[dev];
}

// Stage counts with a sweep_kernel instance (a launch of m generations runs
// the instance with exactly m stages).
#ifndef LIFE_SWEEP_STAGES
#define LIFE_SWEEP_STAGES(X) X(1) X(2) X(4) X(8) X(12) X(16)
#endif

template <bool BYTE>
hipError_t launch_sw(const WArgs &a, int m, unsigned grid, hipStream_t s) {
    switch (m) {
#define LIFE_SW_CASE(N) \
    case N: sweep_kernel<BYTE, N><<<grid, 256, 0, s>>>(a); break;
        LIFE_SWEEP_STAGES(LIFE_SW_CASE)
#undef LIFE_SW_CASE
    default: return hipErrorInvalidValue;
    }
    return hipGetLastError();
}

int waves_per_simd(int m) { return m <= 8 ? 4 : (m <= 16 ? 3 : 2); }

int64_t sweep_target_waves(int m) {
    static const int64_t env = [] {
        const char *e = getenv("LIFE_SWEEP_WAVES");
        return e ? (int64_t)atoll(e) : (int64_t)0;
    }();
    return env > 0 ? env : (int64_t)waves_per_simd(m) * 4 * device_cus();
}
}  // namespace

bool sweep_has(int m) {
    switch (m) {
#define LIFE_SW_HAS(N) case N:
        LIFE_SWEEP_STAGES(LIFE_SW_HAS)
#undef LIFE_SW_HAS
        return true;
    default: return false;
    }
}

namespace {
constexpr int max_instance() {
    int m = 0;
#define LIFE_SW_MAX(N) m = N > m ? N : m;
    LIFE_SWEEP_STAGES(LIFE_SW_MAX)
#undef LIFE_SW_MAX
    return m;
}
}  // namespace

int sweep_max_stages(const life_layout &L) {
    return L.generations_per_exchange < max_instance() ? L.generations_per_exchange : max_instance();
}

SweepGeom sweep_geom(const life_layout &L, bool wrapx) {
    SweepGeom g{};
    const int K = sweep_max_stages(L);
    g.edge = L.generations_per_exchange <= 16 ? 16 : 32;
    g.sw = 64 - g.edge / 16;
    const int64_t W = (L.w + 31) / 32;
    g.lo = wrapx ? g.edge - 32 : 0;
    g.hi = g.lo + 32 * W;
    // strip s owns window cells [32 (s sw - 1) + edge, 32 (s sw - 1) + 2048 - edge)
    g.nstrips = 1;
    while (32 * (g.nstrips * g.sw - g.sw - 1) + 2048 - g.edge < g.hi) ++g.nstrips;
    // one round of resident waves; segments of at least 4K rows (the ramp of
    // the stage pipeline costs about K + 1 rows of work per segment)
    int64_t nseg = sweep_target_waves(K) / g.nstrips;
    const int64_t cap = L.h / (4 * (int64_t)K);
    if (nseg > cap) nseg = cap;
    // a window's rows are addressed by 32-bit scalar offsets from one base:
    // keep (seg + 2K) rows under 1 GiB
    const int64_t maxseg = std::max<int64_t>(1, ((int64_t)1 << 30) / L.pitch - 2 * (int64_t)K);
    nseg = std::max<int64_t>(nseg, (L.h + maxseg - 1) / maxseg);
    if (nseg < 1) nseg = 1;
    g.seg = (L.h + nseg - 1) / nseg;
    g.nseg = (L.h + g.seg - 1) / g.seg;
    return g;
}

double sweep_valu_per_lane(const SweepGeom &g, const TileRegion &r, int64_t h, int m, bool byte) {
    double v = 0.0;
    for (int64_t q = r.ty0; q < r.ty1; ++q) {
        const int64_t S = std::min(g.seg, h - q * g.seg);
        if (S <= 0) continue;
        // stage-steps x 12, the store's realignment, byte pack / unpack
        v += 12.0 * (double)m * (double)(S + m + 1) + (double)S +
             (byte ? 11.0 * (double)(S + 2 * m) + 24.0 * (double)S : 0.0);
    }
    return v * (double)(r.tx1 - r.tx0);
}

hipError_t launch_sweep(const life_layout &L, const SweepGeom &g, const uint8_t *in, uint8_t *out,
                        const TileRegion *r, int nreg, int m, Wrap wrap, hipStream_t s) {
    if (nreg < 0 || nreg > kMaxRegions || m < 1 || m > sweep_max_stages(L) || !sweep_has(m) || m > g.edge ||
        (!wrap.y && L.yapron < m) || in == out)
        return hipErrorInvalidValue;
    WArgs a;
    a.in = in;
    a.out = out;
    a.pitch = L.pitch;
    a.xoff = L.xoff;
    a.W = (L.w + 31) / 32;
    a.h = L.h;
    a.ya = L.yapron;
    a.lo = g.lo;
    a.hi = g.hi;
    a.seg = g.seg;
    a.sw = (int32_t)g.sw;
    a.edge = g.edge;
    a.wrapx = wrap.x ? 1 : 0;
    a.wrapy = wrap.y ? 1 : 0;
    a.nreg = 0;
    a.first[0] = 0;
    for (int k = 0; k < nreg; k++) {
        if (r[k].tx1 <= r[k].tx0 || r[k].ty1 <= r[k].ty0) continue;
        const int n = a.nreg++;
        a.sx0[n] = r[k].tx0;
        a.sx1[n] = r[k].tx1;
        a.q0[n] = r[k].ty0;
        a.q1[n] = r[k].ty1;
        a.first[n + 1] = a.first[n] + (r[k].tx1 - r[k].tx0) * (r[k].ty1 - r[k].ty0);
    }
    if (a.nreg == 0) return hipSuccess;
    const unsigned grid = (unsigned)((a.first[a.nreg] + 3) / 4);  // 4 independent waves per workgroup
    return L.kernel == LIFE_KERNEL_BIT ? launch_sw<false>(a, m, grid, s) : launch_sw<true>(a, m, grid, s);
}

}  // namespace life
