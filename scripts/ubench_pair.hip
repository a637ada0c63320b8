// ubench_pair.hip -- prices the bit stencil's generation loop in registers
// (no HBM, no cross-wave exchange) for two register layouts of a row
// (measurement tool, not product code):
//
//   word : one 32-cell word per lane and row (the shipped tiles): per row and
//          generation 1 DPP + 1 ds_bpermute + 2 v_alignbit + 10 v_bitop3
//   pair : two words per lane and row holding the lane's 64 cells
//          bit-interleaved (E = even cells, O = odd cells): the right
//          neighbour of an even cell is the odd word's same bit, so per PAIR
//          of words 2 v_alignbit + 20 v_bitop3 and two neighbour fetches
//          (pair_dpp: DPP + ds_bpermute; pair_bp: 2 ds_bpermute; pair_1bp:
//          1 ds_bpermute, the other neighbour the lane's own word; pair_nf: no
//          fetch at all -- both neighbour words the lane's own: wrong cells,
//          the same VALU, the LDS pipe's share of the loop)
//
// Every variant runs the same number of word-generations per lane; the
// printed figure is ns per word-row-generation per SIMD (lower is better).
//
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 scripts/ubench_pair.hip -o scripts/ubench_pair
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

#include "../mpi-and-open-mp_amd/csrc/life_bitops.h"

using namespace life;

__device__ __forceinline__ uint32_t left_or_zero(uint32_t v) {
    return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x138, 0xf, 0xf, true);
}

template <int R>
__global__ __launch_bounds__(512, 6) void k_word(uint32_t *out, uint32_t seed, int gens) {
    const int lane = threadIdx.x & 63;
    uint32_t v[R];
#pragma unroll
    for (int r = 0; r < R; ++r) v[r] = (seed + threadIdx.x * 2654435761u) ^ (r * 0x9E3779B9u);
    const int raddr = ((lane + 1) & 63) << 2;
    for (int g = 0; g < gens; ++g) {
        auto hsum = [&](uint32_t x, uint32_t &s0, uint32_t &s1) {
            const uint32_t r = bperm(raddr, x);
            const uint32_t l = left_or_zero(x);
            BitEnc::fa(__builtin_amdgcn_alignbit(x, l, 31), x, __builtin_amdgcn_alignbit(r, x, 1), s0, s1);
        };
        uint32_t t0, t1, p0, p1, c0, c1;
        hsum(v[R - 1], p0, p1);
        hsum(v[0], t0, t1);
        c0 = t0;
        c1 = t1;
        uint32_t cv = v[0];
#pragma unroll
        for (int r = 0; r < R; ++r) {
            uint32_t n0, n1;
            if (r + 1 < R) hsum(v[r + 1], n0, n1);
            else { n0 = t0; n1 = t1; }
            const uint32_t nv = r + 1 < R ? v[r + 1] : 0u;
            v[r] = BitEnc::rule1(p0, p1, c0, c1, n0, n1, cv);
            cv = nv;
            p0 = c0; p1 = c1; c0 = n0; c1 = n1;
        }
    }
    uint32_t x = 0;
#pragma unroll
    for (int r = 0; r < R; ++r) x ^= v[r];
    if (x == 0x12345678u) out[threadIdx.x] = x;
}

// F: 1 both neighbour words by ds_bpermute, 0 the left one by DPP, 2 neither
// (own words), 3 the right one only
template <int R, int F>
__global__ __launch_bounds__(512, 6) void k_pair(uint32_t *out, uint32_t seed, int gens) {
    const int lane = threadIdx.x & 63;
    uint32_t e[R], o[R];
#pragma unroll
    for (int r = 0; r < R; ++r) {
        e[r] = (seed + threadIdx.x * 2654435761u) ^ (r * 0x9E3779B9u);
        o[r] = e[r] * 0x85EBCA6Bu;
    }
    const int raddr = ((lane + 1) & 63) << 2, laddr = ((lane - 1) & 63) << 2;
    for (int g = 0; g < gens; ++g) {
        // even cell 2i: O[i-1] + E[i] + O[i]; odd cell 2i+1: E[i] + O[i] + E[i+1]
        auto hsum = [&](uint32_t E, uint32_t O, uint32_t &e0, uint32_t &e1, uint32_t &o0, uint32_t &o1) {
            const uint32_t en = (F == 0 || F == 1 || F == 3) ? bperm(raddr, E) : O;
            const uint32_t op = F == 1 ? bperm(laddr, O) : F == 0 ? left_or_zero(O) : E;
            const uint32_t osh = __builtin_amdgcn_alignbit(O, op, 31);
            const uint32_t esh = __builtin_amdgcn_alignbit(en, E, 1);
            BitEnc::fa(osh, E, O, e0, e1);
            BitEnc::fa(E, O, esh, o0, o1);
        };
        uint32_t te0, te1, to0, to1, pe0, pe1, po0, po1, ce0, ce1, co0, co1;
        hsum(e[R - 1], o[R - 1], pe0, pe1, po0, po1);
        hsum(e[0], o[0], te0, te1, to0, to1);
        ce0 = te0; ce1 = te1; co0 = to0; co1 = to1;
        uint32_t cve = e[0], cvo = o[0];
#pragma unroll
        for (int r = 0; r < R; ++r) {
            uint32_t ne0, ne1, no0, no1;
            if (r + 1 < R) hsum(e[r + 1], o[r + 1], ne0, ne1, no0, no1);
            else { ne0 = te0; ne1 = te1; no0 = to0; no1 = to1; }
            const uint32_t nve = r + 1 < R ? e[r + 1] : 0u, nvo = r + 1 < R ? o[r + 1] : 0u;
            e[r] = BitEnc::rule1(pe0, pe1, ce0, ce1, ne0, ne1, cve);
            o[r] = BitEnc::rule1(po0, po1, co0, co1, no0, no1, cvo);
            cve = nve; cvo = nvo;
            pe0 = ce0; pe1 = ce1; ce0 = ne0; ce1 = ne1;
            po0 = co0; po1 = co1; co0 = no0; co1 = no1;
        }
    }
    uint32_t x = 0;
#pragma unroll
    for (int r = 0; r < R; ++r) x ^= e[r] ^ o[r];
    if (x == 0x12345678u) out[threadIdx.x] = x;
}

typedef void (*kfn)(uint32_t *, uint32_t, int);

int main() {
    uint32_t *out;
    (void)hipMalloc(&out, 4096);
    int dev = 0, cus = 0;
    (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
    struct K {
        const char *name;
        kfn f;
        int words;  // words per lane and generation
    } ks[] = {{"word R48", k_word<48>, 48},          {"word R24", k_word<24>, 24},
              {"pair_dpp R24", k_pair<24, 0>, 48}, {"pair_bp R24", k_pair<24, 1>, 48},
              {"pair_dpp R16", k_pair<16, 0>, 32}, {"pair_bp R16", k_pair<16, 1>, 32},
              {"pair_bp R32", k_pair<32, 1>, 64}, {"pair_1bp R24", k_pair<24, 3>, 48},
              {"pair_nf R24", k_pair<24, 2>, 48}, {"pair_bp R24 again", k_pair<24, 1>, 48}};
    const int gens = 200;
    for (const K &k : ks) {
        int per = 0;
        (void)hipOccupancyMaxActiveBlocksPerMultiprocessor(&per, (const void *)k.f, 512, 0);
        hipFuncAttributes at{};
        (void)hipFuncGetAttributes(&at, (const void *)k.f);
        const int blocks = cus * (per > 0 ? per : 1) * 4;
        hipEvent_t a, b;
        (void)hipEventCreate(&a);
        (void)hipEventCreate(&b);
        k.f<<<blocks, 512>>>(out, 1, gens);
        (void)hipEventRecord(a);
        for (int r = 0; r < 5; r++) k.f<<<blocks, 512>>>(out, 2 + r, gens);
        (void)hipEventRecord(b);
        (void)hipEventSynchronize(b);
        float ms;
        (void)hipEventElapsedTime(&ms, a, b);
        const double wave_words = (double)blocks * 8 * 5 * gens * k.words;  // wave-word-generations
        const double simds = cus * 4.0;
        printf("%-14s vgpr %3d wg/CU %d  %.3f ms  %.3f ns/word-gen/SIMD  %.1f Tcell-gen/s\n", k.name,
               at.numRegs, per, ms, ms * 1e6 * simds / wave_words, wave_words * 64 * 32 / (ms * 1e-3) / 1e12);
    }
    return 0;
}
