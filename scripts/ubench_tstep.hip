// ubench_tstep.hip -- cost decomposition of the temporal bit stencil
// (measurement tool, not product code; results are NOT checked: variants
// other than MODE 0 compute wrong cells on purpose, to price one ingredient).
//
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -I include -I mpi-and-open-mp_amd/csrc \
//         scripts/ubench_tstep.hip -o scripts/ubench_tstep
//
// MODE 0: as shipped (wave_shr/wave_shl DPP with bound_ctrl)
// MODE 1: row_shr/row_shl DPP (16-lane rows)
// MODE 2: no cross-lane move (L = v<<1, R = v>>1)
// MODE 3: as shipped, but the rule replaced by one xor (prices the rule)
#include "../mpi-and-open-mp_amd/csrc/life_kernels.hip"

#include <stdio.h>
#include <vector>

namespace life {
namespace {

template <int MODE>
__device__ __forceinline__ void hsum_m(uint32_t v, uint32_t &s0, uint32_t &s1) {
    uint32_t l, r;
    if (MODE == 1) {
        l = (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x111, 0xf, 0xf, true);
        r = (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x101, 0xf, 0xf, true);
    } else if (MODE == 2) {
        l = v;
        r = v;
    } else {
        l = left_or_zero(v);
        r = right_or_zero(v);
    }
    const uint32_t L = __builtin_amdgcn_alignbit(v, l, 31);
    const uint32_t R = __builtin_amdgcn_alignbit(r, v, 1);
    BitEnc::fa(L, v, R, s0, s1);
}

template <int NR, int MODE>
__global__ __launch_bounds__(256) void ub_kernel(TArgs a) {
    constexpr int T = NR - 2 * kTK;
    const int lane = threadIdx.x & 63;
    const int64_t wv = (int64_t)blockIdx.x * 4 + __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    if (wv >= a.first[1]) return;
    const int64_t ntx = a.tx1[0] - a.tx0[0];
    const int64_t tx = a.tx0[0] + wv % ntx, ty = a.ty0[0] + wv / ntx;
    const int64_t j = tx * 62 + lane - 1;
    int64_t jl = j % a.W;
    if (jl < 0) jl += a.W;
    const uint32_t voff = (uint32_t)(a.xoff + 4 * jl);
    int64_t y = ty * T - kTK;
    y %= a.h;
    if (y < 0) y += a.h;
    uint32_t v[NR];
#pragma unroll
    for (int r = 0; r < NR; ++r) {
        v[r] = *reinterpret_cast<const uint32_t *>(a.in + (y + a.ya) * a.pitch + voff);
        ++y;
        if (y == a.h) y = 0;
    }
    for (int g = 0; g < a.m; ++g) {
        uint32_t p0 = 0u, p1 = 0u, c0, c1;
        hsum_m<MODE>(v[0], c0, c1);
#pragma unroll
        for (int r = 0; r < NR; ++r) {
            uint32_t n0 = 0u, n1 = 0u;
            if (r + 1 < NR) hsum_m<MODE>(v[r + 1], n0, n1);
            if (MODE == 3)
                v[r] = p0 ^ c1 ^ n0;
            else
                v[r] = BitEnc::rule1(p0, p1, c0, c1, n0, n1, v[r]);
            p0 = c0;
            p1 = c1;
            c0 = n0;
            c1 = n1;
        }
    }
    const bool st = lane >= 1 && lane <= 62 && j < a.W;
    const int64_t yo = ty * T;
    uint8_t *dst = a.out + (yo + a.ya) * a.pitch + voff;
#pragma unroll
    for (int r = 0; r < T; ++r)
        if (st && yo + r < a.h) *reinterpret_cast<uint32_t *>(dst + r * a.pitch) = v[kTK + r];
}

template <int NR, int MODE>
float run(const life_layout &L, uint8_t *in, uint8_t *out, int reps) {
    const int64_t T = NR - 2 * kTK;
    TArgs a{};
    a.in = in;
    a.out = out;
    a.pitch = L.pitch;
    a.xoff = L.xoff;
    a.W = L.w / 32;
    a.h = L.h;
    a.ya = L.yapron;
    a.nreg = 1;
    a.tx0[0] = 0;
    a.tx1[0] = (a.W + 61) / 62;
    a.ty0[0] = 0;
    a.first[0] = 0;
    a.first[1] = a.tx1[0] * ((L.h + T - 1) / T);
    a.m = kTK;
    const int64_t waves = a.first[1];
    const unsigned grid = (unsigned)((waves + 3) / 4);
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    ub_kernel<NR, MODE><<<grid, 256>>>(a);
    (void)hipEventRecord(e0);
    for (int i = 0; i < reps; i++) ub_kernel<NR, MODE><<<grid, 256>>>(a);
    (void)hipEventRecord(e1);
    (void)hipEventSynchronize(e1);
    float ms = 0;
    (void)hipEventElapsedTime(&ms, e0, e1);
    return ms / reps;
}

}  // namespace
}  // namespace life

int main() {
    using namespace life;
    life_layout L;
    if (life_layout_query(65536, 65536, 1, 1, 0, LIFE_KERNEL_BIT, &L)) return 1;
    uint8_t *in, *out;
    const size_t bytes = (size_t)(L.pitch * L.rows);
    if (hipMalloc(&in, bytes) || hipMalloc(&out, bytes)) return 1;
    (void)hipMemset(in, 0x5A, bytes);
    const double cells = 65536.0 * 65536.0 * kTK;
    for (int round = 0; round < 3; round++) {
        printf("round %d\n", round);
#define RUN(NR, MODE)                                                                         \
    {                                                                                         \
        float ms = run<NR, MODE>(L, in, out, 10);                                             \
        printf("  NR=%d mode=%d  %.4f ms/launch  %.1f Gcell/s\n", NR, MODE, ms, cells / ms / 1e6); \
    }
        RUN(64, 0) RUN(64, 1) RUN(64, 2) RUN(64, 3)
        RUN(80, 0) RUN(80, 1) RUN(80, 2) RUN(80, 3)
        RUN(96, 0) RUN(96, 1) RUN(96, 2) RUN(96, 3)
    }
    return 0;
}
