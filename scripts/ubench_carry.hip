// ubench_carry.hip -- issue rate of carry/compare/add-family VALU instructions
// (measurement tool, not product code): candidates for a horizontal-neighbour
// fetch without shifts (v + v + carry-in mask == (v << 1) | left lane's bit 31).
// Same method as ubench_valu.hip: 8 independent chains per lane.
//
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 scripts/ubench_carry.hip -o scripts/ubench_carry
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

constexpr int kIters = 2048;

#define KERNEL(NAME, ASM)                                                                        \
    __global__ __launch_bounds__(256) void NAME(uint32_t *out, uint32_t seed) {                 \
        uint32_t v0 = seed + threadIdx.x, v1 = v0 * 3, v2 = v0 * 5, v3 = v0 * 7, v4 = v0 * 11,   \
                 v5 = v0 * 13, v6 = v0 * 17, v7 = v0 * 19;                                       \
        uint32_t k1 = seed ^ 0x5bd1e995u;                                                        \
        uint64_t m = __builtin_amdgcn_read_exec() ^ (uint64_t)seed;                              \
        uint64_t o0, o1, o2, o3, o4, o5, o6, o7;                                                 \
        for (int i = 0; i < kIters; i++) {                                                      \
            _Pragma("unroll") for (int u = 0; u < 4; u++) {                                     \
                asm volatile(ASM : "+v"(v0), "=s"(o0) : "v"(k1), "s"(m));                        \
                asm volatile(ASM : "+v"(v1), "=s"(o1) : "v"(k1), "s"(m));                        \
                asm volatile(ASM : "+v"(v2), "=s"(o2) : "v"(k1), "s"(m));                        \
                asm volatile(ASM : "+v"(v3), "=s"(o3) : "v"(k1), "s"(m));                        \
                asm volatile(ASM : "+v"(v4), "=s"(o4) : "v"(k1), "s"(m));                        \
                asm volatile(ASM : "+v"(v5), "=s"(o5) : "v"(k1), "s"(m));                        \
                asm volatile(ASM : "+v"(v6), "=s"(o6) : "v"(k1), "s"(m));                        \
                asm volatile(ASM : "+v"(v7), "=s"(o7) : "v"(k1), "s"(m));                        \
            }                                                                                   \
        }                                                                                       \
        uint32_t r = v0 ^ v1 ^ v2 ^ v3 ^ v4 ^ v5 ^ v6 ^ v7;                                    \
        r ^= (uint32_t)(o0 ^ o1 ^ o2 ^ o3 ^ o4 ^ o5 ^ o6 ^ o7);                                  \
        if (r == 0x12345678u) out[threadIdx.x] = r;                                             \
    }

// %0 = v (in/out), %1 = sgpr pair out, %2 = vgpr k, %3 = sgpr pair in
KERNEL(k_addc, "v_addc_co_u32_e64 %0, %1, %0, %0, %3")
KERNEL(k_add_co, "v_add_co_u32_e64 %0, %1, %0, %0")
KERNEL(k_cmp, "v_cmp_gt_i32_e64 %1, %0, %2")
KERNEL(k_cmp_x, "v_cmp_gt_i32_e64 %1, %0, %2\n v_xor_b32_e32 %0, %2, %0")
KERNEL(k_cndmask, "v_cndmask_b32_e64 %0, %0, %2, %3")
KERNEL(k_add3, "v_add3_u32 %0, %0, %0, %2")
KERNEL(k_lshl_add, "v_lshl_add_u32 %0, %0, 1, %2")
KERNEL(k_xad, "v_xad_u32 %0, %0, %2, %0")
KERNEL(k_mad_u24, "v_mad_u32_u24 %0, %0, %2, %0")
KERNEL(k_perm, "v_perm_b32 %0, %0, %2, %2")
KERNEL(k_bcnt, "v_bcnt_u32_b32 %0, %0, %2")
KERNEL(k_sub, "v_sub_u32_e32 %0, %2, %0")
KERNEL(k_max, "v_max_u32_e32 %0, %2, %0")
KERNEL(k_or_e32, "v_or_b32_e32 %0, %2, %0")
KERNEL(k_not, "v_not_b32_e32 %0, %0")
KERNEL(k_lshr_e32, "v_lshrrev_b32_e32 %0, 1, %0")
KERNEL(k_ashr_e32, "v_ashrrev_i32_e32 %0, 1, %0")
KERNEL(k_addc_bitop3, "v_addc_co_u32_e64 %0, %1, %0, %0, %3\n v_bitop3_b32 %0, %0, %2, %2 bitop3:0x96")
KERNEL(k_cmp_addc, "v_cmp_gt_i32_e64 %1, %0, %2\n v_addc_co_u32_e64 %0, %1, %0, %0, %3")

typedef void (*kfn)(uint32_t *, uint32_t);

double run(kfn f, int blocks, uint32_t *out) {
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    f<<<blocks, 256>>>(out, 3);
    hipEventRecord(a);
    for (int r = 0; r < 5; r++) f<<<blocks, 256>>>(out, 3 + r);
    hipEventRecord(b);
    hipEventSynchronize(b);
    float ms;
    hipEventElapsedTime(&ms, a, b);
    const double waves = blocks * 4.0 * 5;
    return waves * kIters * 32.0 / (ms * 1e-3);  // asm statements (wave) per second
}

int main() {
    uint32_t *out;
    (void)hipMalloc(&out, 4096);
    struct {
        const char *name;
        kfn f;
    } ks[] = {{"v_addc_co_u32_e64", k_addc}, {"v_add_co_u32_e64", k_add_co}, {"v_cmp_gt_i32_e64", k_cmp},
              {"cmp+xor (2 instr)", k_cmp_x}, {"v_cndmask_b32_e64", k_cndmask}, {"v_add3_u32", k_add3},
              {"v_lshl_add_u32", k_lshl_add}, {"v_xad_u32", k_xad}, {"v_mad_u32_u24", k_mad_u24},
              {"v_perm_b32", k_perm}, {"v_bcnt_u32_b32", k_bcnt}, {"v_sub_u32_e32", k_sub},
              {"v_max_u32_e32", k_max}, {"v_or_b32_e32", k_or_e32}, {"v_not_b32_e32", k_not}, {"v_lshrrev_b32_e32", k_lshr_e32}, {"v_ashrrev_i32_e32", k_ashr_e32},
              {"addc+bitop3 (2 instr)", k_addc_bitop3}, {"cmp+addc (2 instr)", k_cmp_addc}};
    for (int wpc : {8, 16, 32}) {  // waves per CU
        const int blocks = 256 * wpc / 4;
        for (auto &k : ks) {
            const double r = run(k.f, blocks, out);
            printf("waves/CU=%2d %-24s %7.1f G asm/s  %.3f /clk/SIMD @2.4GHz\n", wpc, k.name, r / 1e9,
                   r / (1024 * 2.4e9));
        }
    }
    return 0;
}
