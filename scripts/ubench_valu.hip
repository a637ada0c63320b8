// ubench_valu.hip -- issue rate of candidate VALU instructions for the bit
// stencil (measurement tool, not product code).  Each kernel runs 8
// independent dependency chains per lane of one instruction; prints
// wave-instructions per clock per SIMD assuming 2.4 GHz (the clock actually
// held is lower under load: MI355X_MICROARCH.md "DVFS give-back").
//
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 scripts/ubench_valu.hip -o scripts/ubench_valu
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

constexpr int kIters = 2048;

#define CH8(X) X(0) X(1) X(2) X(3) X(4) X(5) X(6) X(7)

#define KERNEL(NAME, ASM)                                                                        \
    __global__ __launch_bounds__(256) void NAME(uint32_t *out, uint32_t seed) {                 \
        uint32_t v0 = seed + threadIdx.x, v1 = v0 * 3, v2 = v0 * 5, v3 = v0 * 7, v4 = v0 * 11,   \
                 v5 = v0 * 13, v6 = v0 * 17, v7 = v0 * 19;                                       \
        uint32_t k1 = seed ^ 0x5bd1e995u, k2 = seed + 0x1234567u;                                \
        for (int i = 0; i < kIters; i++) {                                                      \
            _Pragma("unroll") for (int u = 0; u < 4; u++) {                                     \
                asm volatile(ASM : "+v"(v0) : "v"(k1), "v"(k2));                                 \
                asm volatile(ASM : "+v"(v1) : "v"(k1), "v"(k2));                                 \
                asm volatile(ASM : "+v"(v2) : "v"(k1), "v"(k2));                                 \
                asm volatile(ASM : "+v"(v3) : "v"(k1), "v"(k2));                                 \
                asm volatile(ASM : "+v"(v4) : "v"(k1), "v"(k2));                                 \
                asm volatile(ASM : "+v"(v5) : "v"(k1), "v"(k2));                                 \
                asm volatile(ASM : "+v"(v6) : "v"(k1), "v"(k2));                                 \
                asm volatile(ASM : "+v"(v7) : "v"(k1), "v"(k2));                                 \
            }                                                                                   \
        }                                                                                       \
        uint32_t r = v0 ^ v1 ^ v2 ^ v3 ^ v4 ^ v5 ^ v6 ^ v7;                                    \
        if (r == 0x12345678u) out[threadIdx.x] = r;                                             \
    }

KERNEL(k_bitop3, "v_bitop3_b32 %0, %0, %1, %2 bitop3:0x96")
KERNEL(k_or3, "v_or3_b32 %0, %0, %1, %2")
KERNEL(k_and_or, "v_and_or_b32 %0, %0, %1, %2")
KERNEL(k_bfi, "v_bfi_b32 %0, %0, %1, %2")
KERNEL(k_alignbit, "v_alignbit_b32 %0, %0, %1, 31")
KERNEL(k_lshl_or, "v_lshl_or_b32 %0, %0, 1, %1")
KERNEL(k_xor_e32, "v_xor_b32_e32 %0, %1, %0")
KERNEL(k_and_e32, "v_and_b32_e32 %0, %1, %0")
KERNEL(k_xor_e64, "v_xor_b32_e64 %0, %1, %0")
KERNEL(k_lshl_e32, "v_lshlrev_b32_e32 %0, 1, %0")
KERNEL(k_add_e32, "v_add_u32_e32 %0, %1, %0")
KERNEL(k_mov_dpp, "v_mov_b32_dpp %0, %0 wave_shr:1 row_mask:0xf bank_mask:0xf bound_ctrl:0")
KERNEL(k_xor_dpp, "v_xor_b32_dpp %0, %0, %1 wave_shr:1 row_mask:0xf bank_mask:0xf bound_ctrl:0")
KERNEL(k_mov_dpp_row, "v_mov_b32_dpp %0, %0 row_shr:1 row_mask:0xf bank_mask:0xf bound_ctrl:0")
KERNEL(k_fma_f32, "v_fma_f32 %0, %0, %1, %2")
KERNEL(k_pk_add_u16, "v_pk_add_u16 %0, %0, %1")

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
    return waves * kIters * 32.0 / (ms * 1e-3);  // wave-instructions per second
}

int main() {
    uint32_t *out;
    (void)hipMalloc(&out, 4096);
    struct {
        const char *name;
        kfn f;
    } ks[] = {{"v_bitop3_b32", k_bitop3},   {"v_or3_b32", k_or3},
              {"v_and_or_b32", k_and_or},   {"v_bfi_b32", k_bfi},           {"v_alignbit_b32", k_alignbit},
              {"v_lshl_or_b32", k_lshl_or}, {"v_xor_b32_e32", k_xor_e32},   {"v_and_b32_e32", k_and_e32},
              {"v_xor_b32_e64", k_xor_e64}, {"v_lshlrev_b32_e32", k_lshl_e32}, {"v_add_u32_e32", k_add_e32},
              {"v_mov_b32_dpp wave_shr", k_mov_dpp}, {"v_xor_b32_dpp wave_shr", k_xor_dpp},
              {"v_mov_b32_dpp row_shr", k_mov_dpp_row}, {"v_fma_f32", k_fma_f32}, {"v_pk_add_u16", k_pk_add_u16}};
    for (int wpc : {4, 8, 16, 32}) {  // waves per CU
        const int blocks = 256 * wpc / 4;
        for (auto &k : ks) {
            const double r = run(k.f, blocks, out);
            printf("waves/CU=%2d %-26s %7.1f G wave-instr/s  %.3f /clk/SIMD @2.4GHz\n", wpc, k.name, r / 1e9,
                   r / (1024 * 2.4e9));
        }
    }
    return 0;
}
