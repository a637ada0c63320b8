// ubench_bank.hip -- does a VGPR bank conflict among the three sources of
// v_bitop3_b32 cost issue cycles on gfx950?  (measurement tool, not product
// code).  Eight independent chains per lane, explicit registers v40..v63
// (bank = register index mod 4); the chain register D, the sources X and Y:
//
//   distinct : D, X, Y in three different banks
//   pair     : X in D's bank, Y in another
//   same     : D, X, Y all in one bank
//
// and the same three patterns for v_xor_b32 (two sources).  Prints
// wave-instructions per clock per SIMD at the clock GRBM would report is
// not known here, so compare the variants with each other (same occupancy,
// same clock class).
//
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 scripts/ubench_bank.hip -o scripts/ubench_bank
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

constexpr int kIters = 4096;

#define CLOB                                                                                                 \
    "v40", "v41", "v42", "v43", "v44", "v45", "v46", "v47", "v48", "v49", "v50", "v51", "v52", "v53", "v54", \
        "v55", "v56", "v57", "v58", "v59", "v60", "v61", "v62", "v63"

// eight chains: D = v40..v47 (banks 0,1,2,3,0,1,2,3); sources from v48..v63
#define INIT                                                                                                 \
    "v_mov_b32 v40, %1\n v_mov_b32 v41, %1\n v_mov_b32 v42, %1\n v_mov_b32 v43, %1\n"                       \
    "v_mov_b32 v44, %1\n v_mov_b32 v45, %1\n v_mov_b32 v46, %1\n v_mov_b32 v47, %1\n"                       \
    "v_mov_b32 v48, %1\n v_mov_b32 v49, %1\n v_mov_b32 v50, %1\n v_mov_b32 v51, %1\n"                       \
    "v_mov_b32 v52, %1\n v_mov_b32 v53, %1\n v_mov_b32 v54, %1\n v_mov_b32 v55, %1\n"                       \
    "v_mov_b32 v56, %1\n v_mov_b32 v57, %1\n v_mov_b32 v58, %1\n v_mov_b32 v59, %1\n"                       \
    "v_mov_b32 v60, %1\n v_mov_b32 v61, %1\n v_mov_b32 v62, %1\n v_mov_b32 v63, %1\n"

#define BODY_KERNEL(NAME, B8)                                                                                \
    __global__ __launch_bounds__(256) void NAME(uint32_t *out, uint32_t seed) {                              \
        uint32_t r;                                                                                          \
        asm volatile(INIT ::"v"(0), "v"(seed + threadIdx.x) : CLOB);                                         \
        for (int i = 0; i < kIters; i++) asm volatile(B8 B8 B8 B8 ::: CLOB);                                 \
        asm volatile("v_xor_b32 %0, v40, v41\n v_bitop3_b32 %0, %0, v42, v43 bitop3:0x96\n"              \
                     " v_bitop3_b32 %0, %0, v44, v45 bitop3:0x96\n v_bitop3_b32 %0, %0, v46, v47 bitop3:0x96" \
                     : "=v"(r)::CLOB);                                                                       \
        if (r == 0x12345678u) out[threadIdx.x] = r;                                                          \
    }

// v_bitop3 D, D, X, Y for the eight chains
#define B3(D, X, Y) "v_bitop3_b32 v" #D ", v" #D ", v" #X ", v" #Y " bitop3:0x96\n"
#define XO(D, X) "v_xor_b32 v" #D ", v" #X ", v" #D "\n"

// distinct banks: D bank b, X bank b+1, Y bank b+2
#define B8_DIST B3(40, 49, 58) B3(41, 50, 59) B3(42, 51, 56) B3(43, 48, 57) B3(44, 53, 62) B3(45, 54, 63) B3(46, 55, 60) B3(47, 52, 61)
// X shares D's bank, Y in another
#define B8_PAIR B3(40, 48, 57) B3(41, 49, 58) B3(42, 50, 59) B3(43, 51, 56) B3(44, 52, 61) B3(45, 53, 62) B3(46, 54, 63) B3(47, 55, 60)
// all three in D's bank
#define B8_SAME B3(40, 48, 56) B3(41, 49, 57) B3(42, 50, 58) B3(43, 51, 59) B3(44, 52, 60) B3(45, 53, 61) B3(46, 54, 62) B3(47, 55, 63)
#define X8_DIST XO(40, 49) XO(41, 50) XO(42, 51) XO(43, 48) XO(44, 53) XO(45, 54) XO(46, 55) XO(47, 52)
#define X8_SAME XO(40, 48) XO(41, 49) XO(42, 50) XO(43, 51) XO(44, 52) XO(45, 53) XO(46, 54) XO(47, 55)

BODY_KERNEL(k_b3_dist, B8_DIST)
BODY_KERNEL(k_b3_pair, B8_PAIR)
BODY_KERNEL(k_b3_same, B8_SAME)
BODY_KERNEL(k_xor_dist, X8_DIST)
BODY_KERNEL(k_xor_same, X8_SAME)

typedef void (*kfn)(uint32_t *, uint32_t);

int main() {
    uint32_t *out;
    (void)hipMalloc(&out, 4096);
    int cus = 0;
    (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
    struct K {
        const char *name;
        kfn f;
    } ks[] = {{"bitop3 distinct banks", k_b3_dist}, {"bitop3 two in a bank", k_b3_pair},
              {"bitop3 all one bank", k_b3_same},   {"xor distinct banks", k_xor_dist},
              {"xor same bank", k_xor_same}};
    for (int wpc : {8, 16, 32}) {  // waves per CU
        const int blocks = cus * wpc / 4;
        for (int rep = 0; rep < 2; rep++)
            for (const K &k : ks) {
                hipEvent_t a, b;
                (void)hipEventCreate(&a);
                (void)hipEventCreate(&b);
                k.f<<<blocks, 256>>>(out, 1);
                (void)hipEventRecord(a);
                for (int r = 0; r < 5; r++) k.f<<<blocks, 256>>>(out, 2 + r);
                (void)hipEventRecord(b);
                (void)hipEventSynchronize(b);
                float ms;
                (void)hipEventElapsedTime(&ms, a, b);
                const double winst = (double)blocks * 4 * 5 * kIters * 32;  // wave-instructions
                if (rep == 1)
                    printf("waves/CU=%2d %-24s %8.1f G wave-instr/s  %.3f /clk/SIMD @2.4GHz\n", wpc, k.name,
                           winst / (ms * 1e-3) / 1e9, winst / (ms * 1e-3) / (cus * 4.0 * 2.4e9));
            }
    }
    return 0;
}
