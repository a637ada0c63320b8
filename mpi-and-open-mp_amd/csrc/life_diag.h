// life_diag.h -- per-workgroup timeline hooks of the tile kernels
// (diagnostics builds only: scripts/build_variants.sh NAME:WT:LIFE_WG_TRACE=1,
// read out by scripts/wg_trace.py).  In the product build (LIFE_WG_TRACE
// unset) wg_trace() is an empty inline function and no symbol is emitted.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#ifndef LIFE_WG_TRACE
#define LIFE_WG_TRACE 0
#endif

namespace life {
namespace {
// LIFE_WG_TRACE (compile time, diagnostics builds only): thread 0 of every
// workgroup of the bit tile kernels records [start, HW_ID | XCC_ID << 32, end
// of each tile (up to 14)] (wall clock, 100 MHz) for the last launch;
// life_debug_wg_trace copies it out.
#if LIFE_WG_TRACE
__device__ uint64_t g_wg_trace[16 * 65536];
__device__ __forceinline__ void wg_trace(int what) {  // 0: start, k >= 1: end of tile k
    if (threadIdx.x != 0 || blockIdx.x >= 65536 || what > 14) return;
    uint64_t *t = g_wg_trace + 16 * blockIdx.x;
    t[what == 0 ? 0 : what + 1] = wall_clock64();
    if (what == 0) {
        const uint32_t hw = __builtin_amdgcn_s_getreg((31 << 11) | 4);
        const uint32_t xcc = __builtin_amdgcn_s_getreg((15 << 11) | 20);
        t[1] = (uint64_t)hw | ((uint64_t)xcc << 32);
    }
}
#else
__device__ __forceinline__ void wg_trace(int) {}
#endif
}  // namespace
}  // namespace life

#if LIFE_WG_TRACE
extern "C" int life_debug_wg_trace(uint64_t *host, int64_t n) {
    if (n > 16 * 65536) n = 16 * 65536;
    return hipMemcpyFromSymbol(host, HIP_SYMBOL(life::g_wg_trace), n * sizeof(uint64_t), 0, hipMemcpyDeviceToHost) ==
                   hipSuccess
               ? 0
               : -1;
}
#endif
