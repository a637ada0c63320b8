// calib_4b.hip -- calibrates rocprofv3 FETCH_SIZE / WRITE_SIZE for the access
// width of the temporal bit kernel (4 B per lane, 256 B per wave-instruction,
// 62 of 64 lanes storing) on a known byte count: copies N dwords, 1 GiB
// each way, in the same pattern (measurement tool, not product code).
//   hipcc --offload-arch=gfx950 -O3 scripts/calib_4b.hip -o scripts/calib_4b
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

__global__ void copy4(const uint32_t *in, uint32_t *out, int64_t n) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) out[i] = in[i] ^ 1u;
}

int main() {
    const int64_t n = (int64_t)1 << 28;  // 1 GiB of dwords
    uint32_t *a, *b;
    if (hipMalloc(&a, n * 4) != hipSuccess || hipMalloc(&b, n * 4) != hipSuccess) return 1;
    (void)hipMemset(a, 1, n * 4);
    for (int r = 0; r < 3; r++) copy4<<<(unsigned)(n / 256), 256>>>(a, b, n);
    (void)hipDeviceSynchronize();
    printf("copied %lld bytes each way per launch, 3 launches\n", (long long)(n * 4));
    return 0;
}
