// calib_8b.hip -- calibrates rocprofv3 FETCH_SIZE / WRITE_SIZE for the access
// width of the pair bit tiles (8 B per lane: one dwordx2 load / store of an
// interleaved pair, 512 B per wave-instruction) on a known byte count:
// copies 1 GiB each way in that pattern (measurement tool, not product code).
//   hipcc --offload-arch=gfx950 -O3 scripts/calib_8b.hip -o scripts/calib_8b
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

__global__ void copy8(const uint64_t *in, uint64_t *out, int64_t n) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) out[i] = in[i] ^ 1u;
}

int main() {
    const int64_t n = (int64_t)1 << 27;  // 1 GiB of 8-B pairs
    uint64_t *a, *b;
    if (hipMalloc(&a, n * 8) != hipSuccess || hipMalloc(&b, n * 8) != hipSuccess) return 1;
    (void)hipMemset(a, 1, n * 8);
    for (int r = 0; r < 3; r++) copy8<<<(unsigned)(n / 256), 256>>>(a, b, n);
    (void)hipDeviceSynchronize();
    printf("copied %lld bytes each way per launch, 3 launches\n", (long long)(n * 8));
    return 0;
}
