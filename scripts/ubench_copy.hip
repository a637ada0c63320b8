// Copy-ceiling variants (which copy kernel shape reaches the HBM ceiling on
// MI355X): grid-stride x4, contiguous chunk per block, nontemporal, sizes.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

__global__ __launch_bounds__(256) void gs4(const uint4 *__restrict__ in, uint4 *__restrict__ out, int64_t n) {
    const int64_t stride = (int64_t)gridDim.x * 256;
    int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
    for (; i + 3 * stride < n; i += 4 * stride) {
        uint4 a = in[i], b = in[i + stride], c = in[i + 2 * stride], d = in[i + 3 * stride];
        out[i] = a; out[i + stride] = b; out[i + 2 * stride] = c; out[i + 3 * stride] = d;
    }
    for (; i < n; i += stride) out[i] = in[i];
}
__global__ __launch_bounds__(256) void gs1(const uint4 *__restrict__ in, uint4 *__restrict__ out, int64_t n) {
    const int64_t stride = (int64_t)gridDim.x * 256;
    for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += stride) out[i] = in[i];
}
template <int U>
__global__ __launch_bounds__(256) void chunk(const uint4 *__restrict__ in, uint4 *__restrict__ out, int64_t n) {
    const int64_t base = (int64_t)blockIdx.x * 256 * U + threadIdx.x;
    uint4 v[U];
#pragma unroll
    for (int u = 0; u < U; u++) v[u] = in[base + u * 256];
#pragma unroll
    for (int u = 0; u < U; u++) out[base + u * 256] = v[u];
}
typedef unsigned int v4u __attribute__((ext_vector_type(4)));
template <int U>
__global__ __launch_bounds__(256) void chunk_nt(const uint4 *__restrict__ in_, uint4 *__restrict__ out_, int64_t n) {
    const v4u *in = reinterpret_cast<const v4u *>(in_);
    v4u *out = reinterpret_cast<v4u *>(out_);
    const int64_t base = (int64_t)blockIdx.x * 256 * U + threadIdx.x;
    v4u v[U];
#pragma unroll
    for (int u = 0; u < U; u++) v[u] = __builtin_nontemporal_load(in + base + u * 256);
#pragma unroll
    for (int u = 0; u < U; u++) __builtin_nontemporal_store(v[u], out + base + u * 256);
}

int main() {
    const int64_t bytes = 2LL << 30, n = bytes / 16;
    uint4 *a, *b;
    hipMalloc(&a, bytes); hipMalloc(&b, bytes);
    hipMemset(a, 1, bytes); hipMemset(b, 0, bytes);
    hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
    auto time = [&](const char *name, auto launch) {
        launch(); hipDeviceSynchronize();
        float best = 1e9f;
        for (int r = 0; r < 8; r++) {
            hipEventRecord(e0); launch(); hipEventRecord(e1); hipEventSynchronize(e1);
            float ms; hipEventElapsedTime(&ms, e0, e1); if (ms < best) best = ms;
        }
        printf("%-24s %8.3f ms  %7.1f GB/s\n", name, best, 2.0 * bytes / (best * 1e-3) / 1e9);
    };
    for (int g : {1024, 2048, 8192, 32768})
        { char nm[64]; snprintf(nm, 64, "gs4 grid %d", g); time(nm, [&] { gs4<<<g, 256>>>(a, b, n); }); }
    for (int g : {2048, 8192, 65536})
        { char nm[64]; snprintf(nm, 64, "gs1 grid %d", g); time(nm, [&] { gs1<<<g, 256>>>(a, b, n); }); }
    time("chunk U1", [&] { chunk<1><<<n / 256, 256>>>(a, b, n); });
    time("chunk U4", [&] { chunk<4><<<n / 1024, 256>>>(a, b, n); });
    time("chunk U8", [&] { chunk<8><<<n / 2048, 256>>>(a, b, n); });
    time("chunk_nt U4", [&] { chunk_nt<4><<<n / 1024, 256>>>(a, b, n); });
    time("chunk_nt U8", [&] { chunk_nt<8><<<n / 2048, 256>>>(a, b, n); });
    time("hipMemcpy D2D", [&] { hipMemcpyAsync(b, a, bytes, hipMemcpyDeviceToDevice, 0); });
    return 0;
}
