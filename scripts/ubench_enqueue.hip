// Host enqueue cost of the runtime calls an exchange pass is made of
// (measurement tool): hipLaunchKernel, hipMemcpyAsync
// device-to-device (32 KB, 512 KB), hipEventRecord, hipStreamWaitEvent --
// each timed on the host over many calls onto idle-ish streams (24 streams,
// as 8 shards x 3), then synchronised.
//   hipcc --offload-arch=gfx950 -O2 -o scripts/ubench_enqueue scripts/ubench_enqueue.hip
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>
#include <vector>

#define CK(x)                                                                 \
    do {                                                                      \
        hipError_t e_ = (x);                                                  \
        if (e_ != hipSuccess) {                                               \
            fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
            return 1;                                                         \
        }                                                                     \
    } while (0)

__global__ void tiny(int *) {}  // enqueue cost only

int main() {
    const int NS = 24, N = 4000;
    std::vector<hipStream_t> st(NS);
    std::vector<hipEvent_t> ev(NS);
    for (int i = 0; i < NS; i++) {
        CK(hipStreamCreateWithFlags(&st[i], hipStreamNonBlocking));
        CK(hipEventCreateWithFlags(&ev[i], hipEventDisableTiming));
    }
    int *d = nullptr;
    uint8_t *a = nullptr, *b = nullptr;
    CK(hipMalloc(&d, 4096));
    CK(hipMalloc(&a, 1 << 20));
    CK(hipMalloc(&b, 1 << 20));
    CK(hipMemset(d, 0, 4096));
    CK(hipDeviceSynchronize());
    using clk = std::chrono::steady_clock;
    auto us = [](clk::time_point t0, int n) {
        return std::chrono::duration<double, std::micro>(clk::now() - t0).count() / n;
    };
    for (int rep = 0; rep < 2; rep++) {
        auto t0 = clk::now();
        for (int i = 0; i < N; i++) tiny<<<1, 64, 0, st[i % NS]>>>(d + (i % NS) * 16);
        const double launch = us(t0, N);
        CK(hipDeviceSynchronize());
        t0 = clk::now();
        for (int i = 0; i < N; i++) CK(hipMemcpyAsync(b, a, 32768, hipMemcpyDeviceToDevice, st[i % NS]));
        const double cp32 = us(t0, N);
        CK(hipDeviceSynchronize());
        t0 = clk::now();
        for (int i = 0; i < N; i++) CK(hipMemcpyAsync(b, a, 524288, hipMemcpyDeviceToDevice, st[i % NS]));
        const double cp512 = us(t0, N);
        CK(hipDeviceSynchronize());
        t0 = clk::now();
        for (int i = 0; i < N; i++) CK(hipEventRecord(ev[i % NS], st[i % NS]));
        const double rec = us(t0, N);
        CK(hipDeviceSynchronize());
        t0 = clk::now();
        for (int i = 0; i < N; i++) CK(hipStreamWaitEvent(st[i % NS], ev[(i + 1) % NS], 0));
        const double wait = us(t0, N);
        CK(hipDeviceSynchronize());
        t0 = clk::now();
        for (int i = 0; i < N; i++) CK(hipSetDevice(0));
        const double setdev = us(t0, N);
        printf("rep %d: us per call: launch %.2f  memcpy32K %.2f  memcpy512K %.2f  eventRecord %.2f  "
               "streamWaitEvent %.2f  setDevice %.3f\n",
               rep, launch, cp32, cp512, rec, wait, setdev);
    }
    return 0;
}
