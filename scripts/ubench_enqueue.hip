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
    // A pass-shaped graph: 3 streams (fork / join by events), 10 kernels, 6
    // D2D copies, 8 event records -- replayed with one hipGraphLaunch, against
    // enqueueing the same calls directly.
    hipEvent_t fork, j1, j2, x[8];
    CK(hipEventCreateWithFlags(&fork, hipEventDisableTiming));
    CK(hipEventCreateWithFlags(&j1, hipEventDisableTiming));
    CK(hipEventCreateWithFlags(&j2, hipEventDisableTiming));
    for (auto &e : x) CK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
    auto pass = [&](hipStream_t s0, hipStream_t s1, hipStream_t s2) -> int {
        CK(hipEventRecord(fork, s0));
        CK(hipStreamWaitEvent(s1, fork, 0));
        CK(hipStreamWaitEvent(s2, fork, 0));
        for (int k = 0; k < 4; k++) tiny<<<1, 64, 0, s0>>>(d);
        CK(hipEventRecord(x[0], s0));
        CK(hipStreamWaitEvent(s2, x[0], 0));
        for (int k = 0; k < 4; k++) tiny<<<1, 64, 0, s1>>>(d);
        for (int k = 0; k < 6; k++) {
            CK(hipMemcpyAsync(b, a, 32768, hipMemcpyDeviceToDevice, s2));
            CK(hipEventRecord(x[1 + (k % 6)], s2));
        }
        tiny<<<1, 64, 0, s2>>>(d);
        tiny<<<1, 64, 0, s2>>>(d);
        CK(hipEventRecord(j1, s1));
        CK(hipEventRecord(j2, s2));
        CK(hipStreamWaitEvent(s0, j1, 0));
        CK(hipStreamWaitEvent(s0, j2, 0));
        return 0;
    };
    const int P = 500;
    for (int rep = 0; rep < 2; rep++) {
        auto t0 = clk::now();
        for (int i = 0; i < P; i++)
            if (pass(st[0], st[1], st[2])) return 1;
        const double direct = us(t0, P);
        CK(hipDeviceSynchronize());
        hipGraph_t g;
        hipGraphExec_t ge;
        CK(hipStreamBeginCapture(st[0], hipStreamCaptureModeRelaxed));
        if (pass(st[0], st[1], st[2])) return 1;
        CK(hipStreamEndCapture(st[0], &g));
        size_t nodes = 0;
        CK(hipGraphGetNodes(g, nullptr, &nodes));
        CK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
        CK(hipGraphLaunch(ge, st[0]));
        CK(hipDeviceSynchronize());
        t0 = clk::now();
        for (int i = 0; i < P; i++) CK(hipGraphLaunch(ge, st[0]));
        const double graph = us(t0, P);
        CK(hipDeviceSynchronize());
        t0 = clk::now();
        for (int i = 0; i < P; i++) CK(hipGraphLaunch(ge, st[0]));
        CK(hipDeviceSynchronize());
        const double graph_dev = us(t0, P);
        t0 = clk::now();
        for (int i = 0; i < P; i++)
            if (pass(st[0], st[1], st[2])) return 1;
        CK(hipDeviceSynchronize());
        const double direct_dev = us(t0, P);
        printf("pass (%zu graph nodes): host us per pass: direct %.1f  graph %.1f;  with completion: direct %.1f  "
               "graph %.1f\n",
               nodes, direct, graph, direct_dev, graph_dev);
        CK(hipGraphExecDestroy(ge));
        CK(hipGraphDestroy(g));
    }
    return 0;
}
