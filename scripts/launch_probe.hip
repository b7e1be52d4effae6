// launch_probe.hip — the floor of a one-record call on this box: a tiny kernel's launch-to-host
// round trip (hipLaunchKernelGGL + hipStreamSynchronize / hipEventSynchronize / spinning on a
// page-locked flag the kernel writes), and of a persistent kernel that polls a page-locked doorbell
// (no launch per request).  Measurement tooling, not product code.
// Build: hipcc --offload-arch=gfx950 -O2 -o scripts/launch_probe scripts/launch_probe.hip
#include <hip/hip_runtime.h>

#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstdint>

#define CK(x)                                                                                   \
    do {                                                                                        \
        hipError_t e = (x);                                                                     \
        if (e != hipSuccess) {                                                                  \
            std::printf("HIP error %s at %s:%d\n", hipGetErrorString(e), __FILE__, __LINE__);   \
            return 1;                                                                           \
        }                                                                                       \
    } while (0)

__global__ void touch(volatile uint32_t* flag, uint32_t v) {
    if (threadIdx.x == 0) *flag = v;
}

// persistent server: waits for req[0] to change, answers by writing resp[0]; exits on req == ~0u
// or after `idle_spins` polls without a request (so the grid always drains)
__global__ void server(volatile uint32_t* req, volatile uint32_t* resp, uint32_t idle_spins) {
    if (threadIdx.x != 0) return;
    uint32_t last = 0, idle = 0;
    for (;;) {
        const uint32_t r = __atomic_load_n(req, __ATOMIC_ACQUIRE);
        if (r == 0xffffffffu) break;
        if (r != last) {
            last = r;
            idle = 0;
            __atomic_store_n(resp, r, __ATOMIC_RELEASE);
            continue;
        }
        if (++idle > idle_spins) break;
        __builtin_amdgcn_s_sleep(1);
    }
}

using clk = std::chrono::steady_clock;
static double us(clk::time_point a, clk::time_point b) { return std::chrono::duration<double, std::micro>(b - a).count(); }

int main() {
    hipStream_t s;
    CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    uint32_t* flag;
    CK(hipHostMalloc(&flag, 4096, hipHostMallocDefault));
    hipEvent_t ev;
    CK(hipEventCreateWithFlags(&ev, hipEventDisableTiming));
    const int N = 2000;
    for (int i = 0; i < 100; ++i) {
        hipLaunchKernelGGL(touch, dim3(1), dim3(64), 0, s, flag, (uint32_t)i);
        CK(hipStreamSynchronize(s));
    }
    auto t0 = clk::now();
    for (int i = 0; i < N; ++i) {
        hipLaunchKernelGGL(touch, dim3(1), dim3(64), 0, s, flag, (uint32_t)i);
        CK(hipStreamSynchronize(s));
    }
    auto t1 = clk::now();
    std::printf("{\"probe\": \"launch+hipStreamSynchronize\", \"us\": %.2f}\n", us(t0, t1) / N);
    t0 = clk::now();
    for (int i = 0; i < N; ++i) {
        hipLaunchKernelGGL(touch, dim3(1), dim3(64), 0, s, flag, (uint32_t)i);
        CK(hipEventRecord(ev, s));
        CK(hipEventSynchronize(ev));
    }
    t1 = clk::now();
    std::printf("{\"probe\": \"launch+event sync\", \"us\": %.2f}\n", us(t0, t1) / N);
    volatile uint32_t* vf = flag;
    t0 = clk::now();
    for (int i = 0; i < N; ++i) {
        const uint32_t v = 0x10000u + (uint32_t)i;
        hipLaunchKernelGGL(touch, dim3(1), dim3(64), 0, s, flag, v);
        while (*vf != v) {
        }
    }
    CK(hipStreamSynchronize(s));
    t1 = clk::now();
    std::printf("{\"probe\": \"launch+spin on host flag\", \"us\": %.2f}\n", us(t0, t1) / N);
    t0 = clk::now();
    for (int i = 0; i < N; ++i) hipLaunchKernelGGL(touch, dim3(1), dim3(64), 0, s, flag, (uint32_t)i);
    t1 = clk::now();
    CK(hipStreamSynchronize(s));
    std::printf("{\"probe\": \"launch enqueue only\", \"us\": %.2f}\n", us(t0, t1) / N);
    // persistent server round trip
    volatile uint32_t* req = flag + 64;
    volatile uint32_t* resp = flag + 128;
    *req = 0;
    *resp = 0;
    hipLaunchKernelGGL(server, dim3(1), dim3(64), 0, s, (uint32_t*)req, (uint32_t*)resp, 50000000u);
    for (int i = 1; i <= 100; ++i) {
        *req = (uint32_t)i;
        while (*resp != (uint32_t)i) {
        }
    }
    t0 = clk::now();
    for (int i = 101; i <= 100 + N; ++i) {
        std::atomic_thread_fence(std::memory_order_seq_cst);
        *req = (uint32_t)i;
        while (*resp != (uint32_t)i) {
        }
    }
    t1 = clk::now();
    *req = 0xffffffffu;
    CK(hipStreamSynchronize(s));
    std::printf("{\"probe\": \"persistent server round trip\", \"us\": %.2f}\n", us(t0, t1) / N);
    return 0;
}
