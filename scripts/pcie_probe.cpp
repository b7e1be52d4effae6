// pcie_probe.cpp — host<->device copy rates the host mirror's pipeline is bound by (diagnosis,
// not product): page-locked H2D / D2H of one 64 MiB buffer as one copy and as 8 MiB pieces over
// two streams, and both directions at once.  Build + run (GPU box): make -C scripts pcie_probe
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <thread>
#include <vector>

#define CK(x)                                                                   \
    do {                                                                        \
        hipError_t e_ = (x);                                                    \
        if (e_ != hipSuccess) {                                                 \
            std::fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));        \
            std::exit(1);                                                       \
        }                                                                       \
    } while (0)

using clk = std::chrono::steady_clock;

int main() {
    const size_t N = size_t(64) << 20;
    void *h0, *h1, *d0, *d1;
    CK(hipHostMalloc(&h0, N, hipHostMallocDefault));
    CK(hipHostMalloc(&h1, N, hipHostMallocDefault));
    CK(hipMalloc(&d0, N));
    CK(hipMalloc(&d1, N));
    hipStream_t s[2];
    for (auto& x : s) CK(hipStreamCreateWithFlags(&x, hipStreamNonBlocking));
    auto run = [&](const char* name, int mode, size_t piece) {
        double best = 1e30;
        for (int it = 0; it < 6; ++it) {
            CK(hipDeviceSynchronize());
            const auto t0 = clk::now();
            for (size_t o = 0, k = 0; o < N; o += piece, ++k) {
                // one direction: pieces alternate streams; both: H2D on stream 0, D2H on stream 1
                hipStream_t sa = mode == 2 ? s[0] : s[k & 1], sb = mode == 2 ? s[1] : s[k & 1];
                if (mode == 0 || mode == 2) CK(hipMemcpyAsync((char*)d0 + o, (char*)h0 + o, piece, hipMemcpyHostToDevice, sa));
                if (mode == 1 || mode == 2) CK(hipMemcpyAsync((char*)h1 + o, (char*)d1 + o, piece, hipMemcpyDeviceToHost, sb));
            }
            CK(hipDeviceSynchronize());
            const double us = std::chrono::duration<double, std::micro>(clk::now() - t0).count();
            if (it && us < best) best = us;
        }
        const double bytes = (mode == 2 ? 2.0 : 1.0) * N;
        std::printf("{\"copy\": \"%s\", \"piece_MiB\": %zu, \"us\": %.1f, \"GBps\": %.2f}\n", name, piece >> 20, best,
                    bytes / best / 1e3);
        std::fflush(stdout);
    };
    for (size_t piece : {N, N / 8, N / 32}) {
        run("h2d", 0, piece);
        run("d2h", 1, piece);
        run("both", 2, piece);
    }
    // host staging: pageable -> page-locked memcpy by T threads, alone and while the DMA engines
    // copy another buffer host->device (the pipeline's overlap)
    char* pg = (char*)std::malloc(N);
    std::memset(pg, 1, N);
    for (int T : {1, 4, 8, 16}) {
        for (int with_dma = 0; with_dma < 2; ++with_dma) {
            double best = 1e30;
            for (int it = 0; it < 5; ++it) {
                CK(hipDeviceSynchronize());
                if (with_dma)
                    for (int r = 0; r < 2; ++r) CK(hipMemcpyAsync(d1, h1, N, hipMemcpyHostToDevice, s[0]));
                const auto t0 = clk::now();
                std::vector<std::thread> th;
                for (int t = 0; t < T; ++t)
                    th.emplace_back([&, t] { std::memcpy((char*)h0 + N / T * t, pg + N / T * t, N / T); });
                for (auto& x : th) x.join();
                const double us = std::chrono::duration<double, std::micro>(clk::now() - t0).count();
                CK(hipDeviceSynchronize());
                if (us < best) best = us;
            }
            std::printf("{\"memcpy_threads\": %d, \"with_h2d\": %d, \"us\": %.1f, \"GBps\": %.2f}\n", T, with_dma, best,
                        N / best / 1e3);
            std::fflush(stdout);
        }
    }
    // H2D while the host stages (16 threads, repeated)
    return 0;
}
