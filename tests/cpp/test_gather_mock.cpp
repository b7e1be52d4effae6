// GPU test of the product's multi-rank gather (sbe_gather_encoded, include/sbecodec.h) on ONE
// device: the ranks of the communicator are threads of this process, and RCCL is the test stand-in
// tests/mock_rccl/libmock_rccl.so (loaded by the product because SBE_RCCL_LIB names it; the
// product's default is the real RCCL).  Every case shards one batch of variable-length
// TopicMessages into contiguous per-rank ranges, encodes each shard on its rank's stream, gathers
// them to the root and checks the root's stream and offsets against a single-batch encode of the
// whole batch by the oracle restatement (byte for byte), including roots other than 0, zero-record
// shards and both SBE_ENOSPC limits (every rank refuses; the root's buffers stay untouched).
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>
#include <string>
#include <thread>
#include <vector>

#include "sbecodec.h"
#include "../../oracle/sbe_oracle.h"

static int failures = 0;
#define CHECK(c)                                                            \
    do {                                                                    \
        if (!(c)) {                                                         \
            std::fprintf(stderr, "FAIL %s:%d: %s\n", __FILE__, __LINE__, #c); \
            ++failures;                                                     \
        }                                                                   \
    } while (0)
#define HIPCK(x)                                                                          \
    do {                                                                                  \
        hipError_t e_ = (x);                                                              \
        if (e_ != hipSuccess) {                                                           \
            std::fprintf(stderr, "HIP %s:%d: %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
            std::exit(3);                                                                 \
        }                                                                                 \
    } while (0)

struct Batch {  // host SoA of the whole batch (packed arena)
    std::vector<uint8_t> arena;
    std::vector<uint32_t> len;  // [n][5]
    std::vector<uint64_t> ts;
    std::vector<uint64_t> in_base;  // [n+1] arena offset of record i's first string
    size_t n = 0;
};

static Batch make_batch(size_t n, uint64_t seed) {
    Batch b;
    b.n = n;
    std::mt19937_64 rng(seed);
    b.in_base.push_back(0);
    for (size_t i = 0; i < n; ++i) {
        for (int f = 0; f < 5; ++f) {
            const uint32_t L = (uint32_t)(rng() % (f == 3 ? 400 : 40));
            for (uint32_t k = 0; k < L; ++k) b.arena.push_back((uint8_t)(32 + rng() % 95));
            b.len.push_back(L);
        }
        b.ts.push_back(rng() | 1);
        b.in_base.push_back(b.arena.size());
    }
    return b;
}

enum { kOk = 0, kShortBytes = 1, kShortOffsets = 2 };

struct RankResult {
    int rc_enc = -99, rc_gather = -99;
    uint64_t totals[2] = {0, 0};
};

static double now_s() {
    static const auto t0 = std::chrono::steady_clock::now();
    return std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
}
// a rank's phase, unbuffered, so that a stall shows how far every rank got
static void phase(int world, int root, int r, const char* what) {
    std::fprintf(stderr, "[%.3fs] world=%d root=%d rank %d: %s\n", now_s(), world, root, r, what);
}

struct RankBufs {  // one rank's device buffers, all allocated by the main thread
    hipStream_t s = nullptr;
    uint8_t *arena = nullptr, *out = nullptr, *st = nullptr;
    uint32_t* len = nullptr;
    uint64_t *ts = nullptr, *off = nullptr;
    void* ws = nullptr;
    uint64_t cap = 0;
    size_t wsb = 0;
    sbe_comm* c = nullptr;
};

// Memory management, stream creation and communicator setup / teardown all happen on the main
// thread, before the rank threads start and after they have joined: a rank thread only launches
// (encode, gather) and waits on its own stream, so no rank ever allocates or frees (device-wide
// synchronising calls) while a peer is parked inside a collective.
static void run_case(const Batch& B, int world, int root, const std::vector<size_t>& cuts, int limit,
                     const std::vector<uint8_t>& eo, const std::vector<uint64_t>& eoff, bool sized) {
    const double t_case = now_s();
    const size_t N = B.n;
    const uint64_t total = eoff[N];
    uint8_t id[SBE_COMM_ID_BYTES];
    CHECK(sbe_comm_unique_id(id) == SBE_OK);
    // the root's buffers, filled with a sentinel
    const uint64_t dst_cap = limit == kShortBytes ? (total ? total - 1 : 0) : total + 64;
    const uint64_t off_cap = limit == kShortOffsets ? N : N + 1;
    uint8_t* dst = nullptr;
    uint64_t* dst_off = nullptr;
    HIPCK(hipMalloc(&dst, dst_cap + 16));
    HIPCK(hipMalloc(&dst_off, (off_cap + 1) * 8));
    HIPCK(hipMemset(dst, 0xAB, dst_cap + 16));
    HIPCK(hipMemset(dst_off, 0xCD, (off_cap + 1) * 8));
    std::vector<RankBufs> rb(world);
    std::vector<uint64_t> sizes(2 * (size_t)world);  // the sized entry's {bytes, records} per rank
    for (int r = 0; r < world; ++r) {
        RankBufs& b = rb[r];
        const size_t lo = cuts[r], hi = cuts[r + 1], m = hi - lo;
        const size_t ab = B.in_base[hi] - B.in_base[lo];
        b.cap = sbe_encode_output_bound(m, ab, 0);
        b.wsb = sbe_encode_workspace_size(m);
        HIPCK(hipStreamCreateWithFlags(&b.s, hipStreamNonBlocking));
        HIPCK(hipMalloc(&b.arena, ab + 16));
        HIPCK(hipMalloc(&b.len, m * 20 + 16));
        HIPCK(hipMalloc(&b.ts, m * 8 + 16));
        HIPCK(hipMalloc(&b.out, b.cap + 16));
        HIPCK(hipMalloc(&b.off, (m + 1) * 8));
        HIPCK(hipMalloc(&b.st, m + 16));
        HIPCK(hipMalloc(&b.ws, b.wsb + 16));
        if (ab) HIPCK(hipMemcpy(b.arena, B.arena.data() + B.in_base[lo], ab, hipMemcpyHostToDevice));
        if (m) {
            HIPCK(hipMemcpy(b.len, B.len.data() + 5 * lo, m * 20, hipMemcpyHostToDevice));
            HIPCK(hipMemcpy(b.ts, B.ts.data() + lo, m * 8, hipMemcpyHostToDevice));
        }
        const int rci = sbe_comm_init(&b.c, world, r, id);
        if (rci != SBE_OK) std::fprintf(stderr, "rank %d: sbe_comm_init %d (%s)\n", r, rci, sbe_last_error());
        CHECK(rci == SBE_OK);
        sizes[2 * r] = eoff[hi] - eoff[lo];  // the caller's own size plan (fixed-size records, or a host plan)
        sizes[2 * r + 1] = m;
    }
    HIPCK(hipDeviceSynchronize());
    std::vector<RankResult> res(world);
    std::vector<std::thread> th;
    for (int r = 0; r < world; ++r) {
        th.emplace_back([&, r] {
            RankBufs& b = rb[r];
            if (!b.c) return;
            HIPCK(hipSetDevice(0));
            const size_t m = cuts[r + 1] - cuts[r];
            phase(world, root, r, "encode");
            sbe_tm_batch in{b.arena, nullptr, b.len, b.ts};
            res[r].rc_enc = sbe_encode_topic_batch(&in, m, 1, 0, b.out, b.cap, b.off, b.st, b.ws, b.wsb, b.s);
            phase(world, root, r, sized ? "gather (sized)" : "gather");
            const bool am_root = r == root;
            if (sized)
                res[r].rc_gather = sbe_gather_encoded_sized(b.c, root, sizes.data(), b.out, b.off,
                                                            am_root ? dst : nullptr, dst_cap,  // the root's, on every rank
                                                            am_root ? dst_off : nullptr, off_cap, res[r].totals, b.s);
            else
                res[r].rc_gather = sbe_gather_encoded(b.c, root, b.out, b.off, m, am_root ? dst : nullptr,
                                                      am_root ? dst_cap : 0, am_root ? dst_off : nullptr,
                                                      am_root ? off_cap : 0, res[r].totals, b.s);
            if (res[r].rc_gather != SBE_OK && res[r].rc_gather != SBE_ENOSPC)
                std::fprintf(stderr, "rank %d: gather %d (%s)\n", r, res[r].rc_gather, sbe_last_error());
            phase(world, root, r, "stream sync");
            HIPCK(hipStreamSynchronize(b.s));
            phase(world, root, r, "done");
        });
    }
    for (auto& t : th) t.join();
    for (int r = 0; r < world; ++r) {
        CHECK(res[r].rc_enc == SBE_OK);
        CHECK(res[r].rc_gather == (limit == kOk ? SBE_OK : SBE_ENOSPC));
        CHECK(res[r].totals[0] == total && res[r].totals[1] == N);
    }
    std::vector<uint8_t> got(dst_cap + 16);
    std::vector<uint64_t> goff(off_cap + 1);
    HIPCK(hipMemcpy(got.data(), dst, got.size(), hipMemcpyDeviceToHost));
    HIPCK(hipMemcpy(goff.data(), dst_off, goff.size() * 8, hipMemcpyDeviceToHost));
    if (limit == kOk) {
        CHECK(std::memcmp(got.data(), eo.data(), total) == 0);
        CHECK(std::memcmp(goff.data(), eoff.data(), (N + 1) * 8) == 0);
        CHECK(got[total] == 0xAB && goff[N + 1] == 0xCDCDCDCDCDCDCDCDull);  // nothing past the batch
    } else {  // refused on every rank before any transfer: the root's buffers are untouched
        bool clean = true;
        for (uint8_t x : got) clean = clean && x == 0xAB;
        for (uint64_t x : goff) clean = clean && x == 0xCDCDCDCDCDCDCDCDull;
        CHECK(clean);
    }
    HIPCK(hipDeviceSynchronize());
    for (int r = 0; r < world; ++r) {
        RankBufs& b = rb[r];
        CHECK(sbe_comm_destroy(b.c) == SBE_OK);
        for (void* p : {(void*)b.arena, (void*)b.len, (void*)b.ts, (void*)b.out, (void*)b.off, (void*)b.st, b.ws})
            HIPCK(hipFree(p));
        HIPCK(hipStreamDestroy(b.s));
    }
    HIPCK(hipFree(dst));
    HIPCK(hipFree(dst_off));
    std::printf("case %s world=%d root=%d limit=%d shards=", sized ? "sized" : "plain", world, root, limit);
    for (int r = 0; r < world; ++r) std::printf("%zu%s", cuts[r + 1] - cuts[r], r + 1 < world ? "," : "");
    std::printf(" -> %s (%.3f s)\n", failures ? "FAIL" : "ok", now_s() - t_case);
    std::fflush(stdout);
}

// contiguous ranges: shard_range's rule (record i -> rank floor(i * world / n)), or explicit sizes
static std::vector<size_t> even_cuts(size_t n, int world) {
    std::vector<size_t> c(world + 1);
    for (int r = 0; r <= world; ++r) c[r] = (n * (size_t)r + world - 1) / world;
    c[world] = n;
    return c;
}
static std::vector<size_t> sized_cuts(const std::vector<size_t>& sizes) {
    std::vector<size_t> c{0};
    for (size_t s : sizes) c.push_back(c.back() + s);
    return c;
}

int main() {
    const char* lib = std::getenv("SBE_RCCL_LIB");
    if (!lib || !*lib) {
        std::fprintf(stderr, "SBE_RCCL_LIB must name tests/mock_rccl/libmock_rccl.so\n");
        return 2;
    }
    if (sbe_device_ready() != 1) {
        std::fprintf(stderr, "no gfx950 device\n");
        return 2;
    }
    HIPCK(hipSetDevice(0));
    const size_t N = 20000;
    const Batch B = make_batch(N, 0x6A7E);
    std::vector<uint8_t> eo(sbe_encode_output_bound(N, B.arena.size(), 0) + 16);
    std::vector<uint64_t> eoff(N + 1);
    std::vector<uint8_t> est(N);
    orc_encode_batch(B.arena.data(), nullptr, B.len.data(), B.ts.data(), N, 1, 0, eo.data(), eoff.data(), est.data(), 1);
    for (const bool sized : {false, true}) {
        run_case(B, 2, 0, even_cuts(N, 2), kOk, eo, eoff, sized);
        run_case(B, 2, 1, even_cuts(N, 2), kOk, eo, eoff, sized);
        run_case(B, 3, 2, even_cuts(N, 3), kOk, eo, eoff, sized);
        run_case(B, 3, 1, sized_cuts({0, 12345, N - 12345}), kOk, eo, eoff, sized);   // a zero-record shard
        run_case(B, 8, 0, even_cuts(N, 8), kOk, eo, eoff, sized);
        run_case(B, 8, 5, sized_cuts({1, 0, 4999, 0, 7000, 3, 0, N - 12003}), kOk, eo, eoff, sized);
        run_case(B, 8, 7, sized_cuts({0, 0, 0, 0, 0, 0, 0, N}), kOk, eo, eoff, sized);  // all on the last rank
        run_case(B, 4, 3, even_cuts(N, 4), kShortBytes, eo, eoff, sized);
        run_case(B, 4, 0, even_cuts(N, 4), kShortOffsets, eo, eoff, sized);
        run_case(B, 2, 0, sized_cuts({N, 0}), kOk, eo, eoff, sized);  // everything on the root
    }
    std::printf("gather mock test: %s (%d failures)\n", failures ? "FAILED" : "ok", failures);
    return failures ? 1 : 0;
}
