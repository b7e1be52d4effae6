// GPU test of the product's multi-rank gather (sbe_gather_encoded, include/sbecodec.h) on ONE
// device: the ranks of the communicator are threads of this process, and RCCL is the test stand-in
// tests/mock_rccl/libmock_rccl.so (loaded by the product because SBE_RCCL_LIB names it; the
// product's default is the real RCCL).  Every case shards one batch of variable-length
// TopicMessages into contiguous per-rank ranges, encodes each shard on its rank's stream, gathers
// them to the root and checks the root's stream and offsets against a single-batch encode of the
// whole batch by the oracle restatement (byte for byte), including roots other than 0, zero-record
// shards and both SBE_ENOSPC limits (every rank refuses; the root's buffers stay untouched).
#include <hip/hip_runtime.h>

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

static void run_case(const Batch& B, int world, int root, const std::vector<size_t>& cuts, int limit,
                     const std::vector<uint8_t>& eo, const std::vector<uint64_t>& eoff, const char* lib) {
    (void)lib;
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
    std::vector<RankResult> res(world);
    std::vector<std::thread> th;
    for (int r = 0; r < world; ++r) {
        th.emplace_back([&, r] {
            HIPCK(hipSetDevice(0));
            hipStream_t s;
            HIPCK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
            const size_t lo = cuts[r], hi = cuts[r + 1], m = hi - lo;
            // the shard's packed input
            const size_t ab = B.in_base[hi] - B.in_base[lo];
            uint8_t *d_arena, *d_out, *d_st;
            uint32_t* d_len;
            uint64_t *d_ts, *d_off;
            void* d_ws;
            const uint64_t cap = sbe_encode_output_bound(m, ab, 0);
            const size_t wsb = sbe_encode_workspace_size(m);
            HIPCK(hipMalloc(&d_arena, ab + 16));
            HIPCK(hipMalloc(&d_len, m * 20 + 16));
            HIPCK(hipMalloc(&d_ts, m * 8 + 16));
            HIPCK(hipMalloc(&d_out, cap + 16));
            HIPCK(hipMalloc(&d_off, (m + 1) * 8));
            HIPCK(hipMalloc(&d_st, m + 16));
            HIPCK(hipMalloc(&d_ws, wsb + 16));
            if (ab) HIPCK(hipMemcpy(d_arena, B.arena.data() + B.in_base[lo], ab, hipMemcpyHostToDevice));
            if (m) {
                HIPCK(hipMemcpy(d_len, B.len.data() + 5 * lo, m * 20, hipMemcpyHostToDevice));
                HIPCK(hipMemcpy(d_ts, B.ts.data() + lo, m * 8, hipMemcpyHostToDevice));
            }
            sbe_comm* c = nullptr;
            const int rci = sbe_comm_init(&c, world, r, id);
            if (rci != SBE_OK) {
                std::fprintf(stderr, "rank %d: sbe_comm_init %d (%s)\n", r, rci, sbe_last_error());
                res[r].rc_gather = rci;
                return;
            }
            sbe_tm_batch in{d_arena, nullptr, d_len, d_ts};
            res[r].rc_enc = sbe_encode_topic_batch(&in, m, 1, 0, d_out, cap, d_off, d_st, d_ws, wsb, s);
            const bool am_root = r == root;
            res[r].rc_gather = sbe_gather_encoded(c, root, d_out, d_off, m, am_root ? dst : nullptr, am_root ? dst_cap : 0,
                                                  am_root ? dst_off : nullptr, am_root ? off_cap : 0, res[r].totals, s);
            if (res[r].rc_gather != SBE_OK && res[r].rc_gather != SBE_ENOSPC)
                std::fprintf(stderr, "rank %d: gather %d (%s)\n", r, res[r].rc_gather, sbe_last_error());
            HIPCK(hipStreamSynchronize(s));
            CHECK(sbe_comm_destroy(c) == SBE_OK);
            for (void* p : {(void*)d_arena, (void*)d_len, (void*)d_ts, (void*)d_out, (void*)d_off, (void*)d_st, d_ws})
                HIPCK(hipFree(p));
            HIPCK(hipStreamDestroy(s));
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
    HIPCK(hipFree(dst));
    HIPCK(hipFree(dst_off));
    std::printf("case world=%d root=%d limit=%d shards=", world, root, limit);
    for (int r = 0; r < world; ++r) std::printf("%zu%s", cuts[r + 1] - cuts[r], r + 1 < world ? "," : "");
    std::printf(" -> %s\n", failures ? "FAIL" : "ok");
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
    run_case(B, 2, 0, even_cuts(N, 2), kOk, eo, eoff, lib);
    run_case(B, 2, 1, even_cuts(N, 2), kOk, eo, eoff, lib);
    run_case(B, 3, 2, even_cuts(N, 3), kOk, eo, eoff, lib);
    run_case(B, 3, 1, sized_cuts({0, 12345, N - 12345}), kOk, eo, eoff, lib);   // a zero-record shard
    run_case(B, 8, 0, even_cuts(N, 8), kOk, eo, eoff, lib);
    run_case(B, 8, 5, sized_cuts({1, 0, 4999, 0, 7000, 3, 0, N - 12003}), kOk, eo, eoff, lib);
    run_case(B, 8, 7, sized_cuts({0, 0, 0, 0, 0, 0, 0, N}), kOk, eo, eoff, lib);  // all on the last rank
    run_case(B, 4, 3, even_cuts(N, 4), kShortBytes, eo, eoff, lib);
    run_case(B, 4, 0, even_cuts(N, 4), kShortOffsets, eo, eoff, lib);
    run_case(B, 2, 0, sized_cuts({N, 0}), kOk, eo, eoff, lib);  // everything on the root
    std::printf("gather mock test: %s (%d failures)\n", failures ? "FAILED" : "ok", failures);
    return failures ? 1 : 0;
}
