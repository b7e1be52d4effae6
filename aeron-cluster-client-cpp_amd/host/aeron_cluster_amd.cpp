// aeron_cluster_amd.cpp — host side of the reference codec surface over the C ABI.
// Host memory in, host memory out (the reference's API contract).  Every batch call runs a
// chunk pipeline: the batch is cut into chunks of a few MiB; the host threads stage chunk k+1 in
// page-locked memory while chunk k is copied to HBM (copy-in stream), coded by the HIP kernels of
// include/sbecodec.h (compute stream) and chunk k-1 is copied back (copy-out stream).  Encoded
// bytes land by DMA directly in a recycled page-locked block the caller receives (HostBytes);
// decode descriptors land in one the same way, and ParseResults are built from them on the host
// threads.  Results are materialised from the device descriptors (views into the caller's own
// bytes), never recomputed here.
#include "aeron_cluster_amd.hpp"

#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <deque>
#include <ctime>
#include <iomanip>
#include <iostream>
#include <map>
#include <mutex>
#include <sstream>
#include <stdexcept>
#include <thread>

#include "sbecodec.h"
#include "workers.hpp"

namespace aeron_cluster {

// ======================================================================================
// host runtime: worker threads, page-locked block pool
// ======================================================================================
namespace {

[[noreturn]] void fail(const char* what) {
    throw std::runtime_error(std::string("sbecodec: ") + what + " (" + sbe_last_error() + ")");
}

void hip_check(hipError_t e, const char* what) {
    if (e != hipSuccess) throw std::runtime_error(std::string("sbecodec: ") + what + ": " + hipGetErrorString(e));
}

using detail::Workers;  // the worker pool (workers.hpp)

// parallel_for over [0, n) in contiguous ranges of at least `grain` items: fn(lo, hi).
template <class F>
void for_ranges(size_t n, size_t grain, F&& fn) {
    Workers& w = Workers::get();
    const size_t maxt = (size_t)w.size() * 4;
    size_t ntasks = std::min(maxt, std::max<size_t>(1, n / std::max<size_t>(grain, 1)));
    if (ntasks <= 1) {
        if (n) fn(size_t(0), n);
        return;
    }
    w.parallel_for(ntasks, [&](size_t t) { fn(n * t / ntasks, n * (t + 1) / ntasks); });
}

// The page-locked ranges this library knows: its own pool blocks and staging buffers and the
// ranges the caller registered with host_register, each with its device address (looked up once,
// when the range is added).  A per-call lookup here replaces the HIP pointer queries, which cost
// microseconds per call.
class PinnedRegistry {
public:
    static PinnedRegistry& get() {
        static PinnedRegistry* r = new PinnedRegistry();  // never destroyed
        return *r;
    }
    void add(const void* p, size_t bytes) {
        void* d = nullptr;
        if (hipHostGetDevicePointer(&d, const_cast<void*>(p), 0) != hipSuccess) {
            (void)hipGetLastError();
            d = nullptr;
        }
        std::lock_guard<std::mutex> g(m_);
        ranges_[reinterpret_cast<uintptr_t>(p)] = Range{reinterpret_cast<uintptr_t>(p) + bytes, reinterpret_cast<uintptr_t>(d)};
    }
    void remove(const void* p) {
        std::lock_guard<std::mutex> g(m_);
        ranges_.erase(reinterpret_cast<uintptr_t>(p));
    }
    // [p, p + bytes) inside one known range: its device address (nullptr when it has none), true
    bool find(const void* p, size_t bytes, uint8_t** dev) const {
        const uintptr_t a = reinterpret_cast<uintptr_t>(p);
        std::lock_guard<std::mutex> g(m_);
        auto it = ranges_.upper_bound(a);
        if (it == ranges_.begin()) return false;
        --it;
        if (a + bytes > it->second.end) return false;
        *dev = it->second.dev ? reinterpret_cast<uint8_t*>(it->second.dev + (a - it->first)) : nullptr;
        return true;
    }

private:
    struct Range {
        uintptr_t end, dev;
    };
    mutable std::mutex m_;
    std::map<uintptr_t, Range> ranges_;
};

// Page-locked host blocks recycled by size class (powers of two from 4 KiB); hipHostMalloc costs
// milliseconds per call for large blocks, so a block is allocated once and reused.  Free blocks are
// kept up to AERON_AMD_PINNED_CACHE_BYTES (default 4 GiB) in all; a block returned beyond that is
// freed.  Blocks held by callers (EncodedBatch, ParsedBatch) do not count against the cap.
class PinnedPool {
public:
    static PinnedPool& get() {
        static PinnedPool* p = new PinnedPool();  // never destroyed (blocks may outlive statics)
        return *p;
    }
    std::shared_ptr<void> take(size_t bytes) {
        size_t cls = size_t(1) << 12;
        while (cls < bytes) cls <<= 1;
        void* p = nullptr;
        {
            std::lock_guard<std::mutex> g(m_);
            auto& fl = free_[cls];
            if (!fl.empty()) {
                p = fl.back();
                fl.pop_back();
                cached_ -= cls;
            }
        }
        if (!p) {
            hip_check(hipHostMalloc(&p, cls, hipHostMallocDefault), "hipHostMalloc");
            PinnedRegistry::get().add(p, cls);
        }
        return std::shared_ptr<void>(p, [this, cls](void* q) { give(q, cls); });
    }

private:
    void give(void* p, size_t cls) {
        {
            std::lock_guard<std::mutex> g(m_);
            if (cached_ + cls <= max_cached_) {
                free_[cls].push_back(p);
                cached_ += cls;
                return;
            }
        }
        PinnedRegistry::get().remove(p);
        (void)hipHostFree(p);
    }
    PinnedPool() {
        if (const char* e = std::getenv("AERON_AMD_PINNED_CACHE_BYTES")) max_cached_ = (size_t)std::max(0LL, std::atoll(e));
    }
    size_t max_cached_ = size_t(4) << 30;
    std::mutex m_;
    std::map<size_t, std::vector<void*>> free_;
    size_t cached_ = 0;
};

// Growable device / page-locked buffer owned by one thread's context.
struct DevBuf {
    void* p = nullptr;
    size_t cap = 0;
    void need(size_t n) {
        if (n <= cap) return;
        if (p) (void)hipFree(p);
        p = nullptr;
        cap = 0;
        const size_t c = n < 4096 ? 4096 : n + n / 4;
        hip_check(hipMalloc(&p, c), "hipMalloc");
        cap = c;
    }
    uint8_t* b() const { return static_cast<uint8_t*>(p); }
    ~DevBuf() {
        if (p) (void)hipFree(p);
    }
};
struct HostBuf {
    void* p = nullptr;
    uint8_t* dev = nullptr;  // its device address (the zero-copy kernels read it there)
    size_t cap = 0;
    void need(size_t n) {
        if (n <= cap) return;
        release();
        const size_t c = n < 4096 ? 4096 : n + n / 4;
        hip_check(hipHostMalloc(&p, c, hipHostMallocDefault), "hipHostMalloc");
        cap = c;
        PinnedRegistry::get().add(p, c);
        uint8_t* d = nullptr;
        PinnedRegistry::get().find(p, 1, &d);
        dev = d;
    }
    uint8_t* b() const { return static_cast<uint8_t*>(p); }
    void release() {
        if (p) {
            PinnedRegistry::get().remove(p);
            (void)hipHostFree(p);
        }
        p = nullptr;
        dev = nullptr;
        cap = 0;
    }
    ~HostBuf() { release(); }
};

// Three-stream chunk pipeline: host→device copies, kernels and device→host copies each on a
// stream of their own, ordered per chunk by events, so that chunk k+1's H2D, chunk k's kernels and
// chunk k-1's D2H run at once (on one stream the copy engine serialises H2D behind D2H).  Chunk k
// uses slot k % kSlots: its page-locked staging buffer and its device buffers.
struct Pipeline {
    static constexpr int kSlots = 3;
    struct Slot {
        hipEvent_t in_done = nullptr, comp_done = nullptr, out_done = nullptr;
        bool used = false;  // its events were recorded by an earlier chunk
        HostBuf pin;
        DevBuf d_in, d_out;
    };
    hipStream_t s_in = nullptr, s_comp = nullptr, s_out = nullptr;
    Slot slot[kSlots];
    // one-chunk calls: copy-in, kernels and copy-out in order on the compute stream, no events
    // (a small batch is latency-bound: each event record / wait costs more than it overlaps)
    bool serial = false;
    // called before the first copy or kernel of a batch is enqueued (Ctx: stop the resident server)
    void (*before_enqueue)(void*) = nullptr;
    void* before_arg = nullptr;
    void enqueue_hook() {
        if (before_enqueue) before_enqueue(before_arg);
    }

    void create() {
        for (hipStream_t* st : {&s_in, &s_comp, &s_out})
            hip_check(hipStreamCreateWithFlags(st, hipStreamNonBlocking), "hipStreamCreate");
        for (Slot& sl : slot)
            for (hipEvent_t* e : {&sl.in_done, &sl.comp_done, &sl.out_done})
                hip_check(hipEventCreateWithFlags(e, hipEventDisableTiming), "hipEventCreate");
    }
    void destroy() {
        for (Slot& sl : slot)
            for (hipEvent_t e : {sl.in_done, sl.comp_done, sl.out_done})
                if (e) (void)hipEventDestroy(e);
        for (hipStream_t st : {s_in, s_comp, s_out})
            if (st) (void)hipStreamDestroy(st);
    }
    // chunk k's slot, once the host may rewrite its staging buffer (its last H2D is done)
    Slot& begin(size_t k) {
        Slot& sl = slot[serial ? 0 : k % kSlots];
        if (sl.used) hip_check(hipEventSynchronize(sl.in_done), "hipEventSynchronize");
        return sl;
    }
    void drain() {
        if (serial) {
            hip_check(hipStreamSynchronize(s_comp), "hipStreamSynchronize");
            return;
        }
        for (hipStream_t st : {s_in, s_comp, s_out}) hip_check(hipStreamSynchronize(st), "hipStreamSynchronize");
    }
    // device buffers of the slot at least this large (growing drains the pipeline first: the old
    // buffers may still be in use by queued work)
    void reserve(Slot& sl, size_t in_bytes, size_t out_bytes) {
        if (in_bytes <= sl.d_in.cap && out_bytes <= sl.d_out.cap) return;
        drain();
        sl.d_in.need(in_bytes);
        sl.d_out.need(out_bytes);
    }
    // the slot's staged bytes to d_in, plus (direct) `dbytes` page-locked caller bytes to d_in + doff
    void copy_in(Slot& sl, size_t bytes, const void* direct = nullptr, size_t doff = 0, size_t dbytes = 0) {
        enqueue_hook();
        hipStream_t st = serial ? s_comp : s_in;
        if (!serial && sl.used) hip_check(hipStreamWaitEvent(s_in, sl.comp_done, 0), "hipStreamWaitEvent");  // d_in read
        hip_check(hipMemcpyAsync(sl.d_in.p, sl.pin.p, bytes, hipMemcpyHostToDevice, st), "H2D");
        if (dbytes) hip_check(hipMemcpyAsync(sl.d_in.b() + doff, direct, dbytes, hipMemcpyHostToDevice, st), "H2D");
        if (!serial) hip_check(hipEventRecord(sl.in_done, s_in), "hipEventRecord");
    }
    // the stream to launch the chunk's kernels on (after its input copy and the slot's last D2H)
    hipStream_t compute(Slot& sl) {
        enqueue_hook();
        if (serial) return s_comp;
        hip_check(hipStreamWaitEvent(s_comp, sl.in_done, 0), "hipStreamWaitEvent");
        if (sl.used) hip_check(hipStreamWaitEvent(s_comp, sl.out_done, 0), "hipStreamWaitEvent");
        return s_comp;
    }
    // the stream to issue the chunk's D2H copies on (after its kernels)
    hipStream_t copy_out(Slot& sl) {
        if (serial) return s_comp;
        hip_check(hipEventRecord(sl.comp_done, s_comp), "hipEventRecord");
        hip_check(hipStreamWaitEvent(s_out, sl.comp_done, 0), "hipStreamWaitEvent");
        return s_out;
    }
    void end(Slot& sl) {
        if (serial) return;
        hip_check(hipEventRecord(sl.out_done, s_out), "hipEventRecord");
        sl.used = true;
    }
};

// Batches of at most this many records (and within the zero-copy size) go to the thread's serve
// kernel (sbe_server_*: a resident wave polling a page-locked request slot, no launch per call);
// larger ones to the batch kernels.  One wave walks a served batch tile by tile, so the batch
// kernels overtake it between 64 and 256 fixed-256 records (profiles/r04_host_latency_serve.log:
// 64 records served 16.8 / 10.1 µs encode / decode against 24.2 / 18.8 µs launched, 256 records
// 50.0 / 28.6 against 28.1 / 19.6).  AERON_AMD_SERVE_RECORDS overrides (0: never serve).
size_t serve_max_records() {
    static const size_t v = [] {
        const char* e = std::getenv("AERON_AMD_SERVE_RECORDS");
        const long long x = e ? std::atoll(e) : 96;
        return (size_t)std::min<long long>(std::max(0LL, x), SBE_SERVE_MAX_RECORDS);
    }();
    return v;
}

// Batches of up to this many records that the single wave does not take go to the server's other
// workgroups as a whole (decode: tile per workgroup; encode: the tile loop with tile sums from the
// host's plan) instead of a launch: AERON_AMD_SERVE_WIDE_RECORDS (0: never); the server has
// AERON_AMD_SERVE_WGS workgroups (default 32).
size_t serve_wide_max_records() {
    static const size_t v = [] {
        const char* e = std::getenv("AERON_AMD_SERVE_WIDE_RECORDS");
        const long long x = e ? std::atoll(e) : 4096;
        return (size_t)std::min<long long>(std::max(0LL, x), SBE_SERVE_MAX_RECORDS);
    }();
    return v;
}
uint32_t serve_workgroups() {
    static const uint32_t v = [] {
        const char* e = std::getenv("AERON_AMD_SERVE_WGS");
        const long long x = e ? std::atoll(e) : 32;
        return (uint32_t)std::min<long long>(std::max(1LL, x), SBE_SERVE_MAX_WORKGROUPS);
    }();
    return v;
}

// How long an idle serve kernel keeps polling before it exits (AERON_AMD_SERVE_IDLE_US, default
// 1 ms); the next small call relaunches it (one launch, ≈ 6-12 µs).  While it is resident, work
// that HIP maps to the same hardware queue waits behind it (streams share GPU_MAX_HW_QUEUES
// queues), as does any device-wide synchronisation: short is the safe default.
uint32_t serve_idle_us() {
    static const uint32_t v = [] {
        const char* e = std::getenv("AERON_AMD_SERVE_IDLE_US");
        return e ? (uint32_t)std::max(1LL, std::atoll(e)) : 1000u;
    }();
    return v;
}

// Per-thread device context (the reference's codec functions are reentrant statics).
struct Ctx {
    Pipeline pipe;
    DevBuf d_aux;   // reassembly / Order JSON
    DevBuf d_ws;    // encode workspace of the zero-copy path
    HostBuf h_aux;
    std::vector<uint64_t> pin, pout;  // encode plan scratch (kept: first-touch costs on every call otherwise)
    sbe_server* srv = nullptr;
    bool srv_failed = false;   // in a cool-down after a failure (server() returns nullptr)
    int srv_failures = 0;      // failures so far (the cool-down doubles with each)
    std::chrono::steady_clock::time_point srv_retry_at{};
    Ctx() {
        if (sbe_device_ready() != 1) fail("no gfx950 device visible");
        pipe.create();
        pipe.before_enqueue = [](void* self) { static_cast<Ctx*>(self)->quiesce(); };
        pipe.before_arg = this;
    }
    // the compute stream for a launch outside the chunk loop (the resident server stopped first)
    hipStream_t batch_stream() {
        quiesce();
        return pipe.s_comp;
    }
    ~Ctx() {
        if (srv) (void)sbe_server_destroy(srv);
        pipe.destroy();
    }
    // The serve kernel for a batch of n records, or nullptr (too large, disabled, or unavailable:
    // the batch kernels take it).
    // wide: a batch for several workgroups (up to serve_wide_max_records())
    sbe_server* server(size_t n, bool wide = false) {
        if (n == 0 || n > (wide ? serve_wide_max_records() : serve_max_records())) return nullptr;
        if (srv_failed) {
            if (std::chrono::steady_clock::now() < srv_retry_at) return nullptr;
            srv_failed = false;  // the cool-down is over: try a server again
        }
        if (!srv && sbe_server_create_wide(&srv, serve_idle_us(), serve_workgroups()) != SBE_OK) {
            srv = nullptr;
            (void)hipGetLastError();
            back_off();
        }
        return srv;
    }
    // A serve request failed (timed out, or the server's stream failed): the server is freed (a
    // bounded wait, sbe_server_destroy) and this thread's calls go to the batch kernels for a
    // cool-down that doubles with each failure of this thread, from 1 s up to 64 s; then a new server is
    // tried (one transient timeout no longer disables the serve path for good).
    void drop_server() noexcept {
        if (srv) (void)sbe_server_destroy(srv);
        srv = nullptr;
        (void)hipGetLastError();
        back_off();
    }
    void back_off() noexcept {
        srv_failed = true;
        srv_retry_at = std::chrono::steady_clock::now() + std::chrono::seconds(1ll << std::min(srv_failures, 6));
        ++srv_failures;
    }
    // Before batch work is enqueued on this thread's streams: a resident server of this thread
    // exits first (a shutdown request, then its stream drains), so that no kernel or copy of the
    // batch can wait behind it on a shared hardware queue.  Free when the server is not running;
    // the next small call relaunches it.
    void quiesce() noexcept {
        if (srv && sbe_server_quiesce(srv) != SBE_OK) drop_server();
    }
    void sync_all() { pipe.drain(); }
    // After a throw inside a chunk loop: wait for every copy and kernel already queued (their
    // page-locked sources and destinations must not go back to a pool, or be restaged, while a
    // DMA still reads or writes them), then forget the slots' event history.  Never throws.
    void abort_all() noexcept {
        for (hipStream_t st : {pipe.s_in, pipe.s_comp, pipe.s_out})
            if (st) (void)hipStreamSynchronize(st);
        (void)hipGetLastError();
        for (Pipeline::Slot& sl : pipe.slot) sl.used = false;
    }
};

// Drains the pipeline if a chunk loop unwinds (declared after the buffers the queued copies use, so
// it runs before they are released).
struct PipeGuard {
    Ctx& c;
    bool armed = true;
    explicit PipeGuard(Ctx& x) : c(x) {}
    ~PipeGuard() {
        if (armed) c.abort_all();
    }
    void release() { armed = false; }
};

// The device address of page-locked host memory (hipHostMalloc'd or registered), or nullptr when
// it has none: kernels of the zero-copy path read their input and write their results there.
// An interior pointer resolves through the start of its allocation; ranges this library knows
// (PinnedRegistry) need no HIP query.
void* device_view(const void* host) {
    uint8_t* d0 = nullptr;
    if (PinnedRegistry::get().find(host, 1, &d0)) return d0;
    void* start = nullptr;
    if (hipPointerGetAttribute(&start, HIP_POINTER_ATTRIBUTE_RANGE_START_ADDR,
                               (hipDeviceptr_t)const_cast<void*>(host)) != hipSuccess || !start) {
        (void)hipGetLastError();
        return nullptr;
    }
    void* d = nullptr;
    if (hipHostGetDevicePointer(&d, start, 0) != hipSuccess || !d) {
        (void)hipGetLastError();
        return nullptr;
    }
    return static_cast<uint8_t*>(d) + (static_cast<const uint8_t*>(host) - static_cast<const uint8_t*>(start));
}

// Batches up to this many staged bytes (one pipeline chunk) take the zero-copy path: the kernels
// read the page-locked staging buffer and write their results straight into the page-locked result
// block over PCIe, one launch (encode: two) and one completion wait, no hipMemcpyAsync.  Larger
// one-chunk batches, and every chunk of a multi-chunk batch, go through the DMA copy engines.
// AERON_AMD_ZC_BYTES overrides (0: never).
size_t zero_copy_max_bytes() {
    static const size_t v = [] {
        const char* e = std::getenv("AERON_AMD_ZC_BYTES");
        return e ? (size_t)std::max(0LL, std::atoll(e)) : (size_t(4) << 20);
    }();
    return v;
}

Ctx& ctx() {
    thread_local Ctx c;
    return c;
}

inline size_t al16(size_t x) { return (x + 15) & ~(size_t)15; }

// n bytes from src to dst for the short strings of a record (topic, type, uuid, headers: tens of
// bytes): fixed-size, overlapping moves that the compiler inlines, instead of a memcpy call per
// string (the call, not the bytes, was the cost of staging and of building ParseResults)
inline void copy_small(void* dst_, const void* src_, size_t n) {
    uint8_t* dst = static_cast<uint8_t*>(dst_);
    const uint8_t* src = static_cast<const uint8_t*>(src_);
    if (n > 64) {
        std::memcpy(dst, src, n);
    } else if (n >= 16) {
        for (size_t k = 0; k + 16 < n; k += 16) std::memcpy(dst + k, src + k, 16);
        std::memcpy(dst + n - 16, src + n - 16, 16);
    } else if (n >= 8) {
        std::memcpy(dst, src, 8);
        std::memcpy(dst + n - 8, src + n - 8, 8);
    } else if (n >= 4) {
        std::memcpy(dst, src, 4);
        std::memcpy(dst + n - 4, src + n - 4, 4);
    } else if (n) {
        dst[0] = src[0];
        dst[n / 2] = src[n / 2];
        dst[n - 1] = src[n - 1];
    }
}

// AERON_AMD_TRACE=1: one line per batch call on stderr with its phase times (diagnosis only)
struct Trace {
    using clk = std::chrono::steady_clock;
    bool on;
    const char* what;
    clk::time_point t0, last;
    double plan = 0, stage = 0, wait = 0, enqueue = 0, sync = 0, finish = 0;
    explicit Trace(const char* w) : on(enabled()), what(w) {
        if (on) t0 = last = clk::now();
    }
    static bool enabled() {
        static const bool e = [] {
            const char* v = std::getenv("AERON_AMD_TRACE");
            return v && v[0] == '1';
        }();
        return e;
    }
    void lap(double& acc) {
        if (!on) return;
        const clk::time_point t = clk::now();
        acc += std::chrono::duration<double, std::micro>(t - last).count();
        last = t;
    }
    void done(size_t n, size_t chunks) {
        if (!on) return;
        std::fprintf(stderr,
                     "[trace] t0=%.1f %s n=%zu chunks=%zu threads=%u total=%.1fus plan=%.1f stage=%.1f wait=%.1f enqueue=%.1f sync=%.1f "
                     "finish=%.1f\n",
                     std::chrono::duration<double, std::micro>(t0.time_since_epoch()).count(), what, n, chunks,
                     Workers::get().size(), std::chrono::duration<double, std::micro>(clk::now() - t0).count(), plan, stage,
                     wait, enqueue, sync, finish);
    }
};

// Bytes of staged work per pipeline chunk: AERON_AMD_CHUNK_BYTES when set, else a third of the
// batch's bytes within [8, 32] MiB (and at most 65536 records, chunk_records): every chunk pays its
// copies' and launches' fixed costs, and a batch of a few chunks still overlaps its copies.
// host_latency, fixed-256 records, encode + parse_batch, three interleaved repetitions per
// setting (profiles/r03_host_chunks.log): 8 MiB chunks 46 M rec/s at 262 K records (median) and
// 39 M at 1 M; 16 MiB chunks (65536 records) 48 / 43 M at 262 K and 53 / 58 M at 1 M.  This
// rule against fixed 8 MiB chunks, interleaved on one box: 262 K 43.5 vs 41.5 M, 1 M 48.3 vs
// 47.8 M (medians; the box-to-box and run-to-run spread of these host numbers is ~20 %).
size_t chunk_target_bytes(size_t total_bytes) {
    static const size_t env = [] {
        const char* e = std::getenv("AERON_AMD_CHUNK_BYTES");
        const long long x = e ? std::atoll(e) : 0;
        return x > 0 ? (size_t)x : size_t(0);
    }();
    if (env) return env;
    return std::min(size_t(32) << 20, std::max(size_t(8) << 20, total_bytes / 3));
}
// Records per chunk: a power of two so that a chunk holds about chunk_target_bytes().
size_t chunk_records(size_t n, size_t total_bytes) {
    const size_t avg = std::max<size_t>(1, total_bytes / std::max<size_t>(n, 1));
    const size_t target = chunk_target_bytes(total_bytes);
    size_t c = 1;
    while (c < n && c < 65536 && (c * 2) * avg <= target) c *= 2;
    return c;
}

// Exclusive prefix sums of per-item values produced by val(i), in parallel ranges: out[0..n].
template <class V>
void prefix(size_t n, std::vector<uint64_t>& out, V&& val) {
    out.resize(n + 1);
    Workers& w = Workers::get();
    const size_t ntasks = n < 65536 ? 1 : std::min<size_t>(w.size() * 2, n / 16384);
    std::vector<uint64_t> part(ntasks + 1, 0);
    auto lo = [&](size_t t) { return n * t / ntasks; };
    w.parallel_for(ntasks, [&](size_t t) {
        uint64_t s = 0;
        for (size_t i = lo(t); i < lo(t + 1); ++i) {
            out[i] = s;
            s += val(i);
        }
        part[t + 1] = s;
    });
    for (size_t t = 0; t < ntasks; ++t) part[t + 1] += part[t];
    w.parallel_for(ntasks, [&](size_t t) {
        if (part[t])
            for (size_t i = lo(t); i < lo(t + 1); ++i) out[i] += part[t];
    });
    out[n] = part[ntasks];
}

// Two exclusive prefix sums in one pass: val(i, x, y) gives item i's two values.
template <class V>
void prefix2(size_t n, std::vector<uint64_t>& ox, std::vector<uint64_t>& oy, V&& val) {
    ox.resize(n + 1);
    oy.resize(n + 1);
    Workers& w = Workers::get();
    const size_t ntasks = n < 32768 ? 1 : std::min<size_t>(w.size() * 2, n / 8192);
    std::vector<uint64_t> px(ntasks + 1, 0), py(ntasks + 1, 0);
    auto lo = [&](size_t t) { return n * t / ntasks; };
    w.parallel_for(ntasks, [&](size_t t) {
        uint64_t sx = 0, sy = 0;
        for (size_t i = lo(t); i < lo(t + 1); ++i) {
            uint64_t x, y;
            val(i, x, y);
            ox[i] = sx;
            oy[i] = sy;
            sx += x;
            sy += y;
        }
        px[t + 1] = sx;
        py[t + 1] = sy;
    });
    for (size_t t = 0; t < ntasks; ++t) {
        px[t + 1] += px[t];
        py[t + 1] += py[t];
    }
    w.parallel_for(ntasks, [&](size_t t) {
        if (t == 0) return;
        for (size_t i = lo(t); i < lo(t + 1); ++i) {
            ox[i] += px[t];
            oy[i] += py[t];
        }
    });
    ox[n] = px[ntasks];
    oy[n] = py[ntasks];
}

}  // namespace

namespace detail {
struct HostBytesAccess {
    template <class T = uint8_t>
    static HostArray<T> make(size_t n) {
        HostArray<T> h;
        if (n) {
            h.block_ = PinnedPool::get().take(n * sizeof(T));
            h.p_ = static_cast<T*>(h.block_.get());
        }
        h.n_ = n;
        return h;
    }
    // n elements at p inside `block` (several arrays of one result share a block)
    template <class T>
    static HostArray<T> view(const std::shared_ptr<void>& block, void* p, size_t n) {
        HostArray<T> h;
        h.block_ = block;
        h.p_ = n ? static_cast<T*>(p) : nullptr;
        h.n_ = n;
        return h;
    }
    template <class T>
    static void zero(HostArray<T>& h) {
        if (h.n_) std::memset(static_cast<void*>(h.p_), 0, h.n_ * sizeof(T));
    }
};

// Host copy of the decode descriptors, chunk-major: chunk c (records [c*C, c*C + C)) is the
// device's struct of arrays for C records, copied back as one block.
struct Descriptors {
    std::shared_ptr<void> block;
    size_t n = 0;
    unsigned shift = 0;  // C = 1 << shift
    size_t chunk_bytes = 0;
    size_t o_fl = 0, o_hdr = 0, o_ts = 0, o_off = 0, o_len = 0, o_seq = 0;
    bool has_seq = false;

    void layout(size_t C, bool seq) {
        shift = 0;
        while ((size_t(1) << shift) < C) ++shift;
        o_fl = al16(C);
        o_hdr = o_fl + al16(C);
        o_ts = o_hdr + al16(8 * C);
        o_off = o_ts + al16(8 * C);
        o_len = o_off + al16(20 * C);
        o_seq = o_len + al16(20 * C);
        chunk_bytes = o_seq + (seq ? al16(8 * C) : 0);
        has_seq = seq;
    }
    const uint8_t* base(size_t i) const {
        return static_cast<const uint8_t*>(block.get()) + (i >> shift) * chunk_bytes;
    }
    size_t j(size_t i) const { return i & ((size_t(1) << shift) - 1); }
    uint8_t status(size_t i) const { return base(i)[j(i)]; }
    uint8_t flags(size_t i) const { return base(i)[o_fl + j(i)]; }
    const uint16_t* hdr(size_t i) const { return reinterpret_cast<const uint16_t*>(base(i) + o_hdr) + 4 * j(i); }
    uint64_t ts(size_t i) const { return reinterpret_cast<const uint64_t*>(base(i) + o_ts)[j(i)]; }
    const uint32_t* off(size_t i) const { return reinterpret_cast<const uint32_t*>(base(i) + o_off) + 5 * j(i); }
    const uint32_t* len(size_t i) const { return reinterpret_cast<const uint32_t*>(base(i) + o_len) + 5 * j(i); }
    // ParseResult.sequence_number: the device evaluates it for flagged TopicMessages only
    // (include/sbecodec.h, sbe_decoded.seq); every other record's is 0
    uint64_t seq(size_t i) const {
        if (!has_seq || status(i) != SBE_ST_TM || !(flags(i) & (SBE_FL_SEQ_KEY | SBE_FL_SEQ_ESC))) return 0;
        return reinterpret_cast<const uint64_t*>(base(i) + o_seq)[j(i)];
    }
};
}  // namespace detail

using detail::Descriptors;
using detail::HostBytesAccess;

namespace {

// [p, p + bytes) inside one page-locked host allocation (hipHostMalloc, or memory registered with
// host_register, e.g. an Aeron term buffer, or a HostBytes of this library): the copy engines read
// it in place, with no staging copy.
bool page_locked(const void* p, size_t bytes) {
    if (!p || bytes == 0) return false;
    uint8_t* dev = nullptr;
    if (PinnedRegistry::get().find(p, bytes, &dev)) return true;
    // memory page-locked outside this library (the caller's own hipHostMalloc) is found by the HIP
    // pointer query, which costs microseconds: asked only where that is small against the copy
    if (bytes < (size_t(1) << 20)) return false;
    hipPointerAttribute_t a{};
    if (hipPointerGetAttributes(&a, p) != hipSuccess) {
        (void)hipGetLastError();
        return false;
    }
    if (a.type != hipMemoryTypeHost) return false;
    void* start = nullptr;
    size_t size = 0;
    if (hipPointerGetAttribute(&start, HIP_POINTER_ATTRIBUTE_RANGE_START_ADDR, (hipDeviceptr_t)const_cast<void*>(p)) !=
            hipSuccess ||
        hipPointerGetAttribute(&size, HIP_POINTER_ATTRIBUTE_RANGE_SIZE, (hipDeviceptr_t)const_cast<void*>(p)) !=
            hipSuccess) {
        (void)hipGetLastError();
        return false;
    }
    return start && static_cast<const uint8_t*>(p) >= static_cast<const uint8_t*>(start) &&
           static_cast<const uint8_t*>(p) + bytes <= static_cast<const uint8_t*>(start) + size;
}

// Decode n records data[rec_off[i], rec_off[i+1]) with `mode` through the chunk pipeline.
// on_chunk(d, a, m), when given, runs on the calling thread for each chunk (records [a, a+m)) as
// soon as its descriptors are on the host, while the later chunks are still being copied and
// decoded: the host's work on chunk k overlaps the device's on chunk k+1.
using ChunkFn = std::function<void(const Descriptors&, size_t, size_t)>;

// The zero-copy path of a one-chunk decode: the offsets (and, unless the caller's bytes are
// page-locked already, the records) staged in the slot's page-locked buffer, which the kernel reads
// over PCIe; the descriptors written by the kernel straight into d.block.  One launch, one wait.
// false (nothing launched) when some buffer has no device address.
bool decode_zero_copy(Ctx& c, const uint8_t* data, const uint64_t* rec_off, size_t n, uint32_t mode, bool direct,
                      Descriptors& d) {
    Pipeline& P = c.pipe;
    Pipeline::Slot& sl = P.slot[0];  // serial use (the pipeline is idle between calls)
    const uint64_t lo = rec_off[0], bytes = rec_off[n] - lo;
    const size_t o_data = al16((n + 1) * 8);
    const bool parse = mode == SBE_DEC_PARSE_MESSAGE;
    // small batches: the serve kernel, inputs straight from the caller's memory into its request slot
    if (sbe_server* srv = c.server(n); srv && o_data + bytes <= SBE_SERVE_INLINE_BYTES) {
        uint8_t* dblk = static_cast<uint8_t*>(device_view(d.block.get()));
        if (dblk) {
            sbe_decoded out{dblk,
                            dblk + d.o_fl,
                            reinterpret_cast<uint16_t*>(dblk + d.o_hdr),
                            reinterpret_cast<uint64_t*>(dblk + d.o_ts),
                            reinterpret_cast<uint32_t*>(dblk + d.o_off),
                            reinterpret_cast<uint32_t*>(dblk + d.o_len),
                            parse ? reinterpret_cast<uint64_t*>(dblk + d.o_seq) : nullptr};
            if (sbe_serve_decode_host(srv, data, rec_off, n, mode, &out) == SBE_OK) return true;
            c.drop_server();  // the batch kernels take this call and every later one
        }
    }
    // the kernel reads its records from a 16-B aligned base: page-locked caller bytes are read from
    // the 16-B boundary below the first record (offsets rebased to it); staged bytes start aligned
    const uint64_t base = direct ? (lo & ~(uint64_t)15) : lo;
    sl.pin.need((direct ? o_data : o_data + (size_t)bytes) + 16);
    uint8_t* pin = sl.pin.b();
    uint64_t* ro = reinterpret_cast<uint64_t*>(pin);
    uint8_t* dpin = sl.pin.dev;
    uint8_t* dblk = static_cast<uint8_t*>(device_view(d.block.get()));
    const uint8_t* drec = direct ? static_cast<const uint8_t*>(device_view(data + base)) : (dpin ? dpin + o_data : nullptr);
    if (!dpin || !dblk || !drec || (reinterpret_cast<uintptr_t>(drec) & 15u)) return false;
    for_ranges(n + 1, 8192, [&](size_t x, size_t y) {
        for (size_t i = x; i < y; ++i) ro[i] = rec_off[i] - base;
    });
    if (!direct && bytes)
        for_ranges((size_t)bytes, size_t(1) << 16, [&](size_t x, size_t y) { copy_small(pin + o_data + x, data + lo + x, y - x); });
    sbe_decoded out{dblk,
                    dblk + d.o_fl,
                    reinterpret_cast<uint16_t*>(dblk + d.o_hdr),
                    reinterpret_cast<uint64_t*>(dblk + d.o_ts),
                    reinterpret_cast<uint32_t*>(dblk + d.o_off),
                    reinterpret_cast<uint32_t*>(dblk + d.o_len),
                    parse ? reinterpret_cast<uint64_t*>(dblk + d.o_seq) : nullptr};
    if (sbe_server* srv = c.server(n, true)) {  // inputs through the staging buffer, several workgroups
        if (sbe_serve_decode(srv, drec, reinterpret_cast<const uint64_t*>(dpin), n, mode, &out) == SBE_OK) return true;
        c.drop_server();
    }
    if (sbe_decode_batch_sized(drec, reinterpret_cast<const uint64_t*>(dpin), n, bytes, mode, &out, c.batch_stream()) !=
        SBE_OK) {
        c.abort_all();
        fail("sbe_decode_batch");
    }
    hip_check(hipStreamSynchronize(P.s_comp), "hipStreamSynchronize");
    return true;
}

std::shared_ptr<Descriptors> run_decode(const uint8_t* data, const uint64_t* rec_off, size_t n, uint32_t mode,
                                        const ChunkFn* on_chunk = nullptr) {
    auto d = std::make_shared<Descriptors>();
    d->n = n;
    if (n == 0) return d;
    Trace tr("decode");
    Ctx& c = ctx();
    Pipeline& P = c.pipe;
    const uint64_t base = rec_off[0], total = rec_off[n] - base;
    const size_t C = chunk_records(n, (size_t)total);
    const bool parse = mode == SBE_DEC_PARSE_MESSAGE;
    d->layout(C, parse);
    const size_t K = (n + C - 1) / C;
    P.serial = K == 1;
    const bool direct = page_locked(data + base, (size_t)total);  // no staging of the record bytes
    d->block = PinnedPool::get().take(K * d->chunk_bytes);
    uint8_t* hblk = static_cast<uint8_t*>(d->block.get());
    tr.lap(tr.plan);
    if (K == 1 && al16((n + 1) * 8) + (direct ? 0 : (size_t)total) <= zero_copy_max_bytes() &&
        decode_zero_copy(c, data, rec_off, n, mode, direct, *d)) {
        tr.lap(tr.sync);
        if (on_chunk) (*on_chunk)(*d, 0, n);
        tr.lap(tr.finish);
        tr.done(n, 0);
        return d;
    }
    PipeGuard guard(c);
    for (size_t k = 0; k < K; ++k) {
        const size_t a = k * C, m = std::min(n, a + C) - a;
        const uint64_t lo = rec_off[a], bytes = rec_off[a + m] - lo;
        const size_t o_data = al16((m + 1) * 8), in_bytes = o_data + bytes;
        Pipeline::Slot& sl = P.begin(k);
        tr.lap(tr.wait);
        sl.pin.need((direct ? o_data : in_bytes) + 16);
        uint8_t* pin = sl.pin.b();
        uint64_t* ro = reinterpret_cast<uint64_t*>(pin);
        // stage: the chunk's offsets rebased to 0 and (unless page-locked already) its bytes; on
        // the device the bytes start 16-B aligned after the offsets
        for_ranges(m + 1, 8192, [&](size_t x, size_t y) {
            for (size_t i = x; i < y; ++i) ro[i] = rec_off[a + i] - lo;
        });
        if (!direct)
            for_ranges((size_t)bytes, size_t(1) << 18, [&](size_t x, size_t y) {
                std::memcpy(pin + o_data + x, data + lo + x, y - x);
            });
        tr.lap(tr.stage);
        P.reserve(sl, in_bytes + 16, d->chunk_bytes);
        if (direct)
            P.copy_in(sl, (m + 1) * 8, data + lo, o_data, (size_t)bytes);
        else
            P.copy_in(sl, in_bytes);
        hipStream_t st = P.compute(sl);
        uint8_t* db = sl.d_out.b();
        sbe_decoded out{db,
                        db + d->o_fl,
                        reinterpret_cast<uint16_t*>(db + d->o_hdr),
                        reinterpret_cast<uint64_t*>(db + d->o_ts),
                        reinterpret_cast<uint32_t*>(db + d->o_off),
                        reinterpret_cast<uint32_t*>(db + d->o_len),
                        parse ? reinterpret_cast<uint64_t*>(db + d->o_seq) : nullptr};
        if (sbe_decode_batch_sized(sl.d_in.b() + o_data, reinterpret_cast<const uint64_t*>(sl.d_in.p), m, bytes, mode,
                                   &out, st) != SBE_OK)
            fail("sbe_decode_batch");
        st = P.copy_out(sl);
        hip_check(hipMemcpyAsync(hblk + k * d->chunk_bytes, db, d->chunk_bytes, hipMemcpyDeviceToHost, st), "D2H");
        P.end(sl);
        tr.lap(tr.enqueue);
        if (on_chunk && k > 0 && !P.serial) {  // chunk k-1, while chunk k is in flight
            hip_check(hipEventSynchronize(P.slot[(k - 1) % Pipeline::kSlots].out_done), "hipEventSynchronize");
            tr.lap(tr.sync);
            (*on_chunk)(*d, (k - 1) * C, std::min(n, k * C) - (k - 1) * C);
            tr.lap(tr.finish);
        }
    }
    c.sync_all();
    guard.release();
    tr.lap(tr.sync);
    if (on_chunk) {
        (*on_chunk)(*d, (K - 1) * C, n - (K - 1) * C);
        tr.lap(tr.finish);
    }
    tr.done(n, K);
    return d;
}

// Per-record output size of an encode (the plan the chunks are placed by; the device offsets are
// checked against it): overhead + Σ field lengths (PUBLISH_TOPIC: each mod 65536); a record with
// a field above 65534 B is an E109 and emits nothing.
struct EncodePlan {
    uint32_t overhead = 0;
    bool e109 = true;
    bool wrap16 = false;
    uint32_t layout = SBE_LAYOUT_TOPIC;  // tile shape of the kernels (planned serve encodes)
};

// Encode n records (nf strings, a u64 and a u32 each) through the chunk pipeline.  launch(...)
// issues one sbe_encode_*_batch call for a chunk on the given stream, or (server non-null: a small
// zero-copy batch) the synchronous sbe_serve_encode_* call (host_in: the inputs by their host
// addresses, the *_host form).
template <class Field, class U64, class U32, class Launch>
EncodedBatch run_encode(size_t n, int nf, Field&& field, U64&& u64, U32&& u32, EncodePlan plan, Launch&& launch) {
    EncodedBatch b;
    Trace tr("encode");
    if (n == 0) {
        b.offsets = HostBytesAccess::make<uint64_t>(1);
        b.offsets[0] = 0;
        return b;
    }
    Ctx& c = ctx();
    Pipeline& P = c.pipe;
    // per-record input (string) bytes and output bytes, prefixed, in one pass
    std::vector<uint64_t>& pin = c.pin;
    std::vector<uint64_t>& pout = c.pout;
    prefix2(n, pin, pout, [&](size_t i, uint64_t& in_b, uint64_t& out_b) {
        uint64_t si = 0, so = plan.overhead;
        bool e109 = false;
        for (int k = 0; k < nf; ++k) {
            const size_t L = field(i, k).size();
            si += L;
            so += plan.wrap16 ? (L & 0xFFFF) : L;
            e109 |= plan.e109 && L > SBE_VAR_MAX_LEN;
        }
        in_b = si;
        out_b = e109 ? 0 : so;
    });
    const size_t C = chunk_records(n, (size_t)(pin[n] + pout[n]) / 2);
    const size_t K = (n + C - 1) / C;
    P.serial = K == 1;
    {  // offsets | status | stream in one page-locked block (16-B aligned parts)
        const size_t o_st = al16((n + 1) * 8), o_by = o_st + al16(n);
        std::shared_ptr<void> blk = PinnedPool::get().take(o_by + (size_t)pout[n]);
        uint8_t* base = static_cast<uint8_t*>(blk.get());
        b.offsets = HostBytesAccess::view<uint64_t>(blk, base, n + 1);
        b.status = HostBytesAccess::view<uint8_t>(blk, base + o_st, n);
        b.bytes = HostBytesAccess::view<uint8_t>(blk, base + o_by, (size_t)pout[n]);
    }
    // staging layout of records [a, a + m): arena | u32 lengths [m][nf] | u64 [m] | u32 [m]
    struct Stage {
        size_t o_len, o_u64, o_u32, bytes;
    };
    auto stage_layout = [&](size_t a, size_t m) {
        const uint64_t in_bytes = pin[a + m] - pin[a];
        Stage s;
        s.o_len = al16((size_t)in_bytes);
        s.o_u64 = s.o_len + al16((size_t)m * 4 * nf);
        s.o_u32 = s.o_u64 + al16(m * 8);
        s.bytes = s.o_u32 + al16(m * 4);
        return s;
    };
    auto stage_fill = [&](uint8_t* p, const Stage& s, size_t a, size_t m) {
        const uint64_t in_lo = pin[a];
        uint32_t* lp = reinterpret_cast<uint32_t*>(p + s.o_len);
        uint64_t* up = reinterpret_cast<uint64_t*>(p + s.o_u64);
        uint32_t* wp = reinterpret_cast<uint32_t*>(p + s.o_u32);
        for_ranges(m, 1024, [&](size_t x, size_t y) {  // 256: 1 K-record encodes 5-9 us slower (wakes)
            for (size_t r = x; r < y; ++r) {
                const size_t i = a + r;
                uint8_t* at = p + (pin[i] - in_lo);
                for (int k2 = 0; k2 < nf; ++k2) {
                    const std::string_view f = field(i, k2);
                    copy_small(at, f.data(), f.size());
                    at += f.size();
                    lp[(size_t)nf * r + k2] = (uint32_t)f.size();
                }
                up[r] = u64(i);
                wp[r] = u32(i);
            }
        });
    };
    tr.lap(tr.plan);
    if (K == 1) {
        // zero-copy: the kernels read the page-locked staging buffer and write the stream, the
        // offsets and the status straight into the caller's page-locked result arrays
        const Stage s = stage_layout(0, n);
        Pipeline::Slot& sl = P.slot[0];
        if (s.bytes <= zero_copy_max_bytes()) {
            // one wave and inputs in its request slot (small batches), or several workgroups with
            // the tile sums of this plan after the staged inputs, or the batch launches
            sbe_server* srv = c.server(n);
            sbe_server* wsrv = srv ? nullptr : c.server(n, true);
            const size_t R = sbe_encode_tile_records(plan.layout), SB = 128 * R;
            const size_t tiles = (n + R - 1) / R, sbs = (n + SB - 1) / SB;
            const size_t o_sums = al16(s.bytes);
            sl.pin.need(wsrv ? o_sums + 16 * (tiles + sbs) : s.bytes);
            uint8_t* dp = sl.pin.dev;
            // offsets, status and stream share one block (above): one lookup for all three
            uint8_t* const hb = reinterpret_cast<uint8_t*>(b.offsets.data());
            uint8_t* const db = static_cast<uint8_t*>(device_view(hb));
            uint8_t* dbytes = db && pout[n] ? db + (b.bytes.data() - hb) : nullptr;
            uint64_t* doff = reinterpret_cast<uint64_t*>(db);
            uint8_t* dst = db ? db + (b.status.data() - hb) : nullptr;
            if (dp && doff && dst && (dbytes || pout[n] == 0)) {
                stage_fill(sl.pin.b(), s, 0, n);
                const uint64_t* tsums = nullptr;
                const uint64_t* bsums = nullptr;
                if (wsrv) {  // what sbe_enc_sums would compute, from the plan's prefix sums
                    uint64_t* ts = reinterpret_cast<uint64_t*>(sl.pin.b() + o_sums);
                    uint64_t* bs = ts + 2 * tiles;
                    for (size_t t = 0; t < tiles; ++t) {
                        const size_t r0 = t * R, b0 = (r0 / SB) * SB;
                        ts[2 * t] = pout[r0] - pout[b0];
                        ts[2 * t + 1] = pin[r0] - pin[b0];
                    }
                    for (size_t b = 0; b < sbs; ++b) {
                        const size_t r0 = b * SB, r1 = std::min(n, r0 + SB);
                        bs[2 * b] = pout[r1] - pout[r0];
                        bs[2 * b + 1] = pin[r1] - pin[r0];
                    }
                    tsums = reinterpret_cast<const uint64_t*>(dp + o_sums);
                    bsums = tsums + 2 * tiles;
                    srv = wsrv;
                }
                tr.lap(tr.stage);
                PipeGuard zguard(c);
                // a batch whose records all fail (E109) has no bytes: the kernels still want a
                // 16-B aligned output pointer, which they never write at capacity 0
                if (srv) {
                    c.d_ws.need(16);
                    // the single-wave serve takes the staged inputs by their host addresses (copied
                    // into its request slot when they fit, else read through their device addresses)
                    const uint8_t* ip = !wsrv && s.bytes <= SBE_SERVE_INLINE_BYTES ? sl.pin.b() : dp;
                    if (launch(srv, ip != dp, ip, reinterpret_cast<const uint32_t*>(ip + s.o_len),
                               reinterpret_cast<const uint64_t*>(ip + s.o_u64),
                               reinterpret_cast<const uint32_t*>(ip + s.o_u32), n, dbytes ? dbytes : c.d_ws.b(), pout[n],
                               doff, dst, c.d_ws.b(), 16, P.s_comp, tsums, bsums) != SBE_OK) {
                        c.drop_server();  // the batch kernels take this call and every later one
                        srv = nullptr;
                    }
                }
                if (!srv) {
                    const size_t ws_bytes = sbe_encode_workspace_size(n);
                    c.d_ws.need(ws_bytes);
                    hipStream_t st = c.batch_stream();
                    if (launch(nullptr, false, dp, reinterpret_cast<const uint32_t*>(dp + s.o_len),
                               reinterpret_cast<const uint64_t*>(dp + s.o_u64),
                               reinterpret_cast<const uint32_t*>(dp + s.o_u32), n, dbytes ? dbytes : c.d_ws.b(), pout[n],
                               doff, dst, c.d_ws.b(), ws_bytes, st, nullptr, nullptr) != SBE_OK)
                        fail("sbe_encode batch");
                    tr.lap(tr.enqueue);
                    hip_check(hipStreamSynchronize(st), "hipStreamSynchronize");
                }
                zguard.release();
                tr.lap(tr.sync);
                if (b.offsets[n] != pout[n]) throw std::logic_error("sbecodec: encoded batch size differs from its plan");
                tr.done(n, 0);
                return b;
            }
        }
    }
    // per-chunk device offsets (C + 1) and status (C), copied back beside each other
    const size_t meta_stride = al16((C + 1) * 8 + C);
    std::shared_ptr<void> meta = PinnedPool::get().take(K * meta_stride);
    uint8_t* hmeta = static_cast<uint8_t*>(meta.get());
    const size_t ws_bytes = sbe_encode_workspace_size(C);
    PipeGuard guard(c);
    for (size_t k = 0; k < K; ++k) {
        const size_t a = k * C, m = std::min(n, a + C) - a;
        const uint64_t out_lo = pout[a], out_bytes = pout[a + m] - out_lo;
        const Stage s = stage_layout(a, m);
        const size_t o_len = s.o_len, o_u64 = s.o_u64, o_u32 = s.o_u32, stage = s.bytes;
        Pipeline::Slot& sl = P.begin(k);
        tr.lap(tr.wait);
        sl.pin.need(stage);
        stage_fill(sl.pin.b(), s, a, m);
        tr.lap(tr.stage);
        // device: out bytes | out_off [m+1] | status [m] | workspace
        const size_t d_off = al16((size_t)out_bytes), d_ws = d_off + meta_stride;
        P.reserve(sl, stage, d_ws + ws_bytes);
        P.copy_in(sl, stage);
        hipStream_t st = P.compute(sl);
        const uint8_t* di = sl.d_in.b();
        uint8_t* dout = sl.d_out.b();
        if (launch(nullptr, false, di, reinterpret_cast<const uint32_t*>(di + o_len),
                   reinterpret_cast<const uint64_t*>(di + o_u64), reinterpret_cast<const uint32_t*>(di + o_u32), m, dout,
                   out_bytes, reinterpret_cast<uint64_t*>(dout + d_off), dout + d_off + (m + 1) * 8, dout + d_ws, ws_bytes,
                   st, nullptr, nullptr) != SBE_OK)
            fail("sbe_encode batch");
        st = P.copy_out(sl);
        if (out_bytes) hip_check(hipMemcpyAsync(b.bytes.data() + out_lo, dout, out_bytes, hipMemcpyDeviceToHost, st), "D2H");
        hip_check(hipMemcpyAsync(hmeta + k * meta_stride, dout + d_off, (m + 1) * 8 + m, hipMemcpyDeviceToHost, st), "D2H");
        P.end(sl);
        tr.lap(tr.enqueue);
    }
    c.sync_all();
    guard.release();
    tr.lap(tr.sync);
    for (size_t k = 0; k < K; ++k) {
        const size_t a = k * C, m = std::min(n, a + C) - a;
        const uint64_t* off = reinterpret_cast<const uint64_t*>(hmeta + k * meta_stride);
        if (off[m] != pout[a + m] - pout[a])
            throw std::logic_error("sbecodec: encoded chunk size differs from its plan");
    }
    for_ranges(n, 16384, [&](size_t x, size_t y) {
        for (size_t i = x; i < y; ++i) {
            const size_t k = i / C, j = i - k * C, m = std::min(n, k * C + C) - k * C;
            const uint8_t* mk = hmeta + k * meta_stride;
            b.offsets[i] = pout[k * C] + reinterpret_cast<const uint64_t*>(mk)[j];
            b.status[i] = mk[(m + 1) * 8 + j];
        }
    });
    b.offsets[n] = pout[n];
    tr.lap(tr.finish);
    tr.done(n, K);
    return b;
}

inline int64_t rdi64(const uint8_t* p) {
    uint64_t v = 0;
    for (int i = 7; i >= 0; --i) v = (v << 8) | p[i];
    return (int64_t)v;
}
inline int32_t rdi32(const uint8_t* p) { return (int32_t)((uint32_t)p[0] | (p[1] << 8) | (p[2] << 16) | ((uint32_t)p[3] << 24)); }
inline uint16_t rdu16(const uint8_t* p) { return (uint16_t)(p[0] | (p[1] << 8)); }

// r := the ParseResult of record i, every field rewritten; the strings are assigned in place, so a
// reused ParseResult keeps its buffers (parse_batch into a caller's vector allocates nothing once
// the strings have grown to the records' sizes)
void materialize_into(ParseResult& r, const uint8_t* rec, const Descriptors& d, size_t i) {
    r.success = false;
    r.timestamp = 0;
    r.sequence_number = 0;
    r.template_id = r.schema_id = r.version = r.block_length = 0;
    r.correlation_id = r.session_id = r.leadership_term_id = 0;
    r.leader_member_id = r.event_code = 0;
    r.sequence_key_present = false;
    const uint8_t st = d.status(i), fl = d.flags(i);
    const uint16_t* h = d.hdr(i);
    const uint32_t* off = d.off(i);
    const uint32_t* len = d.len(i);
    struct View {  // record bytes [off[k], off[k] + len[k]), assigned into a string in place
        const char* p;
        uint32_t n;
    };
    auto view = [&](int k) { return View{reinterpret_cast<const char*>(rec) + off[k], len[k]}; };
    // strings the status's branch writes (the others are cleared after it): resized only when the
    // length changes, so a reused ParseResult of the same shape is overwritten in place
    enum : unsigned { kType = 2, kId = 4, kPay = 8, kHdr = 16 };
    unsigned written = 0;
    auto set = [&](std::string& s, View v, unsigned which) {
        if (s.size() != v.n) s.resize(v.n);
        copy_small(s.data(), v.p, v.n);
        written |= which;
    };
    auto put = [&](std::string& s, std::string&& v, unsigned which) {
        s = std::move(v);
        written |= which;
    };
    auto take_hdr = [&] {
        r.block_length = h[0];
        r.template_id = h[1];
        r.schema_id = h[2];
        r.version = h[3];
    };
    const uint32_t param = off[0];
    switch (st) {
        case SBE_ST_TM:  // src/sbe_encoder.cpp:1021-1135
            r.success = true;
            set(r.message_type, view(1), kType);
            set(r.message_id, view(2), kId);
            set(r.payload, view(3), kPay);
            set(r.headers, view(4), kHdr);
            r.timestamp = (int64_t)d.ts(i);
            r.sequence_key_present = (fl & SBE_FL_SEQ_KEY) != 0;
            r.sequence_number = d.seq(i);  // src/sbe_encoder.cpp:1031-1125
            take_hdr();
            break;
        case SBE_ST_ACK:  // src/sbe_encoder.cpp:916-941
            r.success = true;
            set(r.message_type, View{"Acknowledgment", 14}, kType);
            r.timestamp = (int64_t)d.ts(i);
            if (fl & SBE_FL_ID_DEFAULT)
                put(r.message_id, "ack_" + std::to_string(d.ts(i)), kId);
            else
                set(r.message_id, view(0), kId);
            if (fl & SBE_FL_PAYLOAD_DEFAULT)
                set(r.payload, View{"SUCCESS", 7}, kPay);
            else
                set(r.payload, view(1), kPay);
            set(r.headers, view(2), kHdr);
            take_hdr();
            break;
        case SBE_ST_SESSION_EVENT:  // src/sbe_encoder.cpp:629-644 (SessionEvent layout sbe_messages.hpp:39-50)
            r.success = true;
            set(r.message_type, View{"SessionEvent", 12}, kType);
            r.correlation_id = rdi64(rec + 8);
            r.session_id = rdi64(rec + 16);
            r.leadership_term_id = rdi64(rec + 24);
            r.leader_member_id = rdi32(rec + 32);
            r.event_code = rdi32(rec + 36);
            set(r.payload, view(3), kPay);
            r.timestamp = 0;
            take_hdr();
            break;
        case SBE_ST_ERR_NULL_EMPTY: r.error_message = "Null or empty data"; break;
        case SBE_ST_ERR_HEADER: r.error_message = "Failed to decode message header"; break;
        case SBE_ST_ERR_UNKNOWN_TYPE:
            take_hdr();
            r.error_message = "Unknown message type: template=" + std::to_string(r.template_id) +
                              ", schema=" + std::to_string(r.schema_id);
            break;
        case SBE_ST_ERR_SESSION_EVENT: r.error_message = "Failed to decode SessionEvent"; break;
        case SBE_ST_ERR_SESSION_SHORT: r.error_message = "Session message too short to contain embedded message"; break;
        case SBE_ST_ERR_EMBEDDED_SHORT: r.error_message = "Embedded message too short"; break;
        case SBE_ST_ERR_EMBEDDED_TEMPLATE:
            r.error_message = "Unknown embedded message template_id: " + std::to_string(param);
            break;
        case SBE_ST_ERR_EMBEDDED_SCHEMA:
            r.error_message = "Unknown embedded message schema_id: " + std::to_string(param);
            break;
        case SBE_ST_ERR_DIRECT_TEMPLATE:
            r.error_message = "Unknown direct message template_id: " + std::to_string(param);
            break;
        case SBE_ST_ERR_TM_E100: r.error_message = "SBE TopicMessage decoding failed: buffer too short [E100]"; break;
        case SBE_ST_ERR_ACK_SHORT:
            r.error_message = "Buffer too short for Acknowledgment message. Need at least 16 bytes, got " +
                              std::to_string(param);
            break;
        default: throw std::runtime_error("sbecodec: unexpected parse status");
    }
    if (st < SBE_ST_ERR_NULL_EMPTY) r.error_message.clear();  // every error branch above sets it
    if (!(written & kType)) r.message_type.clear();
    if (!(written & kId)) r.message_id.clear();
    if (!(written & kPay)) r.payload.clear();
    if (!(written & kHdr)) r.headers.clear();
}

ParseResult materialize(const uint8_t* rec, const Descriptors& d, size_t i) {
    ParseResult r;
    materialize_into(r, rec, d, i);
    return r;
}

const char* kE109[5] = {"topicLength too long for length type [E109]", "messageTypeLength too long for length type [E109]",
                        "uuidLength too long for length type [E109]", "payloadLength too long for length type [E109]",
                        "headersLength too long for length type [E109]"};

std::string_view tm_field(const TopicMessageFields& m, int k) {
    switch (k) {
        case 0: return m.topic;
        case 1: return m.message_type;
        case 2: return m.uuid;
        case 3: return m.payload;
        default: return m.headers;
    }
}

uint64_t clock_ms() {
    return (uint64_t)std::chrono::duration_cast<std::chrono::milliseconds>(
               std::chrono::system_clock::now().time_since_epoch())
        .count();
}
uint64_t clock_ns() {
    return (uint64_t)std::chrono::duration_cast<std::chrono::nanoseconds>(
               std::chrono::high_resolution_clock::now().time_since_epoch())
        .count();
}
uint64_t now_nanos_sys() {  // include/aeron_cluster/protocol.hpp:31-34
    return (uint64_t)std::chrono::duration_cast<std::chrono::nanoseconds>(
               std::chrono::system_clock::now().time_since_epoch())
        .count();
}

EncodedBatch encode_tm(const std::vector<TopicMessageFields>& msgs, EncodeLength length, bool session, int64_t term,
                       int64_t sess, uint64_t ts_default) {
    const uint32_t flags = length == EncodeLength::Reference ? SBE_ENC_REF_TRUNCATE8
                         : length == EncodeLength::Publish   ? SBE_ENC_PUBLISH_TOPIC
                                                             : 0u;
    EncodePlan plan;
    plan.overhead = (length == EncodeLength::Reference ? SBE_TM_REF_OVERHEAD : SBE_TM_WIRE_OVERHEAD) +
                    (session ? SBE_SESSION_HDR_LEN : 0u);
    plan.e109 = length != EncodeLength::Publish;
    plan.wrap16 = length == EncodeLength::Publish;
    plan.layout = session ? SBE_LAYOUT_SESSION : SBE_LAYOUT_TOPIC;
    return run_encode(
        msgs.size(), 5, [&](size_t i, int k) { return tm_field(msgs[i], k); },
        [&](size_t i) { return (uint64_t)msgs[i].timestamp; }, [](size_t) { return 0u; }, plan,
        [&](sbe_server* srv, bool host_in, const uint8_t* arena, const uint32_t* len, const uint64_t* ts,
            const uint32_t*, size_t m, uint8_t* out, uint64_t cap, uint64_t* off, uint8_t* st, void* ws, size_t wsb,
            hipStream_t s, const uint64_t* tsums, const uint64_t* bsums) {
            sbe_tm_batch in{arena, nullptr, len, ts};
            int rc;
            if (srv && tsums)
                rc = session ? sbe_serve_encode_session_planned(srv, &in, m, ts_default, flags, term, sess, out, cap, off,
                                                                st, tsums, bsums)
                             : sbe_serve_encode_topic_planned(srv, &in, m, ts_default, flags, out, cap, off, st, tsums,
                                                              bsums);
            else if (srv && host_in)
                rc = session ? sbe_serve_encode_session_host(srv, &in, m, ts_default, flags, term, sess, out, cap, off, st)
                             : sbe_serve_encode_topic_host(srv, &in, m, ts_default, flags, out, cap, off, st);
            else if (srv)
                rc = session ? sbe_serve_encode_session(srv, &in, m, ts_default, flags, term, sess, out, cap, off, st)
                             : sbe_serve_encode_topic(srv, &in, m, ts_default, flags, out, cap, off, st);
            else
                rc = session ? sbe_encode_session_batch(&in, m, ts_default, flags, term, sess, out, cap, off, st, ws,
                                                        wsb, s)
                             : sbe_encode_topic_batch(&in, m, ts_default, flags, out, cap, off, st, ws, wsb, s);
            return rc;
        });
}

// DEBUG_LOG of the reference (include/aeron_cluster/debug_utils.hpp:11-28, 71): on stdout when
// AERON_CLUSTER_DEBUG=1
bool debug_enabled() {
    static const bool on = [] {
        const char* e = std::getenv("AERON_CLUSTER_DEBUG");
        return e && std::string(e) == "1";
    }();
    return on;
}
template <class... A>
void debug_log(const A&... a) {
    if (!debug_enabled()) return;
    std::cout << "[DEBUG] ";
    (std::cout << ... << a);
    std::cout << std::endl;
}

}  // namespace

// ======================================================================================
// SBEUtils (src/sbe_encoder.cpp:328-485) and ParseResult (sbe_messages.hpp:340-411)
// ======================================================================================
namespace SBEUtils {

void print_hex_dump(const std::uint8_t* data, std::size_t length, const std::string& prefix, std::size_t max_bytes) {
    if (!data || length == 0) return;
    const size_t shown = max_bytes > 0 ? std::min(length, max_bytes) : length;
    for (size_t row = 0; row < shown; row += 16) {
        std::cout << prefix << std::setfill('0') << std::setw(4) << std::hex << row << ": ";
        for (size_t j = 0; j < 16; ++j) {
            if (row + j < shown)
                std::cout << std::setfill('0') << std::setw(2) << std::hex << static_cast<unsigned>(data[row + j]) << " ";
            else
                std::cout << "   ";
            if (j == 7) std::cout << " ";
        }
        std::cout << " |";
        for (size_t j = 0; j < 16 && row + j < shown; ++j) {
            const char ch = static_cast<char>(data[row + j]);
            std::cout << ((ch >= 32 && ch <= 126) ? ch : '.');
        }
        std::cout << "|" << std::dec << std::endl;
    }
    if (max_bytes > 0 && length > max_bytes) std::cout << prefix << "... (" << (length - max_bytes) << " more bytes)" << std::endl;
}

std::string get_session_event_code_string(std::int32_t code) {
    switch (code) {
        case SBEConstants::SESSION_EVENT_OK: return "OK";
        case SBEConstants::SESSION_EVENT_ERROR: return "ERROR";
        case SBEConstants::SESSION_EVENT_AUTHENTICATION_REJECTED: return "AUTHENTICATION_REJECTED";
        case SBEConstants::SESSION_EVENT_REDIRECT: return "REDIRECT";
        case SBEConstants::SESSION_EVENT_CLOSED: return "CLOSED";
        default: return "UNKNOWN(" + std::to_string(code) + ")";
    }
}

std::string get_message_type_name(std::uint16_t template_id, std::uint16_t schema_id) {
    if (schema_id == SBEConstants::CLUSTER_SCHEMA_ID) {
        if (template_id == SBEConstants::SESSION_CONNECT_TEMPLATE_ID) return "SessionConnectRequest";
        if (template_id == SBEConstants::SESSION_EVENT_TEMPLATE_ID) return "SessionEvent";
        return "UnknownClusterMessage(" + std::to_string(template_id) + ")";
    }
    if (schema_id == SBEConstants::TOPIC_SCHEMA_ID) {
        if (template_id == SBEConstants::TOPIC_MESSAGE_TEMPLATE_ID) return "TopicMessage";
        if (template_id == SBEConstants::ACKNOWLEDGMENT_TEMPLATE_ID) return "Acknowledgment";
        return "UnknownTopicMessage(" + std::to_string(template_id) + ")";
    }
    return "UnknownSchema(" + std::to_string(schema_id) + "," + std::to_string(template_id) + ")";
}

bool is_valid_correlation_id(std::int64_t correlation_id) { return correlation_id > 0; }

std::int64_t generate_correlation_id() {
    return (std::int64_t)std::chrono::high_resolution_clock::now().time_since_epoch().count() & 0x7FFFFFFFFFFFFFFFLL;
}

std::string format_timestamp(std::int64_t timestamp) {
    const std::time_t secs = std::chrono::system_clock::to_time_t(
        std::chrono::time_point<std::chrono::system_clock>(std::chrono::nanoseconds(timestamp)));
    std::stringstream ss;
    ss << std::put_time(std::gmtime(&secs), "%Y-%m-%d %H:%M:%S UTC");
    ss << "." << std::setfill('0') << std::setw(9) << (timestamp % 1000000000);
    return ss.str();
}

bool is_valid_sbe_message(const std::uint8_t* data, std::size_t length) {
    if (!data || length < SBEConstants::SBE_HEADER_LENGTH) return false;
    const uint16_t blk = rdu16(data), schema = rdu16(data + 4);
    if (blk == 0 || blk > 10000) return false;
    if (length < SBEConstants::SBE_HEADER_LENGTH + blk) return false;
    return schema == SBEConstants::CLUSTER_SCHEMA_ID || schema == SBEConstants::TOPIC_SCHEMA_ID;
}

std::vector<std::string> extract_readable_strings(const std::uint8_t* data, std::size_t length, std::size_t min_length) {
    std::vector<std::string> out;
    if (!data || length == 0) return out;
    size_t start = 0;
    for (size_t i = 0; i <= length; ++i) {
        const bool printable = i < length && data[i] >= 32 && data[i] <= 126;
        if (printable) continue;
        if (i - start >= min_length) out.emplace_back(reinterpret_cast<const char*>(data) + start, i - start);
        start = i + 1;
    }
    return out;
}

}  // namespace SBEUtils

bool ParseResult::is_topic_message() const {
    if (template_id == SBEConstants::TOPIC_MESSAGE_TEMPLATE_ID && schema_id == SBEConstants::TOPIC_SCHEMA_ID) return true;
    if (schema_id == SBEConstants::CLUSTER_SCHEMA_ID && template_id == SBEConstants::TOPIC_MESSAGE_TEMPLATE_ID) return true;
    if (schema_id == SBEConstants::TOPIC_SCHEMA_ID && template_id == SBEConstants::SESSION_EVENT_TEMPLATE_ID) return true;
    if (!message_type.empty() &&
        (message_type.find("ORDER") != std::string::npos || message_type.find("TopicMessage") != std::string::npos ||
         message_type.find("CREATE_ORDER") != std::string::npos || message_type.find("UPDATE_ORDER") != std::string::npos))
        return true;
    return false;
}

bool ParseResult::is_order_message() const {
    if (!is_topic_message()) return false;
    // every keyword of the reference's type list contains "ORDER" (sbe_messages.hpp:386-391)
    if (!message_type.empty() && message_type.find("ORDER") != std::string::npos) return true;
    if (payload.empty()) return false;
    for (const char* k : {"order_details", "token_pair", "quantity", "side", "client_order_id"})
        if (payload.find(k) != std::string::npos) return true;
    return false;
}

std::string ParseResult::get_description() const {
    std::stringstream ss;
    if (success) {
        ss << SBEUtils::get_message_type_name(template_id, schema_id);
        if (is_session_event())
            ss << " (code: " << SBEUtils::get_session_event_code_string(event_code) << ")";
        else if (!message_type.empty())
            ss << " (type: " << message_type << ")";
        if (!message_id.empty()) ss << " [ID: " << message_id.substr(0, 8) << "...]";
    } else {
        ss << "Parse Error: " << error_message;
    }
    return ss.str();
}

// ======================================================================================
// SBEDecoder (src/sbe_encoder.cpp:174-323): one-record struct readers, host code (see the header)
// ======================================================================================
namespace {
// SBEDecoder::extract_variable_string (:285-318): a u32 length prefix at offset, the string after
// it; 0 (output untouched) when the prefix or the string does not fit or the length is over 10 MiB.
// The reference checks the length against `remaining - 4` whatever the offset (:302), so for a
// field after the first one a corrupt length can make it read up to `offset` bytes past the
// record (undefined behaviour on network input).  Here the string must end inside the record:
// identical results for every record the reference reads in bounds, a refusal for the others.
size_t extract_variable_string(const uint8_t* data, size_t offset, size_t remaining, std::string& output) {
    if (offset + sizeof(uint32_t) > remaining) {
        debug_log("[ERROR] Not enough data for length prefix at offset ", offset, ", remaining: ", remaining);
        return 0;
    }
    uint32_t length;
    std::memcpy(&length, data + offset, sizeof(uint32_t));
    debug_log("[DEBUG] Extracting string at offset ", offset, ", length prefix: ", length, ", remaining: ", remaining);
    offset += sizeof(uint32_t);
    if (length > remaining - offset || length > 10u * 1024u * 1024u) {
        debug_log("[ERROR] Invalid string length: ", length, ", remaining data: ", (remaining - sizeof(uint32_t)));
        return 0;
    }
    if (length > 0) {
        output.assign(reinterpret_cast<const char*>(data + offset), length);
        offset += length;
        debug_log("[DEBUG] Extracted string: \"", output, "\"");
    } else {
        output.clear();
        debug_log("[DEBUG] Extracted empty string");
    }
    return offset;
}
}  // namespace

bool SBEDecoder::decode_message_header(const std::uint8_t* data, std::size_t length, MessageHeader& header) {
    if (!data || length < sizeof(MessageHeader)) return false;
    std::memcpy(&header, data, sizeof(MessageHeader));
    return true;
}

bool SBEDecoder::decode_session_event(const std::uint8_t* data, std::size_t length, SessionEvent& event,
                                      std::string& detail) {
    if (!data || length < sizeof(MessageHeader) + SessionEvent::sbe_block_length()) return false;
    if (debug_enabled()) {  // the reference's raw-data diagnostics (:189-214)
        debug_log("Raw data analysis (", length, " bytes)");
        debug_log("Hex dump: ");
        for (size_t i = 0; i < length && i < 64; ++i) {
            debug_log("0x", static_cast<unsigned>(data[i]), " ");
            if ((i + 1) % 16 == 0) debug_log("\n          ");
        }
        debug_log("Readable content: ");
        std::string readable;
        for (size_t i = 0; i < length && i < 256; ++i) {
            const char ch = static_cast<char>(data[i]);
            if (ch >= 32 && ch <= 126) {
                readable += ch;
            } else if (!readable.empty()) {
                if (readable.length() >= 3) debug_log("\"", readable, "\" ");
                readable.clear();
            }
        }
        if (readable.length() >= 3) debug_log("\"", readable, "\"");
    }
    MessageHeader header;
    if (!decode_message_header(data, length, header)) return false;
    if (!(header.template_id == SessionEvent::sbe_template_id() && header.schema_id == SessionEvent::sbe_schema_id()))
        return false;
    std::memcpy(&event, data + sizeof(MessageHeader), SessionEvent::sbe_block_length());
    const size_t remaining = length - sizeof(MessageHeader) - SessionEvent::sbe_block_length();
    if (remaining > 0)
        extract_variable_string(data + sizeof(MessageHeader) + SessionEvent::sbe_block_length(), 0, remaining, detail);
    return true;
}

bool SBEDecoder::decode_acknowledgment(const std::uint8_t* data, std::size_t length, std::string& message_id,
                                       std::string& status, std::string& error, std::int64_t& timestamp) {
    constexpr size_t kAckBlock = 8;  // Acknowledgment::sbe_block_length() (sbe_messages.hpp:106-118)
    if (!data || length < sizeof(MessageHeader) + kAckBlock) return false;
    MessageHeader header;
    if (!decode_message_header(data, length, header)) return false;
    if (!(header.template_id == SBEConstants::ACKNOWLEDGMENT_TEMPLATE_ID && header.schema_id == SBEConstants::TOPIC_SCHEMA_ID))
        return false;
    const uint8_t* ptr = data + sizeof(MessageHeader);
    std::memcpy(&timestamp, ptr, sizeof(int64_t));
    ptr += kAckBlock;
    const size_t remaining = length - sizeof(MessageHeader) - kAckBlock;
    size_t offset = extract_variable_string(ptr, 0, remaining, message_id);
    if (offset == 0) return false;
    offset = extract_variable_string(ptr, offset, remaining, status);
    if (offset == 0) return false;
    if (offset < remaining) extract_variable_string(ptr, offset, remaining, error);
    return true;
}

std::int64_t SBEEncoder::get_current_timestamp() {
    return (std::int64_t)std::chrono::high_resolution_clock::now().time_since_epoch().count();
}

void quiesce() { ctx().quiesce(); }

bool gpu_codec_available() { return sbe_device_ready() == 1; }
unsigned host_threads() { return Workers::get().size(); }

void host_register(const void* p, std::size_t len) {
    hip_check(hipHostRegister(const_cast<void*>(p), len, hipHostRegisterDefault), "hipHostRegister");
    PinnedRegistry::get().add(p, len);
}
void host_unregister(const void* p) {
    PinnedRegistry::get().remove(p);
    hip_check(hipHostUnregister(const_cast<void*>(p)), "hipHostUnregister");
}

// ======================================================================================
// encode
// ======================================================================================
EncodedBatch SBEEncoder::encode_topic_batch(const std::vector<TopicMessageFields>& msgs, EncodeLength length) {
    Trace tr("encode_topic_batch");
    // timestamp 0 → the clock the reference reads (src/sbe_encoder.cpp:134-138)
    EncodedBatch b = encode_tm(msgs, length, false, 0, 0, clock_ms());
    tr.done(msgs.size(), 0);
    return b;
}

std::vector<std::uint8_t> SBEEncoder::encode_topic_message(const std::string& topic, const std::string& message_type,
                                                           const std::string& uuid, const std::string& payload,
                                                           const std::string& headers, std::int64_t timestamp) {
    TopicMessageFields f{topic, message_type, uuid, payload, headers, timestamp};
    EncodedBatch b = encode_topic_batch({f}, EncodeLength::Reference);
    const uint8_t st = b.status[0];
    if (st >= SBE_ENC_E109_TOPIC && st <= SBE_ENC_E109_HEADERS) throw std::runtime_error(kE109[st - 1]);
    if (st != SBE_ENC_OK) throw std::runtime_error("sbecodec: encode failed");
    return b.bytes.to_vector();
}

EncodedBatch SessionFrameEncoder::encode_batch(const std::vector<TopicMessageFields>& msgs, EncodeLength length) const {
    // create_topic_message stamps high_resolution_clock nanoseconds (src/session_manager.cpp:1075-1076)
    return encode_tm(msgs, length, true, leadership_term_id_, cluster_session_id_, clock_ns());
}

std::vector<std::uint8_t> SessionFrameEncoder::create_combined_message(const std::string& topic,
                                                                       const std::string& message_type,
                                                                       const std::string& message_id,
                                                                       const std::string& payload,
                                                                       const std::string& headers) const {
    TopicMessageFields f{topic, message_type, message_id, payload, headers, 0};
    EncodedBatch b = encode_batch({f}, EncodeLength::Reference);
    const uint8_t st = b.status[0];
    if (st >= SBE_ENC_E109_TOPIC && st <= SBE_ENC_E109_HEADERS) throw std::runtime_error(kE109[st - 1]);
    if (st != SBE_ENC_OK) throw std::runtime_error("sbecodec: encode failed");
    return b.bytes.to_vector();
}

std::vector<std::string> TopicPublisher::publish_topic_batch(const std::vector<TopicMessageFields>& msgs) {
    const size_t n = msgs.size();
    std::vector<std::string> uuids(n);
    std::vector<TopicMessageFields> f(msgs);
    for (size_t i = 0; i < n; ++i) {
        uuids[i] = std::string("pub_") + std::to_string(now_nanos_sys());  // src/cluster_client.cpp:1818
        f[i].uuid = uuids[i];
        if (f[i].headers.empty()) f[i].headers = "{}";                     // :1821
        f[i].timestamp = (int64_t)now_nanos_sys();                         // :1845
    }
    EncodedBatch b = encode_tm(f, EncodeLength::Publish, false, 0, 0, now_nanos_sys());
    for (size_t i = 0; i < n; ++i) (void)offer_(b.bytes.data() + b.offsets[i], b.offsets[i + 1] - b.offsets[i]);
    return uuids;
}

std::string TopicPublisher::publish_topic(std::string_view topic, std::string_view message_type,
                                          std::string_view json_payload, std::string_view headers_json) {
    TopicMessageFields m{topic, message_type, {}, json_payload, headers_json, 0};
    return publish_topic_batch({m})[0];
}

std::uint32_t CommitManager::topic_to_id(const std::string& topic) {
    if (topic == "order_request_topic") return 1;
    if (topic == "order_notification_topic") return 2;
    if (topic == "orders") return 3;
    if (topic == "order_status_request_topic") return 4;
    return 0;
}

EncodedBatch CommitManager::build_commit_offset_batch(const std::vector<CommitOffset>& offsets) const {
    std::vector<uint32_t> ids(offsets.size());
    for (size_t i = 0; i < offsets.size(); ++i) {
        ids[i] = topic_to_id(offsets[i].topic);
        if (ids[i] == 0)
            throw std::runtime_error("sbecodec: commit offset for unknown topic '" + offsets[i].topic +
                                     "' needs the jsoncpp TopicMessage fallback (not built)");
    }
    EncodePlan plan;
    plan.overhead = SBE_LITE_OVERHEAD(2);
    plan.layout = SBE_LAYOUT_LITE;
    return run_encode(
        offsets.size(), 2,
        [&](size_t i, int k) { return std::string_view(k == 0 ? offsets[i].message_id : offsets[i].message_identifier); },
        [&](size_t i) { return offsets[i].sequence_number; }, [&](size_t i) { return ids[i]; }, plan,
        [&](sbe_server* srv, bool host_in, const uint8_t* arena, const uint32_t* len, const uint64_t* seq,
            const uint32_t* tid, size_t m, uint8_t* out, uint64_t cap, uint64_t* off, uint8_t* st, void* ws, size_t wsb,
            hipStream_t s, const uint64_t* tsums, const uint64_t* bsums) {
            sbe_lite_batch in{arena, nullptr, len, tid, seq};
            const int rc =
                srv && tsums ? sbe_serve_encode_lite_planned(srv, &in, m, SBE_COMMIT_OFFSET_LITE_TEMPLATE_ID, out, cap,
                                                             off, st, tsums, bsums)
                : srv && host_in ? sbe_serve_encode_lite_host(srv, &in, m, SBE_COMMIT_OFFSET_LITE_TEMPLATE_ID, out, cap, off, st)
                : srv          ? sbe_serve_encode_lite(srv, &in, m, SBE_COMMIT_OFFSET_LITE_TEMPLATE_ID, out, cap, off, st)
                               : sbe_encode_lite_batch(&in, m, SBE_COMMIT_OFFSET_LITE_TEMPLATE_ID, out, cap, off, st, ws,
                                                       wsb, s);
            return rc;
        });
}

std::vector<std::uint8_t> CommitManager::build_commit_offset_message(const std::string& topic,
                                                                     const std::string& client_id,
                                                                     const CommitOffset& offset) const {
    (void)topic;  // the reference keys the template on offset.topic (src/commit_manager.cpp:110)
    (void)client_id;
    EncodedBatch b = build_commit_offset_batch({offset});
    static const char* kLiteE109[2] = {"messageIdLength too long for length type [E109]",
                                       "messageIdentifierLength too long for length type [E109]"};
    const uint8_t st = b.status[0];
    if (st == 1 || st == 2) throw std::runtime_error(kLiteE109[st - 1]);
    if (st != SBE_ENC_OK) throw std::runtime_error("sbecodec: encode failed");
    return b.bytes.to_vector();
}

OrderJsonBatch orders_to_json(const std::vector<Order>& orders, const std::vector<std::string>& message_ids) {
    const size_t n = orders.size();
    if (message_ids.size() != n) throw std::invalid_argument("orders_to_json: one message id per order");
    OrderJsonBatch r;
    for (EncodedBatch* b : {&r.payload, &r.headers}) {
        b->offsets = HostBytesAccess::make<uint64_t>(n + 1);
        b->status = HostBytesAccess::make<uint8_t>(n);
        HostBytesAccess::zero(b->offsets);
        HostBytesAccess::zero(b->status);
    }
    if (n == 0) return r;
    auto field = [&](size_t i, int k) -> std::string_view {
        const Order& o = orders[i];
        switch (k) {
            case 0: return o.client_order_uuid;
            case 1: return o.identifier;
            case 2: return o.base_token;
            case 3: return o.quote_token;
            case 4: return o.side;
            case 5: return o.id;
            case 6: return message_ids[i];
            default: return o.status;
        }
    };
    Ctx& c = ctx();
    Pipeline::Slot& s = c.pipe.slot[0];  // serial use of the pipeline's first slot (idle between calls)
    hipStream_t stream = c.batch_stream();
    std::vector<uint64_t> pin;
    prefix(n, pin, [&](size_t i) {
        uint64_t t = 0;
        for (int k = 0; k < (int)SBE_ORDER_FIELDS; ++k) t += field(i, k).size();
        return t;
    });
    const size_t arena = (size_t)pin[n];
    const size_t o_len = al16(arena), nlen = n * 4 * SBE_ORDER_FIELDS, o_num = o_len + al16(nlen), stage = o_num + n * 24;
    s.pin.need(stage);
    uint8_t* ap = s.pin.b();
    uint32_t* lp = reinterpret_cast<uint32_t*>(ap + o_len);
    int64_t* cid = reinterpret_cast<int64_t*>(ap + o_num);
    int64_t* ts = cid + n;
    double* q = reinterpret_cast<double*>(ts + n);
    for_ranges(n, 2048, [&](size_t x, size_t y) {
        for (size_t i = x; i < y; ++i) {
            uint8_t* at = ap + pin[i];
            for (int k = 0; k < (int)SBE_ORDER_FIELDS; ++k) {
                const std::string_view f = field(i, k);
                if (!f.empty()) std::memcpy(at, f.data(), f.size());
                at += f.size();
                lp[SBE_ORDER_FIELDS * i + k] = (uint32_t)f.size();
            }
            cid[i] = orders[i].customer_id;
            ts[i] = orders[i].timestamp;
            q[i] = orders[i].quantity;
        }
    });
    // a record is at most ~800 B besides its strings (428 fixed, 316 for "%f" of a quantity near
    // DBL_MAX, 24 for "%.17g", 34 for two integers); strings escape to <= 6x and appear <= twice.
    // out_off always holds the full sizes, so a record past the capacity is redone below.
    uint64_t cap = 12 * (uint64_t)arena + 900 * (uint64_t)n + 16;
    s.d_in.need(stage);
    const size_t o_off = 0, o_st = al16(2 * (n + 1) * 8), o_ws = o_st + al16(2 * n);
    const size_t wsb = sbe_order_json_workspace_size(n);
    c.d_aux.need(o_ws + wsb);
    hip_check(hipMemcpyAsync(s.d_in.p, ap, stage, hipMemcpyHostToDevice, stream), "H2D");
    const uint8_t* di = s.d_in.b();
    const int64_t* d_cid = reinterpret_cast<const int64_t*>(di + o_num);
    sbe_order_batch in{di, nullptr, reinterpret_cast<const uint32_t*>(di + o_len), d_cid, d_cid + n,
                       reinterpret_cast<const double*>(d_cid + 2 * n)};
    for (int w = 0; w < 2; ++w) {
        EncodedBatch& b = w ? r.headers : r.payload;
        uint64_t* off = reinterpret_cast<uint64_t*>(c.d_aux.b() + o_off) + w * (n + 1);
        uint8_t* st = c.d_aux.b() + o_st + w * n;
        for (int attempt = 0;; ++attempt) {
            s.d_out.need(cap);
            if (sbe_order_to_json_batch(&in, n, w ? SBE_JSON_PUBLISH_HEADERS : SBE_JSON_ORDER_PAYLOAD, s.d_out.b(), cap,
                                        off, st, c.d_aux.b() + o_ws, wsb, stream) != SBE_OK)
                fail("sbe_order_to_json_batch");
            hip_check(hipMemcpyAsync(b.offsets.data(), off, (n + 1) * 8, hipMemcpyDeviceToHost, stream), "D2H");
            hip_check(hipMemcpyAsync(b.status.data(), st, n, hipMemcpyDeviceToHost, stream), "D2H");
            hip_check(hipStreamSynchronize(stream), "sync");
            if (b.offsets[n] <= cap || attempt > 0) break;
            cap = b.offsets[n];  // the measured size: one rerun
        }
        for (size_t i = 0; i < n; ++i)
            if (b.status[i] != SBE_JSON_OK) throw std::runtime_error("sbecodec: order JSON record did not fit");
        b.bytes = HostBytesAccess::make((size_t)b.offsets[n]);
        if (b.offsets[n]) {
            hip_check(hipMemcpyAsync(b.bytes.data(), s.d_out.p, b.offsets[n], hipMemcpyDeviceToHost, stream), "D2H");
            hip_check(hipStreamSynchronize(stream), "sync");
        }
    }
    return r;
}

std::string Order::to_json() const {
    OrderJsonBatch b = orders_to_json({*this}, {std::string()});
    return std::string(b.payload.bytes.begin(), b.payload.bytes.end());
}

// ======================================================================================
// decode
// ======================================================================================
ParseResult MessageParser::parse_message(const std::uint8_t* data, std::size_t length) {
    if (!data || length == 0) {  // src/sbe_encoder.cpp:516-519 (no device round trip needed)
        ParseResult r;
        r.error_message = "Null or empty data";
        return r;
    }
    const uint64_t off[2] = {0, length};
    auto d = run_decode(data, off, 1, SBE_DEC_PARSE_MESSAGE);
    return materialize(data, *d, 0);
}

ParseResult MessageParser::decode_topic_message_with_sbe(const std::uint8_t* data, std::size_t length) {
    ParseResult r;
    if (!data || length < SBEConstants::SBE_HEADER_LENGTH) {  // MessageHeader::wrap (MessageHeader.h:165-168)
        r.error_message = "SBE TopicMessage decoding failed: buffer too short for flyweight [E107]";
        return r;
    }
    const uint16_t tmpl = rdu16(data + 2), schema = rdu16(data + 4);
    if (tmpl != SBEConstants::TOPIC_MESSAGE_TEMPLATE_ID || schema != SBEConstants::TOPIC_SCHEMA_ID) {  // :976-983
        r.error_message = "Not a TopicMessage (got template_id=" + std::to_string(tmpl) +
                          ", schema_id=" + std::to_string(schema) + ")";
        return r;
    }
    // template 1 / schema 1: parse_message dispatches straight to this function (:539-541, :812-816)
    return parse_message(data, length);
}

ParseResult MessageParser::decode_acknowledgment_with_sbe(const std::uint8_t* data, std::size_t length) {
    ParseResult r;
    if (!data || length < SBEConstants::SBE_HEADER_LENGTH) {  // :842-845
        r.error_message = "Buffer too short for SBE header";
        return r;
    }
    const uint16_t tmpl = rdu16(data + 2), schema = rdu16(data + 4);
    if (tmpl != SBEConstants::ACKNOWLEDGMENT_TEMPLATE_ID || schema != SBEConstants::TOPIC_SCHEMA_ID) {  // :859-865
        r.error_message = "Message is not an Acknowledgment. Expected: template_id=2, schema_id=1. Got: template_id=" +
                          std::to_string(tmpl) + ", schema_id=" + std::to_string(schema);
        return r;
    }
    // template 2 / schema 1: is_topic_message()'s third clause sends parse_message here (:539-541, :817-819)
    return parse_message(data, length);
}

ParseResult MessageParser::parse_message_debug(const std::uint8_t* data, std::size_t length, const std::string& debug_prefix) {
    debug_log(debug_prefix, "📋 Parsing message (", length, " bytes)");
    if (length > 0 && length <= 200) {
        debug_log(debug_prefix, "📋 Hex dump:");
        SBEUtils::print_hex_dump(data, length, debug_prefix + "  ", 64);
    }
    ParseResult result = parse_message(data, length);
    debug_log(debug_prefix, "📋 Parse result: ", (result.success ? "SUCCESS" : "FAILED"));
    debug_log(debug_prefix, "📋 Description: ", result.get_description());
    if (!result.success) {
        debug_log(debug_prefix, "📋 Error: ", result.error_message);
        const auto strings = SBEUtils::extract_readable_strings(data, length, 3);
        if (!strings.empty()) {
            debug_log(debug_prefix, "📋 Readable strings found:");
            for (const auto& str : strings) debug_log(debug_prefix, "  \"", str, "\"");
        }
    }
    return result;
}

std::string MessageParser::get_message_type(const std::uint8_t* data, std::size_t length) {
    if (!data || length < SBEConstants::SBE_HEADER_LENGTH) return "INVALID";
    return SBEUtils::get_message_type_name(rdu16(data + 2), rdu16(data + 4));
}

std::int64_t MessageParser::extract_correlation_id(const std::uint8_t* data, std::size_t length) {
    if (!data || length < SBEConstants::SBE_HEADER_LENGTH + 8) return 0;
    if (rdu16(data + 4) != SBEConstants::CLUSTER_SCHEMA_ID) return 0;
    return rdi64(data + 8);
}

bool MessageParser::is_acknowledgment_for(const std::uint8_t* data, std::size_t length, const std::string& message_id) {
    const ParseResult r = parse_message(data, length);
    if (!r.success || !r.is_acknowledgment()) return false;
    return r.message_id == message_id || r.payload.find(message_id) != std::string::npos ||
           r.headers.find(message_id) != std::string::npos;
}

std::vector<ParseResult> MessageParser::parse_batch(const std::uint8_t* data, const std::uint64_t* rec_off, std::size_t n) {
    std::vector<ParseResult> out;
    parse_batch(data, rec_off, n, out);
    return out;
}

void MessageParser::parse_batch(const std::uint8_t* data, const std::uint64_t* rec_off, std::size_t n,
                                std::vector<ParseResult>& out) {
    if (out.size() != n) out.resize(n);
    if (n == 0) return;
    // each chunk's ParseResults are built while the next chunk is on the device
    const ChunkFn fill = [&](const Descriptors& d, size_t a, size_t m) {
        for_ranges(m, 256, [&](size_t x, size_t y) {
            for (size_t i = a + x; i < a + y; ++i) materialize_into(out[i], data + rec_off[i], d, i);
        });
    };
    run_decode(data, rec_off, n, SBE_DEC_PARSE_MESSAGE, &fill);
}

// ---- BatchingParser -------------------------------------------------------------------------
// One batch fills on the caller's thread; handed-off batches queue for the decode thread (its own
// device context), which decodes them in order, and wait, decoded, for the caller's next poll() /
// flush() to deliver them in order.  Options::batches batches are kept (more are made when the
// caller hands off faster than it polls), so a decode overlaps both the next fill and the previous
// delivery: with two batches a 1024-record batch's decode (a serve round trip, ~20 us) could not,
// and each hand-off paid two futex wake-ups (the decode thread's, then the caller's): 23 M rec/s,
// below one CPU thread of the restatement (profiles/r05_host_latency.log).  Waits spin on an
// atomic for a while before they block (states change under the mutex, so a waiter that blocks
// cannot miss the notification).  Handlers run only inside poll() / flush(): on_fragment never
// delivers, so it never throws a handler's exception and never drops the fragment it is given.
struct BatchingParser::Impl {
    using clk = std::chrono::steady_clock;
    enum State : int { kFilling, kDecoding, kReady };
    struct Batch {
        // page-locked (a block of the library's pool, so a new parser reuses the blocks of earlier
        // ones instead of pinning fresh memory): the one-chunk decode reads it in place
        std::shared_ptr<void> blk;
        size_t cap = 0;
        size_t bytes = 0;
        uint8_t* b() const { return static_cast<uint8_t*>(blk.get()); }
        std::vector<uint64_t> off{0};
        ParsedBatch pb;  // the device descriptors; ParseResults are built at delivery
        std::atomic<int> state{kFilling};
        size_t done = 0;  // records already handed to the handler (a throwing handler resumes here)
        clk::time_point first{};
        std::exception_ptr err;
        size_t n() const { return off.size() - 1; }
        void reset() {
            bytes = 0;
            off.resize(1);
            done = 0;
            err = nullptr;
            pb = ParsedBatch();
            state.store(kFilling, std::memory_order_release);
        }
    };
    Handler handler;
    Options opt;
    std::vector<std::unique_ptr<Batch>> all;  // every batch (owner)
    std::vector<Batch*> spare;                // free batches (caller's thread)
    std::deque<Batch*> inflight;              // handed off, oldest first (caller's thread)
    Batch* cur = nullptr;                     // the filling batch
    ParseResult res;  // the result handed to the handler (rewritten in place per record)
    uint64_t n_delivered = 0;
    mutable std::mutex m;
    std::condition_variable cv;
    std::deque<Batch*> todo;                  // the decode thread's queue (under m)
    std::atomic<size_t> todo_n{0};
    std::atomic<bool> stop{false};
    std::thread worker;

    Impl(Handler h, Options o) : handler(std::move(h)), opt(o) {
        if (sbe_device_ready() != 1) fail("no gfx950 device visible");  // as every mirror entry point
        if (opt.max_records == 0) opt.max_records = 1;
        opt.batches = std::max<size_t>(2, std::min<size_t>(opt.batches, 64));
        for (size_t i = 0; i < opt.batches; ++i) spare.push_back(make_batch());
        cur = take();
        worker = std::thread([this] { run(); });
    }
    ~Impl() {
        {
            std::lock_guard<std::mutex> g(m);
            stop.store(true);
        }
        cv.notify_all();
        worker.join();
    }
    Batch* make_batch() {
        all.push_back(std::make_unique<Batch>());
        all.back()->off.reserve(opt.max_records + 1);
        return all.back().get();
    }
    Batch* take() {
        if (spare.empty()) return make_batch();
        Batch* x = spare.back();
        spare.pop_back();
        return x;
    }
    // spin (up to opt.spin) on pred, then block on the condition variable
    template <class Pred>
    void wait_for(Pred pred) {
        if (pred()) return;
        const auto until = clk::now() + opt.spin;
        while (clk::now() < until) {
            for (int k = 0; k < 64; ++k) {
                if (pred()) return;
#if defined(__x86_64__)
                __builtin_ia32_pause();
#endif
            }
        }
        std::unique_lock<std::mutex> g(m);
        cv.wait(g, pred);
    }
    void run() {  // the decode thread: batches in hand-off order
        for (;;) {
            wait_for([&] { return stop.load() || todo_n.load(std::memory_order_acquire) > 0; });
            Batch* x = nullptr;
            {
                std::lock_guard<std::mutex> g(m);
                if (todo.empty()) {
                    if (stop.load()) return;
                    continue;
                }
                x = todo.front();
                todo.pop_front();
                todo_n.fetch_sub(1, std::memory_order_relaxed);
            }
            try {
                x->pb = MessageParser::decode_batch(x->b(), x->off.data(), x->n());
            } catch (...) {
                x->err = std::current_exception();
            }
            {
                std::lock_guard<std::mutex> g(m);
                x->state.store(kReady, std::memory_order_release);
            }
            cv.notify_all();
        }
    }
    void hand_off() {  // the filling batch to the decode thread; filling goes on in a free batch
        Batch* x = cur;
        x->state.store(kDecoding, std::memory_order_relaxed);
        {
            std::lock_guard<std::mutex> g(m);
            todo.push_back(x);
            todo_n.fetch_add(1, std::memory_order_release);
        }
        cv.notify_all();
        inflight.push_back(x);
        cur = take();
    }
    // the oldest in-flight batch, decoded; a handler that throws leaves it at the front with `done`
    // past the record that threw, so the next call resumes after it
    size_t deliver_front() {
        Batch& x = *inflight.front();
        size_t got = 0;
        if (x.err) {
            std::exception_ptr e = x.err;
            n_delivered += x.n() - x.done;  // the batch's records are consumed by the error
            inflight.pop_front();
            x.reset();
            spare.push_back(&x);
            std::rethrow_exception(e);
        }
        // each result built on this thread into one reused ParseResult right before its handler
        // (the record and the result stay in this core's cache; the reference's handler likewise
        // receives a ParseResult that lives for the call, src/cluster_client.cpp:1185-1190)
        const size_t n = x.n();
        while (x.done < n) {
            const size_t i = x.done++;
            ++n_delivered;
            ++got;
            x.pb.result_into(i, res);
            handler(res);
        }
        inflight.pop_front();
        x.reset();
        spare.push_back(&x);
        return got;
    }
    size_t deliver_ready() {  // in order, up to the first batch still decoding
        size_t got = 0;
        while (!inflight.empty() && inflight.front()->state.load(std::memory_order_acquire) == kReady)
            got += deliver_front();
        return got;
    }
    size_t deliver_all() {
        size_t got = 0;
        while (!inflight.empty()) {
            Batch* x = inflight.front();
            wait_for([&] { return x->state.load(std::memory_order_acquire) == kReady; });
            got += deliver_front();
        }
        return got;
    }
};

BatchingParser::BatchingParser(Handler handler) : BatchingParser(std::move(handler), Options{}) {}
BatchingParser::BatchingParser(Handler handler, Options options)
    : impl_(std::make_unique<Impl>(std::move(handler), options)) {}
BatchingParser::~BatchingParser() {
    for (int k = 0; k < 1000000; ++k) {  // every record given is delivered (a throwing handler's
        try {                            // exception is dropped here: a destructor cannot throw)
            flush();
            return;
        } catch (...) {
        }
    }
}

void BatchingParser::on_fragment(const std::uint8_t* data, std::size_t length) {
    Impl& I = *impl_;
    if (I.cur->n() > 0 && (I.cur->n() + 1 > I.opt.max_records || I.cur->bytes + length > I.opt.max_bytes))
        I.hand_off();
    Impl::Batch& f = *I.cur;
    if (f.bytes + length > f.cap) {  // grow, keeping the bytes already copied
        const size_t want = std::max(f.bytes + length, std::max(I.opt.max_bytes, (size_t)4096));
        std::shared_ptr<void> nb = PinnedPool::get().take(want);
        if (f.bytes) std::memcpy(nb.get(), f.blk.get(), f.bytes);
        f.blk = std::move(nb);
        f.cap = want;
    }
    if (f.n() == 0) f.first = Impl::clk::now();
    if (length) copy_small(f.b() + f.bytes, data, length);
    f.bytes += length;
    f.off.push_back(f.bytes);
}

std::size_t BatchingParser::poll() {
    Impl& I = *impl_;
    // the filling batch goes first when its deadline has passed, so its decode overlaps the
    // delivery of the older ones
    if (I.cur->n() > 0 && Impl::clk::now() - I.cur->first >= I.opt.max_delay) I.hand_off();
    return I.deliver_ready();
}

std::size_t BatchingParser::flush() {
    Impl& I = *impl_;
    if (I.cur->n() > 0) I.hand_off();
    return I.deliver_all();
}

std::size_t BatchingParser::pending() const {
    const Impl& I = *impl_;
    size_t p = I.cur->n();
    for (const Impl::Batch* x : I.inflight) p += x->n() - x->done;
    return p;
}

std::uint64_t BatchingParser::delivered() const { return impl_->n_delivered; }

ParsedBatch MessageParser::decode_batch(const std::uint8_t* data, const std::uint64_t* rec_off, std::size_t n) {
    ParsedBatch b;
    b.desc_ = run_decode(data, rec_off, n, SBE_DEC_PARSE_MESSAGE);
    b.data_ = data;
    b.rec_off_ = rec_off;
    b.n_ = n;
    return b;
}

ParseResult ParsedBatch::result(std::size_t i) const { return materialize(data_ + rec_off_[i], *desc_, i); }
void ParsedBatch::result_into(std::size_t i, ParseResult& out) const {
    materialize_into(out, data_ + rec_off_[i], *desc_, i);
}
bool ParsedBatch::success(std::size_t i) const { return desc_->status(i) < SBE_ST_ERR_NULL_EMPTY; }
std::uint8_t ParsedBatch::status(std::size_t i) const { return desc_->status(i); }
std::uint16_t ParsedBatch::template_id(std::size_t i) const {
    const uint8_t st = desc_->status(i);
    return (st < SBE_ST_ERR_NULL_EMPTY || st == SBE_ST_ERR_UNKNOWN_TYPE) ? desc_->hdr(i)[1] : 0;
}
std::uint16_t ParsedBatch::schema_id(std::size_t i) const {
    const uint8_t st = desc_->status(i);
    return (st < SBE_ST_ERR_NULL_EMPTY || st == SBE_ST_ERR_UNKNOWN_TYPE) ? desc_->hdr(i)[2] : 0;
}
std::int64_t ParsedBatch::timestamp(std::size_t i) const {
    const uint8_t st = desc_->status(i);
    return (st == SBE_ST_TM || st == SBE_ST_ACK) ? (int64_t)desc_->ts(i) : 0;
}
std::uint64_t ParsedBatch::sequence_number(std::size_t i) const { return desc_->seq(i); }
std::string_view ParsedBatch::view(std::size_t i, int field) const {
    if (field < 0 || field > 4 || desc_->status(i) >= SBE_ST_ERR_NULL_EMPTY) return {};
    return {reinterpret_cast<const char*>(data_ + rec_off_[i]) + desc_->off(i)[field], desc_->len(i)[field]};
}
void ParsedBatch::for_each(const std::function<void(std::size_t, const ParseResult&)>& fn) const {
    const size_t block = 4096;
    std::vector<ParseResult> buf[1];
    auto build = [&](size_t k, std::vector<ParseResult>& v) {
        const size_t a = k * block, m = std::min(n_, a + block) - a;
        v.resize(m);
        for_ranges(m, 256, [&](size_t x, size_t y) {
            for (size_t r = x; r < y; ++r) v[r] = result(a + r);
        });
    };
    const size_t K = (n_ + block - 1) / block;
    for (size_t k = 0; k < K; ++k) {  // a block's ParseResults on the workers, then fn in order
        build(k, buf[0]);
        for (size_t r = 0; r < buf[0].size(); ++r) fn(k * block + r, buf[0][r]);
    }
}

namespace {
std::optional<AckInfo> ack_from(const uint8_t* rec, const Descriptors& d, size_t i) {
    const uint8_t st = d.status(i);
    if (st != SBE_ST_EG_ACK_SIMPLE && st != SBE_ST_EG_ACK) return std::nullopt;
    AckInfo a;
    a.timestamp_nanos = d.ts(i);
    a.simple_control_ack = st == SBE_ST_EG_ACK_SIMPLE;
    if (st == SBE_ST_EG_ACK) {
        const uint32_t* off = d.off(i);
        const uint32_t* len = d.len(i);
        auto v = [&](int k) { return std::string(reinterpret_cast<const char*>(rec) + off[k], len[k]); };
        a.message_id = v(0);
        a.topic = v(1);
        a.correlation_id = v(2);
    }
    return a;
}
}  // namespace

std::optional<AckInfo> decode_ack(const std::uint8_t* data, std::size_t len) {
    if (!data || len < 8) return std::nullopt;  // src/ack_decoder.cpp:30
    const uint64_t off[2] = {0, len};
    auto d = run_decode(data, off, 1, SBE_DEC_ON_EGRESS);
    return ack_from(data, *d, 0);
}

std::optional<LiteRecord> decode_lite(const std::uint8_t* data, std::size_t len) {
    if (!data || len < 8) return std::nullopt;
    const uint64_t off[2] = {0, len};
    auto d = run_decode(data, off, 1, SBE_DEC_LITE);
    if (d->status(0) != SBE_ST_LITE) return std::nullopt;
    LiteRecord r;
    r.template_id = d->hdr(0)[1];
    r.topic_id = d->off(0)[4];
    r.sequence = d->ts(0);
    const int nf = (int)sbe_lite_fields(r.template_id);
    for (int k = 0; k < nf; ++k) r.fields.emplace_back(reinterpret_cast<const char*>(data) + d->off(0)[k], d->len(0)[k]);
    return r;
}

EncodedBatch FragmentReassembler::on_fragments(const std::uint8_t* data, const std::uint64_t* frag_off,
                                               const std::uint8_t* flags, std::size_t n) {
    Ctx& c = ctx();
    Pipeline::Slot& s = c.pipe.slot[0];  // serial use of the pipeline's first slot (idle between calls)
    hipStream_t stream = c.batch_stream();
    EncodedBatch b;
    // the accumulator so far goes first as a middle fragment (flags 0): it is appended to exactly
    // as the reference's acc_ would be, or cleared by a BEGIN
    const size_t pre = acc_.empty() ? 0 : 1, nf = n + pre;
    if (nf == 0) {
        b.offsets = HostBytesAccess::make<uint64_t>(1);
        b.offsets[0] = 0;
        return b;
    }
    const uint64_t base = n ? frag_off[0] : 0, body = n ? frag_off[n] - base : 0, total = acc_.size() + body;
    const size_t o_fl = (nf + 1) * 8, o_data = al16(o_fl + nf), stage = o_data + total;
    s.pin.need(stage + 16);
    uint8_t* hp = s.pin.b();
    uint64_t* ho = reinterpret_cast<uint64_t*>(hp);
    uint8_t* hf = hp + o_fl;
    std::memcpy(hp + o_data, acc_.data(), acc_.size());
    if (body) std::memcpy(hp + o_data + acc_.size(), data + base, body);
    ho[0] = 0;
    if (pre) {
        ho[1] = acc_.size();
        hf[0] = 0;
    }
    for (size_t i = 0; i < n; ++i) {
        ho[pre + i + 1] = acc_.size() + (frag_off[i + 1] - base);
        hf[pre + i] = flags[i];
    }
    s.d_in.need(stage + 16);
    const size_t d_off = al16(total), d_cnt = d_off + (nf + 1) * 8, d_ws = al16(d_cnt + 16);
    const size_t wsb = sbe_reassemble_workspace_size(nf);
    s.d_out.need(d_ws + wsb);
    hip_check(hipMemcpyAsync(s.d_in.p, hp, stage, hipMemcpyHostToDevice, stream), "H2D");
    uint8_t* dout = s.d_out.b();
    uint64_t* dmo = reinterpret_cast<uint64_t*>(dout + d_off);
    uint64_t* dcnt = reinterpret_cast<uint64_t*>(dout + d_cnt);
    if (sbe_reassemble_fragments(s.d_in.b() + o_data, reinterpret_cast<const uint64_t*>(s.d_in.p), s.d_in.b() + o_fl, nf,
                                 dout, dmo, dcnt, dout + d_ws, wsb, stream) != SBE_OK)
        fail("sbe_reassemble_fragments");
    c.h_aux.need(16);
    uint64_t* counts = reinterpret_cast<uint64_t*>(c.h_aux.p);
    hip_check(hipMemcpyAsync(counts, dcnt, 16, hipMemcpyDeviceToHost, stream), "D2H");
    hip_check(hipStreamSynchronize(stream), "sync");
    const uint64_t m = counts[0], carry = counts[1];
    b.offsets = HostBytesAccess::make<uint64_t>(m + 1);
    b.status = HostBytesAccess::make<uint8_t>(m);
    HostBytesAccess::zero(b.status);
    hip_check(hipMemcpyAsync(b.offsets.data(), dmo, (m + 1) * 8, hipMemcpyDeviceToHost, stream), "D2H");
    hip_check(hipStreamSynchronize(stream), "sync");
    const uint64_t msg_bytes = b.offsets[m];
    b.bytes = HostBytesAccess::make((size_t)msg_bytes);
    acc_.resize(carry);
    if (msg_bytes) hip_check(hipMemcpyAsync(b.bytes.data(), dout, msg_bytes, hipMemcpyDeviceToHost, stream), "D2H");
    if (carry) hip_check(hipMemcpyAsync(acc_.data(), dout + msg_bytes, carry, hipMemcpyDeviceToHost, stream), "D2H");
    hip_check(hipStreamSynchronize(stream), "sync");
    return b;
}

MessageHandler::MessageHandler() = default;
MessageHandler::~MessageHandler() = default;

void MessageHandler::handleMessage(const ParseResult& result) {
    // src/message_handler.cpp:10-16: std::cout << std::string, so every byte of the string is
    // written (embedded NULs included), then std::endl
    if (result.success)
        std::cout << "[MessageHandler] Handled message: " << result.message_type << std::endl;
    else
        std::cout << "[MessageHandler] Failed to handle message: " << result.error_message << std::endl;
}

void MessageHandler::on_egress(const std::uint8_t* data, std::size_t len) {
    if (len < 8) return;
    const uint64_t off[2] = {0, len};
    on_egress_batch(data, off, 1);
}

void MessageHandler::on_egress_batch(const std::uint8_t* data, const std::uint64_t* rec_off, std::size_t n) {
    auto d = run_decode(data, rec_off, n, SBE_DEC_ON_EGRESS);
    for (size_t i = 0; i < n; ++i) {
        const uint8_t* rec = data + rec_off[i];
        switch (d->status(i)) {
            case SBE_ST_EG_ACK_SIMPLE:
            case SBE_ST_EG_ACK:
                if (ack_cb_) ack_cb_(*ack_from(rec, *d, i));
                break;
            case SBE_ST_EG_TM:
                if (tm_cb_) {
                    const uint32_t* off = d->off(i);
                    const uint32_t* len = d->len(i);
                    auto v = [&](int k) { return std::string_view(reinterpret_cast<const char*>(rec) + off[k], len[k]); };
                    tm_cb_(v(0), v(1), v(2), v(3), v(4));
                }
                break;
            case SBE_ST_EG_THROW_E100: throw std::runtime_error("buffer too short [E100]");
            default: break;  // SBE_ST_EG_NONE
        }
    }
}

std::size_t offer_batch(const EncodedBatch& batch, const OfferFn& offer) {
    const size_t n = batch.offsets.empty() ? 0 : batch.offsets.size() - 1;
    for (size_t i = 0; i < n; ++i) {
        if (batch.offsets[i + 1] == batch.offsets[i]) continue;  // failed record (status != 0)
        if (!offer(batch.bytes.data() + batch.offsets[i], batch.offsets[i + 1] - batch.offsets[i])) return i;
    }
    return n;
}

}  // namespace aeron_cluster
