// mock_rccl.cpp — TEST INFRASTRUCTURE ONLY: a stand-in for librccl that runs the ranks of a
// communicator as threads of ONE process on ONE device, so that the product's multi-rank gather
// (sbe_gather_encoded, aeron-cluster-client-cpp_amd/csrc/sbe_codec.hip) executes its size
// all-gather, its grouped ncclSend / ncclRecv into the root's prefix offsets and the root's offset
// rebase at world > 1 on a one-GPU box.  The product loads it only when the test-only environment
// variable SBE_RCCL_LIB names it; by default it loads the real RCCL.
//
// Semantics (the subset sbe_gather_encoded uses): ncclGetUniqueId / ncclCommInitRank /
// ncclCommDestroy / ncclAllGather / ncclSend / ncclRecv / ncclGroupStart / ncclGroupEnd /
// ncclGetErrorString.  Every call is host-synchronous: the caller's stream is synchronised before
// its buffers are read or written, the copies are issued on the CALLER'S stream (never the null
// stream) and the call returns once that stream has drained, so the stream order of the caller's
// later work holds.  Point-to-point transfers are matched by (sender, receiver, sequence number),
// as RCCL matches them.
//
// Every wait is bounded (SBE_MOCK_DEADLINE_S, default 60 s): on expiry the waiting rank prints
// the world's whole state (all-gather counters, mailbox keys, which rank waits on what) to stderr
// and ends the process with _Exit(1), so a stall names its wait instead of dying silently at the
// test runner's limit.  SBE_MOCK_TRACE=1 prints every call as it starts and ends.
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <atomic>
#include <chrono>
#include <condition_variable>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <map>
#include <memory>
#include <mutex>
#include <string>
#include <tuple>
#include <vector>

namespace {

using Clock = std::chrono::steady_clock;

double now_s() {
    static const Clock::time_point t0 = Clock::now();
    return std::chrono::duration<double>(Clock::now() - t0).count();
}

std::chrono::seconds deadline() {
    static const long s = [] {
        const char* e = std::getenv("SBE_MOCK_DEADLINE_S");
        const long v = e ? std::atol(e) : 0;
        return v > 0 ? v : 60L;
    }();
    return std::chrono::seconds(s);
}

bool tracing() {
    static const bool t = [] {
        const char* e = std::getenv("SBE_MOCK_TRACE");
        return e && *e && *e != '0';
    }();
    return t;
}

struct World {
    std::string name;
    int size = 0;
    std::mutex m;
    std::condition_variable cv;
    // all-gather rendezvous
    uint64_t ag_gen = 0;
    int ag_arrived = 0, ag_left = 0;
    std::vector<const void*> ag_src;
    // point-to-point mailbox: (src, dst, seq) -> posted send
    struct Post {
        const void* p;
        size_t bytes;
        bool taken = false;
    };
    std::map<std::tuple<int, int, uint64_t>, Post> box;
    // what each rank is blocked on (for the stall report); guarded by m
    std::vector<std::string> waiting;
};

std::mutex g_worlds_m;
std::map<std::string, std::shared_ptr<World>> g_worlds;
std::atomic<uint64_t> g_id_counter{1};

// called with w.m held: the stall report, then the process ends
[[noreturn]] void stall(World& w, int rank, const char* what) {
    std::fprintf(stderr, "[mock_rccl %.3fs] STALL: rank %d waited %lld s in %s (world %s, size %d)\n", now_s(), rank,
                 (long long)deadline().count(), what, w.name.c_str(), w.size);
    std::fprintf(stderr, "  all-gather: gen %llu arrived %d left %d\n", (unsigned long long)w.ag_gen, w.ag_arrived,
                 w.ag_left);
    for (int r = 0; r < w.size; ++r)
        std::fprintf(stderr, "  rank %d: %s\n", r, w.waiting[r].empty() ? "(not waiting)" : w.waiting[r].c_str());
    std::fprintf(stderr, "  mailbox (%zu posts):\n", w.box.size());
    for (auto& [k, p] : w.box)
        std::fprintf(stderr, "    src %d -> dst %d seq %llu: %zu B %s\n", std::get<0>(k), std::get<1>(k),
                     (unsigned long long)std::get<2>(k), p.bytes, p.taken ? "taken" : "pending");
    std::fflush(stderr);
    std::_Exit(1);
}

// wait on w.cv until pred(), bounded; `what` names the wait for the report
template <class Pred>
void bounded_wait(World& w, std::unique_lock<std::mutex>& g, int rank, const std::string& what, Pred pred) {
    w.waiting[rank] = what;
    if (!w.cv.wait_for(g, deadline(), pred)) stall(w, rank, what.c_str());
    w.waiting[rank].clear();
}

size_t dtype_bytes(ncclDataType_t t) {
    switch (t) {
        case ncclInt8:
        case ncclUint8: return 1;
        case ncclInt32:
        case ncclUint32:
        case ncclFloat32: return 4;
        case ncclInt64:
        case ncclUint64:
        case ncclFloat64: return 8;
        default: return 0;
    }
}

struct Op {
    bool send;
    void* p;
    size_t bytes;
    int peer;
    hipStream_t stream;
};
thread_local int t_group_depth = 0;
thread_local std::vector<std::pair<ncclComm_t, Op>> t_ops;

// a device-to-device copy ordered on the caller's stream, complete on return
bool stream_copy(void* dst, const void* src, size_t bytes, hipStream_t s) {
    if (!bytes) return true;
    if (hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToDevice, s) != hipSuccess) return false;
    return hipStreamSynchronize(s) == hipSuccess;
}

}  // namespace

struct ncclComm {
    std::shared_ptr<World> w;
    int rank = 0;
    std::map<int, uint64_t> send_seq, recv_seq;  // per peer
};

namespace {

void trace(const ncclComm* c, const char* what, const char* phase) {
    if (!tracing()) return;
    std::fprintf(stderr, "[mock_rccl %.3fs] %s rank %d %s %s\n", now_s(), c->w->name.c_str(), c->rank, what, phase);
}

ncclResult_t run_ops(std::vector<std::pair<ncclComm_t, Op>>& ops) {
    if (ops.empty()) return ncclSuccess;
    // every stream involved was synchronised when its op was queued (p2p below)
    std::vector<std::tuple<ncclComm_t, std::tuple<int, int, uint64_t>>> my_sends;
    for (auto& [c, op] : ops) {  // post the sends first (non-blocking)
        if (!op.send) continue;
        World& w = *c->w;
        const uint64_t seq = c->send_seq[op.peer]++;
        auto key = std::make_tuple(c->rank, op.peer, seq);
        {
            std::lock_guard<std::mutex> g(w.m);
            w.box[key] = World::Post{op.p, op.bytes, false};
        }
        w.cv.notify_all();
        my_sends.emplace_back(c, key);
    }
    ncclResult_t r = ncclSuccess;
    for (auto& [c, op] : ops) {  // then every receive: wait for its matching send, copy
        if (op.send) continue;
        World& w = *c->w;
        const uint64_t seq = c->recv_seq[op.peer]++;
        auto key = std::make_tuple(op.peer, c->rank, seq);
        World::Post post{};
        {
            std::unique_lock<std::mutex> g(w.m);
            bounded_wait(w, g, c->rank,
                         "recv from " + std::to_string(op.peer) + " seq " + std::to_string(seq) + " (" +
                             std::to_string(op.bytes) + " B): waiting for the matching send",
                         [&] { return w.box.count(key) != 0; });
            post = w.box[key];
        }
        if (post.bytes != op.bytes) {
            std::fprintf(stderr, "[mock_rccl] rank %d: recv of %zu B from %d matched a send of %zu B\n", c->rank,
                         op.bytes, op.peer, post.bytes);
            r = ncclInvalidArgument;
        } else if (!stream_copy(op.p, post.p, op.bytes, op.stream)) {
            r = ncclUnhandledCudaError;
        }
        {  // mark it taken whatever happened, so the sender is never left waiting
            std::lock_guard<std::mutex> g(w.m);
            w.box[key].taken = true;
        }
        w.cv.notify_all();
    }
    for (auto& [c, key] : my_sends) {  // the senders' buffers stay valid until their receives are done
        World& w = *c->w;
        std::unique_lock<std::mutex> g(w.m);
        bounded_wait(w, g, c->rank,
                     "send to " + std::to_string(std::get<1>(key)) + " seq " + std::to_string(std::get<2>(key)) +
                         ": waiting for the receiver to take it",
                     [&] { return w.box[key].taken; });
        w.box.erase(key);
    }
    return r;
}

}  // namespace

extern "C" {

ncclResult_t ncclGetUniqueId(ncclUniqueId* id) {
    if (!id) return ncclInvalidArgument;
    std::memset(id, 0, sizeof(*id));
    const uint64_t k = g_id_counter.fetch_add(1);
    std::snprintf(id->internal, sizeof(id->internal), "mock-rccl-%llu", (unsigned long long)k);
    return ncclSuccess;
}

// not a rendezvous here (RCCL's is): the ranks of a world may be initialised one after another
ncclResult_t ncclCommInitRank(ncclComm_t* comm, int nranks, ncclUniqueId id, int rank) {
    if (!comm || nranks < 1 || rank < 0 || rank >= nranks) return ncclInvalidArgument;
    const std::string key(id.internal, strnlen(id.internal, sizeof(id.internal)));
    std::shared_ptr<World> w;
    {
        std::lock_guard<std::mutex> g(g_worlds_m);
        auto& slot = g_worlds[key];
        if (!slot) {
            slot = std::make_shared<World>();
            slot->name = key;
            slot->size = nranks;
            slot->ag_src.assign(nranks, nullptr);
            slot->waiting.assign(nranks, std::string());
        }
        w = slot;
    }
    if (w->size != nranks) return ncclInvalidArgument;
    auto* c = new ncclComm;
    c->w = w;
    c->rank = rank;
    *comm = c;
    return ncclSuccess;
}

ncclResult_t ncclCommDestroy(ncclComm_t comm) {
    delete comm;
    return ncclSuccess;
}

// every rank's `count` elements of sendbuff land at rank * count of every rank's recvbuff
ncclResult_t ncclAllGather(const void* sendbuff, void* recvbuff, size_t count, ncclDataType_t dt, ncclComm_t comm,
                           hipStream_t stream) {
    const size_t eb = dtype_bytes(dt);
    if (!comm || !eb) return ncclInvalidArgument;
    trace(comm, "AllGather", "enter");
    if (hipStreamSynchronize(stream) != hipSuccess) return ncclUnhandledCudaError;
    World& w = *comm->w;
    const size_t bytes = count * eb;
    std::unique_lock<std::mutex> g(w.m);
    bounded_wait(w, g, comm->rank, "all-gather: waiting for the previous round to drain",
                 [&] { return w.ag_left == 0; });
    const uint64_t gen = w.ag_gen;
    w.ag_src[comm->rank] = sendbuff;
    if (++w.ag_arrived == w.size) {
        w.ag_left = w.size;
        w.cv.notify_all();
    }
    bounded_wait(w, g, comm->rank, "all-gather gen " + std::to_string(gen) + ": waiting for every rank to arrive",
                 [&] { return w.ag_arrived == w.size && w.ag_gen == gen; });
    std::vector<const void*> src = w.ag_src;
    g.unlock();
    ncclResult_t r = ncclSuccess;
    for (int q = 0; q < w.size && r == ncclSuccess; ++q)
        if (bytes && hipMemcpyAsync(static_cast<uint8_t*>(recvbuff) + q * bytes, src[q], bytes,
                                    hipMemcpyDeviceToDevice, stream) != hipSuccess)
            r = ncclUnhandledCudaError;
    if (hipStreamSynchronize(stream) != hipSuccess) r = ncclUnhandledCudaError;
    g.lock();
    if (--w.ag_left == 0) {  // the last one out opens the next round
        w.ag_arrived = 0;
        ++w.ag_gen;
        w.cv.notify_all();
    } else {
        // a sender's buffer stays valid until every rank has copied from it
        bounded_wait(w, g, comm->rank,
                     "all-gather gen " + std::to_string(gen) + ": waiting for every rank to finish copying",
                     [&] { return w.ag_gen != gen; });
    }
    g.unlock();
    trace(comm, "AllGather", "leave");
    return r;
}

ncclResult_t ncclGroupStart() {
    ++t_group_depth;
    return ncclSuccess;
}

ncclResult_t ncclGroupEnd() {
    if (t_group_depth <= 0) return ncclInvalidUsage;
    if (--t_group_depth > 0) return ncclSuccess;
    std::vector<std::pair<ncclComm_t, Op>> ops;
    ops.swap(t_ops);
    if (!ops.empty()) trace(ops.front().first, "GroupEnd", "enter");
    const ncclResult_t r = run_ops(ops);
    if (!ops.empty()) trace(ops.front().first, "GroupEnd", "leave");
    return r;
}

static ncclResult_t p2p(bool send, const void* buf, size_t count, ncclDataType_t dt, int peer, ncclComm_t comm,
                        hipStream_t stream) {
    const size_t eb = dtype_bytes(dt);
    if (!comm || !eb || peer < 0 || peer >= comm->w->size) return ncclInvalidArgument;
    if (hipStreamSynchronize(stream) != hipSuccess) return ncclUnhandledCudaError;
    t_ops.push_back({comm, Op{send, const_cast<void*>(buf), count * eb, peer, stream}});
    if (t_group_depth == 0) {  // outside a group: the op runs now
        std::vector<std::pair<ncclComm_t, Op>> ops;
        ops.swap(t_ops);
        return run_ops(ops);
    }
    return ncclSuccess;
}

ncclResult_t ncclSend(const void* sendbuff, size_t count, ncclDataType_t dt, int peer, ncclComm_t comm,
                      hipStream_t stream) {
    return p2p(true, sendbuff, count, dt, peer, comm, stream);
}

ncclResult_t ncclRecv(void* recvbuff, size_t count, ncclDataType_t dt, int peer, ncclComm_t comm, hipStream_t stream) {
    return p2p(false, recvbuff, count, dt, peer, comm, stream);
}

const char* ncclGetErrorString(ncclResult_t r) { return r == ncclSuccess ? "no error" : "mock rccl error"; }

}  // extern "C"
