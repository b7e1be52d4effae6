// Compile check of INTEGRATION.md's C / C++ snippets, verbatim, against include/sbecodec.h and the
// host mirror's header (tests/test_integration_snippets.py extracts every ```cpp block tagged
// <!-- snippet: NAME --> into snip_NAME.inc and compiles this file with -fsyntax-only).  Each
// function below declares the names a snippet takes from its surroundings in the reference
// (src/cluster_client.cpp:1185, :1857-1860, src/session_manager.cpp:1118-1144), then includes the
// snippet's text unchanged.
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdint>
#include <string>
#include <vector>

#include "aeron_cluster_amd.hpp"
#include "sbecodec.h"

namespace ctx {
struct Client {  // ClusterClient::offer_ingress (include/aeron_cluster/cluster_client.hpp:409)
    bool offer_ingress(const std::uint8_t*, std::size_t) { return true; }
};
struct Publication {  // aeron::ExclusivePublication::offer (returns the new position, < 0 on refusal)
    std::int64_t offer(const std::uint8_t*, std::size_t) { return 1; }
};
struct PendingOrder {  // whatever the caller holds per order: id, JSON payload, headers JSON
    std::string id, json, headers;
};
}  // namespace ctx

std::vector<aeron_cluster::Order> load_orders() { return {}; }

void snippet_encode_batch() {
    ctx::Client client;
    std::vector<ctx::PendingOrder> orders;
#include "snip_encode_batch.inc"
}

void snippet_publish_topic() {
    ctx::Client client;
    std::string json;
    std::vector<aeron_cluster::TopicMessageFields> msgs;
#include "snip_publish_topic.inc"
}

void snippet_session_frames() {
    std::int64_t leadership_term_id = 0, cluster_session_id = 0;
    std::vector<aeron_cluster::TopicMessageFields> msgs;
    ctx::Publication pub_obj;
    ctx::Publication* publication = &pub_obj;
#include "snip_session_frames.inc"
}

void snippet_orders_json() {
#include "snip_orders_json.inc"
}

void snippet_parse_batch() {
    auto message_callback_ = [](const aeron_cluster::ParseResult&) {};
#include "snip_parse_batch.inc"
}

void snippet_batching_parser() {
    auto message_callback_ = [](const aeron_cluster::ParseResult&) {};
#include "snip_batching_parser.inc"
}

void snippet_materialize() {
    std::uint64_t n = 0, arena_capacity = 0;
    const std::uint8_t* d_in = nullptr;
    const std::uint64_t* d_rec_off = nullptr;
    sbe_decoded dec{};
    std::uint8_t* d_arena = nullptr;
    std::uint64_t* d_arena_off = nullptr;
    void* d_ws = nullptr;
    hipStream_t stream = nullptr;
#include "snip_materialize.inc"
    (void)rc;
}

void snippet_gather() {
    int rank = 0, world = 1;
    sbe_tm_batch shard{};
    std::uint64_t m = 0, now_ms = 0, cap = 0, dst_cap = 0, dst_off_cap = 0;
    std::uint8_t *out = nullptr, *status = nullptr, *dst = nullptr;
    std::uint64_t *out_off = nullptr, *dst_off = nullptr;
    void* ws = nullptr;
    std::size_t ws_bytes = 0;
    hipStream_t stream = nullptr;
#include "snip_gather.inc"
}

void snippet_serve() {
    std::uint8_t *d_arena = nullptr, *d_out = nullptr, *d_status = nullptr, *d_rec = nullptr;
    std::uint32_t* d_len = nullptr;
    std::uint64_t *d_ts = nullptr, *d_off = nullptr, *d_rec_off = nullptr;
    std::uint64_t now_ns = 0, cap = 0;
    sbe_decoded dd{};
#include "snip_serve.inc"
}
