// aeron_cluster_amd.cpp — host side of the reference codec surface over the C ABI.
// Host memory in, host memory out (the reference's API contract): each call stages its batch in
// pinned buffers, copies it to HBM on a private stream, launches the HIP kernels through
// include/sbecodec.h and copies the results back.  Results are materialised on the host from the
// device descriptors (views into the caller's own bytes), never recomputed here.
#include "aeron_cluster_amd.hpp"

#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>
#include <cstring>
#include <iostream>
#include <mutex>
#include <stdexcept>

#include "sbecodec.h"

namespace aeron_cluster {
namespace {

[[noreturn]] void fail(const char* what) {
    throw std::runtime_error(std::string("sbecodec: ") + what + " (" + sbe_last_error() + ")");
}

void hip_check(hipError_t e, const char* what) {
    if (e != hipSuccess) throw std::runtime_error(std::string("sbecodec: ") + what + ": " + hipGetErrorString(e));
}

// Growable device / pinned host buffer.
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
    ~DevBuf() {
        if (p) (void)hipFree(p);
    }
};
struct HostBuf {
    void* p = nullptr;
    size_t cap = 0;
    void need(size_t n) {
        if (n <= cap) return;
        if (p) (void)hipHostFree(p);
        p = nullptr;
        cap = 0;
        const size_t c = n < 4096 ? 4096 : n + n / 4;
        hip_check(hipHostMalloc(&p, c, hipHostMallocDefault), "hipHostMalloc");
        cap = c;
    }
    ~HostBuf() {
        if (p) (void)hipHostFree(p);
    }
};

// Per-thread device context (the reference's codec functions are reentrant statics).
struct Ctx {
    hipStream_t stream = nullptr;
    DevBuf d_arena, d_len, d_ts, d_out, d_off, d_st, d_ws, d_in, d_roff, d_dec;
    HostBuf h_arena, h_len, h_ts, h_out, h_off, h_st, h_in, h_roff, h_dec;
    Ctx() {
        if (sbe_device_ready() != 1) fail("no gfx950 device visible");
        hip_check(hipStreamCreateWithFlags(&stream, hipStreamNonBlocking), "hipStreamCreate");
    }
    ~Ctx() {
        if (stream) (void)hipStreamDestroy(stream);
    }
};

Ctx& ctx() {
    thread_local Ctx c;
    return c;
}

inline int64_t rdi64(const uint8_t* p) {
    uint64_t v = 0;
    for (int i = 7; i >= 0; --i) v = (v << 8) | p[i];
    return (int64_t)v;
}
inline int32_t rdi32(const uint8_t* p) { return (int32_t)((uint32_t)p[0] | (p[1] << 8) | (p[2] << 16) | ((uint32_t)p[3] << 24)); }

// device descriptors of n records, in one allocation
struct Desc {
    std::vector<uint8_t> status, flags;
    std::vector<uint16_t> hdr;
    std::vector<uint64_t> ts;
    std::vector<uint32_t> off, len;
    std::vector<uint64_t> seq;  // parse mode: ParseResult.sequence_number (sbe_eval_sequence_numbers)
};

Desc run_decode(const uint8_t* data, const uint64_t* rec_off, size_t n, uint32_t mode) {
    Ctx& c = ctx();
    Desc d;
    if (n == 0) return d;
    const uint64_t base = rec_off[0], total = rec_off[n] - base;
    // records rebased to 0 so the device stream starts 16-B aligned
    c.h_in.need(total + 16);
    std::memcpy(c.h_in.p, data + base, total);
    c.h_roff.need((n + 1) * 8);
    uint64_t* ro = static_cast<uint64_t*>(c.h_roff.p);
    for (size_t i = 0; i <= n; ++i) ro[i] = rec_off[i] - base;
    c.d_in.need(total + 16);
    c.d_roff.need((n + 1) * 8);
    // descriptor SoA: status n, flags n, hdr 8n, ts 8n, off 20n, len 20n, seq 8n (each 16-B aligned)
    auto al = [](size_t x) { return (x + 15) & ~(size_t)15; };
    const bool parse = mode == SBE_DEC_PARSE_MESSAGE;
    const size_t o_st = 0, o_fl = al(n), o_hdr = o_fl + al(n), o_ts = o_hdr + al(8 * n), o_off = o_ts + al(8 * n),
                 o_len = o_off + al(20 * n), o_seq = o_len + al(20 * n), dbytes = o_seq + (parse ? al(8 * n) : 0);
    c.d_dec.need(dbytes);
    c.h_dec.need(dbytes);
    hip_check(hipMemcpyAsync(c.d_in.p, c.h_in.p, total, hipMemcpyHostToDevice, c.stream), "H2D");
    hip_check(hipMemcpyAsync(c.d_roff.p, c.h_roff.p, (n + 1) * 8, hipMemcpyHostToDevice, c.stream), "H2D");
    uint8_t* db = static_cast<uint8_t*>(c.d_dec.p);
    sbe_decoded out{db + o_st, db + o_fl, reinterpret_cast<uint16_t*>(db + o_hdr), reinterpret_cast<uint64_t*>(db + o_ts),
                    reinterpret_cast<uint32_t*>(db + o_off), reinterpret_cast<uint32_t*>(db + o_len), nullptr};
    if (parse) {  // sequence_number of the flagged TopicMessages, in the decode launch; 0 elsewhere
        out.seq = reinterpret_cast<uint64_t*>(db + o_seq);
        hip_check(hipMemsetAsync(out.seq, 0, 8 * n, c.stream), "memset");
    }
    if (sbe_decode_batch(static_cast<uint8_t*>(c.d_in.p), static_cast<uint64_t*>(c.d_roff.p), n, mode, &out, c.stream) != SBE_OK)
        fail("sbe_decode_batch");
    hip_check(hipMemcpyAsync(c.h_dec.p, c.d_dec.p, dbytes, hipMemcpyDeviceToHost, c.stream), "D2H");
    hip_check(hipStreamSynchronize(c.stream), "sync");
    const uint8_t* hb = static_cast<const uint8_t*>(c.h_dec.p);
    d.status.assign(hb + o_st, hb + o_st + n);
    d.flags.assign(hb + o_fl, hb + o_fl + n);
    d.hdr.assign(reinterpret_cast<const uint16_t*>(hb + o_hdr), reinterpret_cast<const uint16_t*>(hb + o_hdr) + 4 * n);
    d.ts.assign(reinterpret_cast<const uint64_t*>(hb + o_ts), reinterpret_cast<const uint64_t*>(hb + o_ts) + n);
    d.off.assign(reinterpret_cast<const uint32_t*>(hb + o_off), reinterpret_cast<const uint32_t*>(hb + o_off) + 5 * n);
    d.len.assign(reinterpret_cast<const uint32_t*>(hb + o_len), reinterpret_cast<const uint32_t*>(hb + o_len) + 5 * n);
    if (parse)
        d.seq.assign(reinterpret_cast<const uint64_t*>(hb + o_seq), reinterpret_cast<const uint64_t*>(hb + o_seq) + n);
    return d;
}

ParseResult materialize(const uint8_t* rec, const Desc& d, size_t i) {
    ParseResult r;
    const uint8_t st = d.status[i], fl = d.flags[i];
    const uint16_t* h = &d.hdr[4 * i];
    auto view = [&](int k) {
        return std::string(reinterpret_cast<const char*>(rec) + d.off[5 * i + k], d.len[5 * i + k]);
    };
    auto take_hdr = [&] {
        r.block_length = h[0];
        r.template_id = h[1];
        r.schema_id = h[2];
        r.version = h[3];
    };
    const uint32_t param = d.off[5 * i];
    switch (st) {
        case SBE_ST_TM:  // src/sbe_encoder.cpp:1021-1135
            r.success = true;
            r.message_type = view(1);
            r.message_id = view(2);
            r.payload = view(3);
            r.headers = view(4);
            r.timestamp = (int64_t)d.ts[i];
            r.sequence_key_present = (fl & SBE_FL_SEQ_KEY) != 0;
            r.sequence_number = d.seq.empty() ? 0 : d.seq[i];  // src/sbe_encoder.cpp:1031-1125
            take_hdr();
            break;
        case SBE_ST_ACK:  // src/sbe_encoder.cpp:916-941
            r.success = true;
            r.message_type = "Acknowledgment";
            r.timestamp = (int64_t)d.ts[i];
            r.message_id = (fl & SBE_FL_ID_DEFAULT) ? "ack_" + std::to_string(d.ts[i]) : view(0);
            r.payload = (fl & SBE_FL_PAYLOAD_DEFAULT) ? std::string("SUCCESS") : view(1);
            r.headers = view(2);
            take_hdr();
            break;
        case SBE_ST_SESSION_EVENT:  // src/sbe_encoder.cpp:629-644 (SessionEvent layout sbe_messages.hpp:39-50)
            r.success = true;
            r.message_type = "SessionEvent";
            r.correlation_id = rdi64(rec + 8);
            r.session_id = rdi64(rec + 16);
            r.leadership_term_id = rdi64(rec + 24);
            r.leader_member_id = rdi32(rec + 32);
            r.event_code = rdi32(rec + 36);
            r.payload = view(3);
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
    return r;
}

const char* kE109[5] = {"topicLength too long for length type [E109]", "messageTypeLength too long for length type [E109]",
                        "uuidLength too long for length type [E109]", "payloadLength too long for length type [E109]",
                        "headersLength too long for length type [E109]"};

}  // namespace

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

bool gpu_codec_available() { return sbe_device_ready() == 1; }

namespace {
// Stage a batch of records (nf strings, a u64 and a u32 each) in pinned memory, copy it to HBM,
// run `launch` (one sbe_encode_*_batch call) and copy the encoded stream back.
template <class Launch>
EncodedBatch run_encode(size_t n, int nf, const std::function<std::string_view(size_t, int)>& field,
                        const std::function<uint64_t(size_t)>& u64, const std::function<uint32_t(size_t)>& u32,
                        uint64_t bound_per_record, Launch launch) {
    Ctx& c = ctx();
    EncodedBatch b;
    b.offsets.assign(n + 1, 0);
    b.status.assign(n, 0);
    if (n == 0) return b;
    size_t arena = 0;
    for (size_t i = 0; i < n; ++i)
        for (int k = 0; k < nf; ++k) arena += field(i, k).size();
    c.h_arena.need(arena + 16);
    c.h_len.need(n * 4 * nf);
    c.h_ts.need(n * 12);
    uint8_t* ap = static_cast<uint8_t*>(c.h_arena.p);
    uint32_t* lp = static_cast<uint32_t*>(c.h_len.p);
    uint64_t* tp = static_cast<uint64_t*>(c.h_ts.p);
    uint32_t* ip = reinterpret_cast<uint32_t*>(tp + n);
    size_t at = 0;
    for (size_t i = 0; i < n; ++i) {
        for (int k = 0; k < nf; ++k) {
            const std::string_view f = field(i, k);
            std::memcpy(ap + at, f.data(), f.size());
            at += f.size();
            lp[(size_t)nf * i + k] = (uint32_t)f.size();
        }
        tp[i] = u64(i);
        ip[i] = u32(i);
    }
    const uint64_t cap = arena + bound_per_record * n + 16;
    c.d_arena.need(arena + 16);
    c.d_len.need(n * 4 * nf);
    c.d_ts.need(n * 12);
    c.d_out.need(cap);
    c.d_off.need((n + 1) * 8);
    c.d_st.need(n);
    c.d_ws.need(sbe_encode_workspace_size(n));
    hip_check(hipMemcpyAsync(c.d_arena.p, ap, arena, hipMemcpyHostToDevice, c.stream), "H2D");
    hip_check(hipMemcpyAsync(c.d_len.p, lp, n * 4 * nf, hipMemcpyHostToDevice, c.stream), "H2D");
    hip_check(hipMemcpyAsync(c.d_ts.p, tp, n * 12, hipMemcpyHostToDevice, c.stream), "H2D");
    const uint64_t* d_u64 = static_cast<const uint64_t*>(c.d_ts.p);
    launch(static_cast<const uint8_t*>(c.d_arena.p), static_cast<const uint32_t*>(c.d_len.p), d_u64,
           reinterpret_cast<const uint32_t*>(d_u64 + n), static_cast<uint8_t*>(c.d_out.p), cap,
           static_cast<uint64_t*>(c.d_off.p), static_cast<uint8_t*>(c.d_st.p), c.d_ws.p, c.d_ws.cap, c.stream);
    hip_check(hipMemcpyAsync(b.offsets.data(), c.d_off.p, (n + 1) * 8, hipMemcpyDeviceToHost, c.stream), "D2H");
    hip_check(hipMemcpyAsync(b.status.data(), c.d_st.p, n, hipMemcpyDeviceToHost, c.stream), "D2H");
    hip_check(hipStreamSynchronize(c.stream), "sync");
    b.bytes.resize(b.offsets[n]);
    if (b.offsets[n]) {
        hip_check(hipMemcpyAsync(b.bytes.data(), c.d_out.p, b.offsets[n], hipMemcpyDeviceToHost, c.stream), "D2H");
        hip_check(hipStreamSynchronize(c.stream), "sync");
    }
    return b;
}

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

EncodedBatch encode_tm(const std::vector<TopicMessageFields>& msgs, EncodeLength length, bool session, int64_t term,
                       int64_t sess, uint64_t ts_default) {
    const uint32_t flags = length == EncodeLength::Reference ? SBE_ENC_REF_TRUNCATE8
                         : length == EncodeLength::Publish   ? SBE_ENC_PUBLISH_TOPIC
                                                             : 0u;
    return run_encode(
        msgs.size(), 5, [&](size_t i, int k) { return tm_field(msgs[i], k); },
        [&](size_t i) { return (uint64_t)msgs[i].timestamp; }, [](size_t) { return 0u; },
        SBE_TM_WIRE_OVERHEAD + SBE_SESSION_HDR_LEN,
        [&](const uint8_t* arena, const uint32_t* len, const uint64_t* ts, const uint32_t*, uint8_t* out, uint64_t cap,
            uint64_t* off, uint8_t* st, void* ws, size_t wsb, hipStream_t s) {
            sbe_tm_batch in{arena, nullptr, len, ts};
            const int rc = session ? sbe_encode_session_batch(&in, msgs.size(), ts_default, flags, term, sess, out, cap,
                                                              off, st, ws, wsb, s)
                                   : sbe_encode_topic_batch(&in, msgs.size(), ts_default, flags, out, cap, off, st, ws,
                                                            wsb, s);
            if (rc != SBE_OK) fail(session ? "sbe_encode_session_batch" : "sbe_encode_topic_batch");
        });
}
}  // namespace

EncodedBatch SBEEncoder::encode_topic_batch(const std::vector<TopicMessageFields>& msgs, EncodeLength length) {
    // timestamp 0 → the clock the reference reads (src/sbe_encoder.cpp:134-138)
    return encode_tm(msgs, length, false, 0, 0, clock_ms());
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
    return b.bytes;
}

static uint64_t now_nanos_sys() {  // include/aeron_cluster/protocol.hpp:31-34
    return (uint64_t)std::chrono::duration_cast<std::chrono::nanoseconds>(
               std::chrono::system_clock::now().time_since_epoch())
        .count();
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
    return run_encode(
        offsets.size(), 2,
        [&](size_t i, int k) { return std::string_view(k == 0 ? offsets[i].message_id : offsets[i].message_identifier); },
        [&](size_t i) { return offsets[i].sequence_number; }, [&](size_t i) { return ids[i]; },
        SBE_LITE_OVERHEAD(2),
        [&](const uint8_t* arena, const uint32_t* len, const uint64_t* seq, const uint32_t* tid, uint8_t* out,
            uint64_t cap, uint64_t* off, uint8_t* st, void* ws, size_t wsb, hipStream_t s) {
            sbe_lite_batch in{arena, nullptr, len, tid, seq};
            if (sbe_encode_lite_batch(&in, offsets.size(), SBE_COMMIT_OFFSET_LITE_TEMPLATE_ID, out, cap, off, st, ws,
                                      wsb, s) != SBE_OK)
                fail("sbe_encode_lite_batch");
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
    return b.bytes;
}

OrderJsonBatch orders_to_json(const std::vector<Order>& orders, const std::vector<std::string>& message_ids) {
    const size_t n = orders.size();
    if (message_ids.size() != n) throw std::invalid_argument("orders_to_json: one message id per order");
    OrderJsonBatch r;
    for (EncodedBatch* b : {&r.payload, &r.headers}) {
        b->offsets.assign(n + 1, 0);
        b->status.assign(n, 0);
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
    size_t arena = 0;
    for (size_t i = 0; i < n; ++i)
        for (int k = 0; k < (int)SBE_ORDER_FIELDS; ++k) arena += field(i, k).size();
    const size_t nlen = n * 4 * SBE_ORDER_FIELDS, nnum = n * 24;
    c.h_arena.need(arena + 16);
    c.h_len.need(nlen + nnum);
    uint8_t* ap = static_cast<uint8_t*>(c.h_arena.p);
    uint32_t* lp = static_cast<uint32_t*>(c.h_len.p);
    int64_t* cid = reinterpret_cast<int64_t*>(static_cast<uint8_t*>(c.h_len.p) + ((nlen + 7) & ~(size_t)7));
    int64_t* ts = cid + n;
    double* q = reinterpret_cast<double*>(ts + n);
    size_t at = 0;
    for (size_t i = 0; i < n; ++i) {
        for (int k = 0; k < (int)SBE_ORDER_FIELDS; ++k) {
            const std::string_view f = field(i, k);
            std::memcpy(ap + at, f.data(), f.size());
            at += f.size();
            lp[SBE_ORDER_FIELDS * i + k] = (uint32_t)f.size();
        }
        cid[i] = orders[i].customer_id;
        ts[i] = orders[i].timestamp;
        q[i] = orders[i].quantity;
    }
    const size_t small = ((nlen + 7) & ~(size_t)7) + nnum;
    // a record is at most ~800 B besides its strings (428 fixed, 316 for "%f" of a quantity near
    // DBL_MAX, 24 for "%.17g", 34 for two integers); strings escape to <= 6x and appear <= twice.
    // out_off always holds the full sizes, so a record past the capacity is redone below.
    uint64_t cap = 12 * (uint64_t)arena + 900 * (uint64_t)n + 16;
    c.d_arena.need(arena + 16);
    c.d_len.need(small);
    c.d_off.need(2 * (n + 1) * 8);
    c.d_st.need(2 * n);
    c.d_ws.need(sbe_order_json_workspace_size(n));
    hip_check(hipMemcpyAsync(c.d_arena.p, ap, arena, hipMemcpyHostToDevice, c.stream), "H2D");
    hip_check(hipMemcpyAsync(c.d_len.p, c.h_len.p, small, hipMemcpyHostToDevice, c.stream), "H2D");
    const uint8_t* dl = static_cast<const uint8_t*>(c.d_len.p);
    const int64_t* d_cid = reinterpret_cast<const int64_t*>(dl + ((nlen + 7) & ~(size_t)7));
    sbe_order_batch in{static_cast<const uint8_t*>(c.d_arena.p), nullptr, reinterpret_cast<const uint32_t*>(dl),
                       d_cid, d_cid + n, reinterpret_cast<const double*>(d_cid + 2 * n)};
    for (int w = 0; w < 2; ++w) {
        EncodedBatch& b = w ? r.headers : r.payload;
        uint64_t* off = static_cast<uint64_t*>(c.d_off.p) + w * (n + 1);
        uint8_t* st = static_cast<uint8_t*>(c.d_st.p) + w * n;
        for (int attempt = 0;; ++attempt) {
            c.d_out.need(2 * cap);
            uint8_t* out = static_cast<uint8_t*>(c.d_out.p) + w * cap;
            if (sbe_order_to_json_batch(&in, n, w ? SBE_JSON_PUBLISH_HEADERS : SBE_JSON_ORDER_PAYLOAD, out, cap, off,
                                        st, c.d_ws.p, c.d_ws.cap, c.stream) != SBE_OK)
                fail("sbe_order_to_json_batch");
            hip_check(hipMemcpyAsync(b.offsets.data(), off, (n + 1) * 8, hipMemcpyDeviceToHost, c.stream), "D2H");
            hip_check(hipMemcpyAsync(b.status.data(), st, n, hipMemcpyDeviceToHost, c.stream), "D2H");
            hip_check(hipStreamSynchronize(c.stream), "sync");
            if (b.offsets[n] <= cap || attempt > 0) break;
            cap = b.offsets[n];  // the measured size: one rerun
        }
        for (size_t i = 0; i < n; ++i)
            if (b.status[i] != SBE_JSON_OK) throw std::runtime_error("sbecodec: order JSON record did not fit");
        uint8_t* out = static_cast<uint8_t*>(c.d_out.p) + w * cap;
        b.bytes.resize(b.offsets[n]);
        if (b.offsets[n]) {
            hip_check(hipMemcpyAsync(b.bytes.data(), out, b.offsets[n], hipMemcpyDeviceToHost, c.stream), "D2H");
            hip_check(hipStreamSynchronize(c.stream), "sync");
        }
    }
    return r;
}

std::string Order::to_json() const {
    OrderJsonBatch b = orders_to_json({*this}, {std::string()});
    return std::string(b.payload.bytes.begin(), b.payload.bytes.end());
}

std::vector<std::uint8_t> SBEEncoder::encode_topic_message(const std::string& topic, const std::string& message_type,
                                                           const std::string& uuid, const std::string& payload,
                                                           const std::string& headers, std::int64_t timestamp) {
    TopicMessageFields f{topic, message_type, uuid, payload, headers, timestamp};
    EncodedBatch b = encode_topic_batch({f}, EncodeLength::Reference);
    const uint8_t st = b.status[0];
    if (st >= SBE_ENC_E109_TOPIC && st <= SBE_ENC_E109_HEADERS) throw std::runtime_error(kE109[st - 1]);
    if (st != SBE_ENC_OK) throw std::runtime_error("sbecodec: encode failed");
    return b.bytes;
}

ParseResult MessageParser::parse_message(const std::uint8_t* data, std::size_t length) {
    if (!data || length == 0) {  // src/sbe_encoder.cpp:516-519 (no device round trip needed)
        ParseResult r;
        r.error_message = "Null or empty data";
        return r;
    }
    const uint64_t off[2] = {0, length};
    Desc d = run_decode(data, off, 1, SBE_DEC_PARSE_MESSAGE);
    return materialize(data, d, 0);
}

std::vector<ParseResult> MessageParser::parse_batch(const std::uint8_t* data, const std::uint64_t* rec_off, std::size_t n) {
    Desc d = run_decode(data, rec_off, n, SBE_DEC_PARSE_MESSAGE);
    std::vector<ParseResult> out;
    out.reserve(n);
    for (size_t i = 0; i < n; ++i) out.push_back(materialize(data + rec_off[i], d, i));
    return out;
}

namespace {
std::optional<AckInfo> ack_from(const uint8_t* rec, const Desc& d, size_t i) {
    const uint8_t st = d.status[i];
    if (st != SBE_ST_EG_ACK_SIMPLE && st != SBE_ST_EG_ACK) return std::nullopt;
    AckInfo a;
    a.timestamp_nanos = d.ts[i];
    a.simple_control_ack = st == SBE_ST_EG_ACK_SIMPLE;
    if (st == SBE_ST_EG_ACK) {
        auto v = [&](int k) { return std::string(reinterpret_cast<const char*>(rec) + d.off[5 * i + k], d.len[5 * i + k]); };
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
    Desc d = run_decode(data, off, 1, SBE_DEC_ON_EGRESS);
    return ack_from(data, d, 0);
}

std::optional<LiteRecord> decode_lite(const std::uint8_t* data, std::size_t len) {
    if (!data || len < 8) return std::nullopt;
    const uint64_t off[2] = {0, len};
    Desc d = run_decode(data, off, 1, SBE_DEC_LITE);
    if (d.status[0] != SBE_ST_LITE) return std::nullopt;
    LiteRecord r;
    r.template_id = d.hdr[1];
    r.topic_id = d.off[4];
    r.sequence = d.ts[0];
    const int nf = (int)sbe_lite_fields(r.template_id);
    for (int k = 0; k < nf; ++k) r.fields.emplace_back(reinterpret_cast<const char*>(data) + d.off[k], d.len[k]);
    return r;
}

EncodedBatch FragmentReassembler::on_fragments(const std::uint8_t* data, const std::uint64_t* frag_off,
                                               const std::uint8_t* flags, std::size_t n) {
    Ctx& c = ctx();
    EncodedBatch b;
    // the accumulator so far goes first as a middle fragment (flags 0): it is appended to exactly
    // as the reference's acc_ would be, or cleared by a BEGIN
    const size_t pre = acc_.empty() ? 0 : 1, nf = n + pre;
    if (nf == 0) {
        b.offsets.assign(1, 0);
        return b;
    }
    const uint64_t base = n ? frag_off[0] : 0, body = n ? frag_off[n] - base : 0, total = acc_.size() + body;
    c.h_in.need(total + 16);
    uint8_t* hi = static_cast<uint8_t*>(c.h_in.p);
    std::memcpy(hi, acc_.data(), acc_.size());
    if (body) std::memcpy(hi + acc_.size(), data + base, body);
    c.h_roff.need((nf + 1) * 8 + nf);
    uint64_t* ho = static_cast<uint64_t*>(c.h_roff.p);
    uint8_t* hf = reinterpret_cast<uint8_t*>(ho + nf + 1);
    ho[0] = 0;
    if (pre) {
        ho[1] = acc_.size();
        hf[0] = 0;
    }
    for (size_t i = 0; i < n; ++i) {
        ho[pre + i + 1] = acc_.size() + (frag_off[i + 1] - base);
        hf[pre + i] = flags[i];
    }
    c.d_in.need(total + 16);
    c.d_roff.need((nf + 1) * 8 + nf);
    c.d_out.need(total + 16);
    c.d_off.need((nf + 1) * 8 + 16);
    const size_t wsb = sbe_reassemble_workspace_size(nf);
    c.d_ws.need(wsb);
    hip_check(hipMemcpyAsync(c.d_in.p, hi, total, hipMemcpyHostToDevice, c.stream), "H2D");
    hip_check(hipMemcpyAsync(c.d_roff.p, ho, (nf + 1) * 8 + nf, hipMemcpyHostToDevice, c.stream), "H2D");
    uint64_t* d_off = static_cast<uint64_t*>(c.d_off.p);
    uint64_t* d_counts = d_off + nf + 1;
    if (sbe_reassemble_fragments(static_cast<uint8_t*>(c.d_in.p), static_cast<uint64_t*>(c.d_roff.p),
                                 reinterpret_cast<uint8_t*>(static_cast<uint64_t*>(c.d_roff.p) + nf + 1), nf,
                                 static_cast<uint8_t*>(c.d_out.p), d_off, d_counts, c.d_ws.p, c.d_ws.cap,
                                 c.stream) != SBE_OK)
        fail("sbe_reassemble_fragments");
    uint64_t counts[2];
    hip_check(hipMemcpyAsync(counts, d_counts, 16, hipMemcpyDeviceToHost, c.stream), "D2H");
    hip_check(hipStreamSynchronize(c.stream), "sync");
    const uint64_t m = counts[0];
    b.offsets.resize(m + 1);
    b.status.assign(m, 0);
    hip_check(hipMemcpyAsync(b.offsets.data(), d_off, (m + 1) * 8, hipMemcpyDeviceToHost, c.stream), "D2H");
    hip_check(hipStreamSynchronize(c.stream), "sync");
    const uint64_t out_bytes = b.offsets[m] + counts[1];
    std::vector<uint8_t> all(out_bytes);
    if (out_bytes) {
        hip_check(hipMemcpyAsync(all.data(), c.d_out.p, out_bytes, hipMemcpyDeviceToHost, c.stream), "D2H");
        hip_check(hipStreamSynchronize(c.stream), "sync");
    }
    acc_.assign(all.begin() + b.offsets[m], all.end());
    all.resize(b.offsets[m]);
    b.bytes = std::move(all);
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
    Desc d = run_decode(data, rec_off, n, SBE_DEC_ON_EGRESS);
    for (size_t i = 0; i < n; ++i) {
        const uint8_t* rec = data + rec_off[i];
        switch (d.status[i]) {
            case SBE_ST_EG_ACK_SIMPLE:
            case SBE_ST_EG_ACK:
                if (ack_cb_) ack_cb_(*ack_from(rec, d, i));
                break;
            case SBE_ST_EG_TM:
                if (tm_cb_) {
                    auto v = [&](int k) {
                        return std::string_view(reinterpret_cast<const char*>(rec) + d.off[5 * i + k], d.len[5 * i + k]);
                    };
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
