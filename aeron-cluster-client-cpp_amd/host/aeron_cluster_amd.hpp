// aeron_cluster_amd.hpp — C++17 host mirror of the reference's codec surface, backed by the
// MI355X kernels behind include/sbecodec.h.
//
// Same names, argument meaning and error behaviour as the reference (paths relative to it):
//   SBEEncoder::encode_topic_message   include/aeron_cluster/sbe_messages.hpp:158-164,
//                                      src/sbe_encoder.cpp:131-167 (E109 → std::runtime_error)
//   MessageParser::parse_message       include/aeron_cluster/sbe_messages.hpp:422, src/sbe_encoder.cpp:513-551
//   ParseResult                        include/aeron_cluster/sbe_messages.hpp:306-412
//   decode_ack / AckInfo               include/aeron_cluster/ack_decoder.hpp:9-19, src/ack_decoder.cpp:29-105
//   MessageHandler::on_egress          include/aeron_cluster/message_handler.hpp:35-89 (E100 escapes
//                                      as std::runtime_error("buffer too short [E100]"))
//   SessionManager frame               create_topic_message + send_combined_message,
//                                      src/session_manager.cpp:936-967, :1018-1046, :1050-1144
//   CommitManager                      build_commit_offset_message (CommitOffsetLite),
//                                      src/commit_manager.cpp:16-22, :107-132; CommitOffset
//                                      include/aeron_cluster/commit_manager.hpp:17-24
//   LocalFragmentReassembler           src/cluster_client.cpp:39-82 (FragmentReassembler below)
//   ClusterClient::offer_ingress       include/aeron_cluster/cluster_client.hpp:409 — the sink the
//                                      encoded records are handed to (OfferFn below)
// plus batched overloads, which are the point of the GPU path: one launch per batch.
//
// Everything computes on the GPU.  There is no CPU codec here: without a gfx950 device every
// codec entry point throws std::runtime_error("sbecodec: ...") (SBEUtils, SBEDecoder and the
// header-only MessageParser helpers are host struct readers, as in the reference).  Host work is
// staging and result building only, on min(16, cores) host threads (AERON_AMD_HOST_THREADS):
//  - a batch of at most 65536 records and 8-32 MiB (AERON_AMD_CHUNK_BYTES) is one chunk; up to
//    4 MiB staged (AERON_AMD_ZC_BYTES) it takes the zero-copy path: the kernels read the
//    page-locked staging buffer and write the results straight into the page-locked result
//    block over PCIe, one launch (encode: two) and one wait, no copy step;
//  - larger batches are cut into chunks that flow through three HIP streams (copy-in, kernels,
//    copy-out) three slots deep, so chunk k+1's H2D, chunk k's kernels and chunk k-1's D2H
//    overlap while the host threads stage the next chunk.
#pragma once

#include <cstdint>
#include <chrono>
#include <functional>
#include <memory>
#include <optional>
#include <string>
#include <string_view>
#include <vector>

namespace aeron_cluster {

// include/aeron_cluster/config.hpp:169-199
namespace SBEConstants {
constexpr std::uint16_t CLUSTER_SCHEMA_ID = 111;
constexpr std::uint16_t CLUSTER_SCHEMA_VERSION = 8;
constexpr std::uint16_t TOPIC_SCHEMA_ID = 1;
constexpr std::uint16_t TOPIC_SCHEMA_VERSION = 1;
constexpr std::uint16_t SESSION_CONNECT_TEMPLATE_ID = 3;
constexpr std::uint16_t SESSION_EVENT_TEMPLATE_ID = 2;
constexpr std::uint16_t SESSION_CLOSE_TEMPLATE_ID = 4;
constexpr std::uint16_t SESSION_KEEPALIVE_TEMPLATE_ID = 5;
constexpr std::uint16_t TOPIC_MESSAGE_TEMPLATE_ID = 1;
constexpr std::uint16_t ACKNOWLEDGMENT_TEMPLATE_ID = 2;
constexpr std::uint16_t SESSION_CONNECT_BLOCK_LENGTH = 16;
constexpr std::uint16_t SESSION_EVENT_BLOCK_LENGTH = 32;
constexpr std::uint16_t TOPIC_MESSAGE_BLOCK_LENGTH = 48;
constexpr std::uint16_t ACKNOWLEDGMENT_BLOCK_LENGTH = 8;
constexpr std::int32_t SESSION_EVENT_OK = 0;
constexpr std::int32_t SESSION_EVENT_ERROR = 1;
constexpr std::int32_t SESSION_EVENT_REDIRECT = 2;
constexpr std::int32_t SESSION_EVENT_AUTHENTICATION_REJECTED = 3;
constexpr std::int32_t SESSION_EVENT_CLOSED = 4;
constexpr std::size_t SBE_HEADER_LENGTH = 8;
}  // namespace SBEConstants

// include/aeron_cluster/sbe_messages.hpp:14-20: the 8-byte SBE message header, packed
struct MessageHeader {
    std::uint16_t block_length;
    std::uint16_t template_id;
    std::uint16_t schema_id;
    std::uint16_t version;
} __attribute__((packed));
static_assert(sizeof(MessageHeader) == 8, "MessageHeader must be exactly 8 bytes");

// include/aeron_cluster/sbe_messages.hpp:39-54: SessionEvent's 32-byte fixed block (template 2,
// schema 111), packed
struct SessionEvent {
    std::int64_t correlation_id;
    std::int64_t cluster_session_id;
    std::int64_t leadership_term_id;
    std::int32_t leader_member_id;
    std::int32_t code;
    static constexpr std::uint16_t sbe_block_length() { return 32; }
    static constexpr std::uint16_t sbe_template_id() { return 2; }
    static constexpr std::uint16_t sbe_schema_id() { return 111; }
    static constexpr std::uint16_t sbe_schema_version() { return 8; }
} __attribute__((packed));
static_assert(sizeof(SessionEvent) == 32, "SessionEvent must be exactly 32 bytes");

// include/aeron_cluster/sbe_messages.hpp:189-247, bodies src/sbe_encoder.cpp:174-323: the
// reference's one-record struct readers.  Host code: each is a header / fixed-block copy plus at
// most three u32-length-prefixed strings, and none is on the batch decode path (parse_message
// reaches SessionEvent through the GPU decode, whose fields these return for the same record; the
// u32-prefixed Acknowledgment layout of decode_acknowledgment is unreachable from parse_message,
// whose is_topic_message() claims template 2 / schema 1 first, src/sbe_encoder.cpp:536-544).
// decode_topic_message is declared by the reference but never defined (no definition in src/), so
// it is not provided here either.
class SBEDecoder {
public:
    // :174-181: false for null data or fewer than 8 bytes, else the header bytes
    static bool decode_message_header(const std::uint8_t* data, std::size_t length, MessageHeader& header);
    // :183-238: false below 40 bytes or unless template 2 / schema 111; event = the 32-B block;
    // detail = the u32-prefixed string after it when one fits (<= 10 MiB; empty when its length is
    // 0; left as the caller had it when the prefix or the string does not fit)
    static bool decode_session_event(const std::uint8_t* data, std::size_t length, SessionEvent& event,
                                     std::string& detail);
    // :240-282: false below 16 bytes, unless template 2 / schema 1, or when message_id or status (u32
    // prefixes after the 8-B block) do not fit; error is read when bytes remain after status;
    // timestamp = the i64 after the header (written whenever the header checks pass)
    static bool decode_acknowledgment(const std::uint8_t* data, std::size_t length, std::string& message_id,
                                      std::string& status, std::string& error, std::int64_t& timestamp);
};

// The reference's debug helpers (include/aeron_cluster/sbe_messages.hpp:252-301, bodies
// src/sbe_encoder.cpp:328-485).  Host-side formatting only: ParseResult::get_description and the
// reference's tools (tools/message_inspector.cpp) call them; none of them is on the codec path.
namespace SBEUtils {
void print_hex_dump(const std::uint8_t* data, std::size_t length, const std::string& prefix = "",
                    std::size_t max_bytes = 0);
std::string get_session_event_code_string(std::int32_t code);           // :370-385
std::string get_message_type_name(std::uint16_t template_id, std::uint16_t schema_id);  // :387-409
bool is_valid_correlation_id(std::int64_t correlation_id);             // :411-413
std::int64_t generate_correlation_id();                                 // :415-419
std::string format_timestamp(std::int64_t timestamp);                   // :421-433
bool is_valid_sbe_message(const std::uint8_t* data, std::size_t length);  // :435-457
std::vector<std::string> extract_readable_strings(const std::uint8_t* data, std::size_t length,
                                                  std::size_t min_length = 3);  // :459-485
}  // namespace SBEUtils

// include/aeron_cluster/sbe_messages.hpp:306-328 (fields), :332-411 (predicates, description)
struct ParseResult {
    bool success = false;
    std::string error_message;
    std::string message_type;
    std::string message_id;
    std::string payload;
    std::string headers;
    std::int64_t timestamp = 0;
    std::uint64_t sequence_number = 0;
    std::uint16_t template_id = 0;
    std::uint16_t schema_id = 0;
    std::uint16_t version = 0;
    std::uint16_t block_length = 0;
    std::int64_t correlation_id = 0;
    std::int64_t session_id = 0;
    std::int32_t leader_member_id = 0;
    std::int32_t event_code = 0;
    std::int64_t leadership_term_id = 0;
    // sequence_number: "_sequence_number" of the payload JSON (src/sbe_encoder.cpp:1031-1125),
    // evaluated on the device with jsoncpp 1.9.5 semantics (sbe_eval_sequence_numbers; jsoncpp is
    // absent here, so parity with it is unpinned).  sequence_key_present: the payload holds the
    // literal key bytes (SBE_FL_SEQ_KEY).
    bool sequence_key_present = false;

    bool is_session_event() const {
        return template_id == SBEConstants::SESSION_EVENT_TEMPLATE_ID && schema_id == SBEConstants::CLUSTER_SCHEMA_ID;
    }
    bool is_topic_message() const;
    bool is_acknowledgment() const {
        return template_id == SBEConstants::ACKNOWLEDGMENT_TEMPLATE_ID && schema_id == SBEConstants::TOPIC_SCHEMA_ID;
    }
    // sbe_messages.hpp:382-406: a topic message whose type or payload names order content
    bool is_order_message() const;
    // src/sbe_encoder.cpp:490-510: "<type name>[ (code: …)| (type: …)][ [ID: <8 chars>...]]" or
    // "Parse Error: <error_message>"
    std::string get_description() const;
};

// include/aeron_cluster/ack_decoder.hpp:9-15
struct AckInfo {
    std::uint64_t timestamp_nanos{};
    std::string message_id;
    std::string topic;
    std::string correlation_id;
    bool simple_control_ack{false};
};

// One TopicMessage's fields, wire order (TopicMessage.h:515-1231).
struct TopicMessageFields {
    std::string_view topic, message_type, uuid, payload, headers;
    std::int64_t timestamp = 0;  // 0 → the encoder's clock, as the reference does
};

namespace detail {
struct HostBytesAccess;
struct Descriptors;
}  // namespace detail

// An array in page-locked host memory taken from a recycled pool: the device writes results
// straight into it (DMA, or the kernels themselves on the zero-copy path: no staging copy, no zero
// fill, no page faults on reuse), and the caller reads it in place.
// Aliasing: copying a HostArray (or an EncodedBatch) copies a reference, not the bytes: the copies
// share one block, and the arrays of one EncodedBatch (offsets, status, bytes) share one block.
// to_vector() makes an independent copy.  Retention: the block (a power of two of at least 4 KiB)
// stays page-locked while any copy lives, then returns to the pool, which keeps up to
// AERON_AMD_PINNED_CACHE_BYTES (default 4 GiB) of free blocks for reuse; a caller that holds many
// small results pins at least 4 KiB per result.
template <class T>
class HostArray {
public:
    const T* data() const { return p_; }
    T* data() { return p_; }
    std::size_t size() const { return n_; }
    bool empty() const { return n_ == 0; }
    const T* begin() const { return p_; }
    const T* end() const { return p_ + n_; }
    T* begin() { return p_; }
    T* end() { return p_ + n_; }
    const T& operator[](std::size_t i) const { return p_[i]; }
    T& operator[](std::size_t i) { return p_[i]; }
    const T& back() const { return p_[n_ - 1]; }
    std::vector<T> to_vector() const { return std::vector<T>(begin(), end()); }
    friend bool operator==(const HostArray& a, const std::vector<T>& v) {
        if (a.n_ != v.size()) return false;
        for (std::size_t i = 0; i < a.n_; ++i)
            if (!(a.p_[i] == v[i])) return false;
        return true;
    }

private:
    friend struct detail::HostBytesAccess;
    std::shared_ptr<void> block_;
    T* p_ = nullptr;
    std::size_t n_ = 0;
};
using HostBytes = HostArray<std::uint8_t>;

// A packed batch of encoded records: record i = bytes[offsets[i], offsets[i+1]).
struct EncodedBatch {
    HostBytes bytes;
    HostArray<std::uint64_t> offsets;
    HostArray<std::uint8_t> status;  // SBE_ENC_* per record
    std::string_view record(std::size_t i) const {
        return {reinterpret_cast<const char*>(bytes.data()) + offsets[i], static_cast<std::size_t>(offsets[i + 1] - offsets[i])};
    }
};

enum class EncodeLength {
    Reference,  // exactly what SBEEncoder::encode_topic_message returns (26+Σlen)
    Wire,       // the full wire record (34+Σlen), computeLength's E109 above 65534 B
    Publish     // ClusterClient::publish_topic's put*(const char*, int) calls (src/cluster_client.cpp:
                // 1850-1854): wire length, each length mod 65536 with that many bytes, no E109
};

class SBEEncoder {
public:
    // src/sbe_encoder.cpp:131-167: timestamp 0 → system_clock milliseconds; throws
    // std::runtime_error("<field>Length too long for length type [E109]") above 65534 bytes.
    static std::vector<std::uint8_t> encode_topic_message(const std::string& topic, const std::string& message_type,
                                                          const std::string& uuid, const std::string& payload,
                                                          const std::string& headers, std::int64_t timestamp = 0);
    // Batch encode: one GPU launch; records with E109 get status != 0 and zero bytes.
    static EncodedBatch encode_topic_batch(const std::vector<TopicMessageFields>& msgs,
                                           EncodeLength length = EncodeLength::Wire);
    // src/sbe_encoder.cpp:169-172: high_resolution_clock ticks since its epoch (nanoseconds)
    static std::int64_t get_current_timestamp();
};

class ParsedBatch;

class MessageParser {
public:
    // src/sbe_encoder.cpp:513-551 (never throws; success = false + error_message)
    static ParseResult parse_message(const std::uint8_t* data, std::size_t length);
    // src/sbe_encoder.cpp:957-1143 called directly (sbe_messages.hpp:423): no dispatch — a header
    // other than template 1 / schema 1 gives "Not a TopicMessage (got template_id=T, schema_id=S)",
    // fewer than 8 bytes the flyweight's E107 ("SBE TopicMessage decoding failed: buffer too short
    // for flyweight [E107]"); otherwise the GPU decode of the record.
    static ParseResult decode_topic_message_with_sbe(const std::uint8_t* data, std::size_t length);
    // src/sbe_encoder.cpp:833-954 called directly (sbe_messages.hpp:424): the printable-run
    // heuristic on any record whose header says template 2 / schema 1.
    static ParseResult decode_acknowledgment_with_sbe(const std::uint8_t* data, std::size_t length);
    // src/sbe_encoder.cpp:554-575: parse_message plus the reference's diagnostics (hex dump of
    // records of 1..200 bytes on stdout; DEBUG_LOG lines when AERON_CLUSTER_DEBUG=1).
    static ParseResult parse_message_debug(const std::uint8_t* data, std::size_t length,
                                           const std::string& debug_prefix = "");
    // src/sbe_encoder.cpp:577-586: "INVALID" below 8 bytes, else the header's type name
    static std::string get_message_type(const std::uint8_t* data, std::size_t length);
    // src/sbe_encoder.cpp:588-603: the i64 after the header of a schema-111 message, else 0
    static std::int64_t extract_correlation_id(const std::uint8_t* data, std::size_t length);
    // src/sbe_encoder.cpp:605-616
    static bool is_acknowledgment_for(const std::uint8_t* data, std::size_t length, const std::string& message_id);

    // Batch: records data[rec_off[i], rec_off[i+1]), ParseResults built on the host threads.
    static std::vector<ParseResult> parse_batch(const std::uint8_t* data, const std::uint64_t* rec_off, std::size_t n);
    // The same into the caller's vector (resized to n): each ParseResult is rewritten in place and
    // keeps its string buffers, so a caller that parses batch after batch into one vector does not
    // allocate once the strings have grown (out[i] == parse_message(record i) either way).
    static void parse_batch(const std::uint8_t* data, const std::uint64_t* rec_off, std::size_t n,
                            std::vector<ParseResult>& out);
    // Batch without materialising: the device descriptors and views into `data` (valid while the
    // caller's bytes are), ParseResults built on demand.  See ParsedBatch.
    static ParsedBatch decode_batch(const std::uint8_t* data, const std::uint64_t* rec_off, std::size_t n);
};

// parse_message's outcome for a batch, kept as the device descriptors (host copy) plus views into
// the caller's records.  result(i) == MessageParser::parse_message(record i); the string_view
// accessors give the same bytes without building the ParseResult.
class ParsedBatch {
public:
    std::size_t size() const { return n_; }
    ParseResult result(std::size_t i) const;
    ParseResult operator[](std::size_t i) const { return result(i); }
    // result(i) written into `out`, which keeps its string buffers (no allocation once they have grown)
    void result_into(std::size_t i, ParseResult& out) const;
    bool success(std::size_t i) const;
    std::uint8_t status(std::size_t i) const;  // SBE_ST_* of include/sbecodec.h
    std::uint16_t template_id(std::size_t i) const;
    std::uint16_t schema_id(std::size_t i) const;
    std::int64_t timestamp(std::size_t i) const;
    std::uint64_t sequence_number(std::size_t i) const;
    // TopicMessage: message_type / message_id (uuid) / payload / headers views; other statuses:
    // the views ParseResult would copy (Ack defaults and error texts are not views: use result(i)).
    std::string_view view(std::size_t i, int field) const;
    // Calls fn(i, result(i)) in record order on the calling thread; the ParseResults of each
    // 4096-record block are built on the host threads first.
    void for_each(const std::function<void(std::size_t, const ParseResult&)>& fn) const;

private:
    friend class MessageParser;
    std::shared_ptr<const detail::Descriptors> desc_;  // host copy of the device descriptors
    const std::uint8_t* data_ = nullptr;               // the caller's records (borrowed)
    const std::uint64_t* rec_off_ = nullptr;           // the caller's offsets (borrowed)
    std::size_t n_ = 0;
};

std::optional<AckInfo> decode_ack(const std::uint8_t* data, std::size_t len);

// MessageParser::parse_message at the reference's call granularity, batched across polls.  The
// reference parses one fragment per call from its poll handler (handle_incoming_message,
// src/cluster_client.cpp:1185) in polls of up to 100 fragments
// (include/aeron_cluster/performance_config.hpp:17); one GPU call per fragment costs a launch or
// a serve round trip, far more than the parse.  A BatchingParser takes the fragments of many
// polls: on_fragment copies each one (the fragment is only valid during the poll callback) into
// a page-locked batch; when the batch holds max_records records or max_bytes bytes, or at a poll()
// whose oldest pending record has waited max_delay, the batch goes to a decode thread
// (MessageParser::decode_batch) and filling continues in another batch (`batches` are kept; more
// are made when the caller hands off faster than it polls).  Handlers run on the caller's thread,
// in arrival order, only inside poll() / flush(), with handler(result) ==
// handler(MessageParser::parse_message(fragment)); on_fragment never runs a handler.  Waits spin
// for `spin` before they block.  A handler that throws propagates out of poll() / flush(); the
// records after it are delivered by the next call, none twice.  Call poll() after every poll of
// the subscription (the reference's loop), or flush().
// Added latency per record: at most max_delay + one batch decode after the poll that follows it
// (a caller polling continuously), or whatever the caller waits between polls.
class BatchingParser {
public:
    struct Options {
        std::size_t max_records = 8192;
        std::size_t max_bytes = std::size_t(4) << 20;
        std::chrono::microseconds max_delay{200};
        std::size_t batches = 4;               // batches kept (2..64)
        std::chrono::microseconds spin{200};   // spin before blocking in a wait (0: block at once)
    };
    using Handler = std::function<void(const ParseResult&)>;
    explicit BatchingParser(Handler handler);
    BatchingParser(Handler handler, Options options);
    ~BatchingParser();  // flush(): every record given is delivered
    BatchingParser(const BatchingParser&) = delete;
    BatchingParser& operator=(const BatchingParser&) = delete;

    void on_fragment(const std::uint8_t* data, std::size_t length);
    // After each poll: delivers every decoded batch; hands the filling batch to the decoder if its
    // oldest record has waited max_delay.  Returns the records delivered.
    std::size_t poll();
    // Decodes everything given so far and delivers it.  Returns the records delivered.
    std::size_t flush();
    std::size_t pending() const;  // given but not yet delivered
    std::uint64_t delivered() const;

private:
    struct Impl;
    std::unique_ptr<Impl> impl_;
};

using TopicMessageCallback = std::function<void(std::string_view topic, std::string_view msg_type,
                                                std::string_view uuid, std::string_view payload,
                                                std::string_view headers)>;
using AckCallback = std::function<void(const AckInfo&)>;

class MessageHandler {
public:
    MessageHandler();
    ~MessageHandler();
    void handleMessage(const ParseResult& result);  // src/message_handler.cpp:10-16
    void on_egress(const std::uint8_t* data, std::size_t len);
    // Batch form: callbacks in record order; a record where the reference throws stops the batch
    // with the same std::runtime_error after the callbacks of the records before it.
    void on_egress_batch(const std::uint8_t* data, const std::uint64_t* rec_off, std::size_t n);
    void set_topic_message_callback(TopicMessageCallback cb) { tm_cb_ = std::move(cb); }
    void set_ack_callback(AckCallback cb) { ack_cb_ = std::move(cb); }

private:
    TopicMessageCallback tm_cb_;
    AckCallback ack_cb_;
};

// The frame SessionManager::Impl publishes (src/session_manager.cpp:1050-1144): the 32-B
// SessionMessageHeader {24, 1, 111, 8, leadershipTermId, clusterSessionId, 0} followed by
// create_topic_message's record (26+Σlen bytes, timestamp = high_resolution_clock nanoseconds).
class SessionFrameEncoder {
public:
    // update_session_header (:1018-1046)
    void update_session_header(std::int64_t leadership_term_id, std::int64_t cluster_session_id) {
        leadership_term_id_ = leadership_term_id;
        cluster_session_id_ = cluster_session_id;
    }
    // One frame as send_combined_message builds it (:1118-1144); throws E109 like
    // create_topic_message (:1111-1114).
    std::vector<std::uint8_t> create_combined_message(const std::string& topic, const std::string& message_type,
                                                      const std::string& message_id, const std::string& payload,
                                                      const std::string& headers) const;
    // Batch: one GPU launch.  A message's timestamp 0 → the nanosecond clock.
    EncodedBatch encode_batch(const std::vector<TopicMessageFields>& msgs,
                              EncodeLength length = EncodeLength::Reference) const;

private:
    std::int64_t leadership_term_id_ = 0, cluster_session_id_ = 0;
};

// The raw ingress sink (ClusterClient::offer_ingress signature, include/aeron_cluster/cluster_client.hpp:409).
using OfferFn = std::function<bool(const std::uint8_t* data, std::size_t len)>;

// ClusterClient::publish_topic (src/cluster_client.cpp:1809-1864) minus the connection checks:
// uuid = "pub_" + now_nanos() (:1818), headers "{}" when empty (:1821), timestamp now_nanos()
// (:1845), sequenceNumber 0, the put*(const char*, int) length wrap (EncodeLength::Publish), and
// the record handed to the offer_ingress-shaped sink (:1860).  Returns the uuid, as the reference
// does whether or not the offer succeeded.
class TopicPublisher {
public:
    explicit TopicPublisher(OfferFn offer) : offer_(std::move(offer)) {}
    std::string publish_topic(std::string_view topic, std::string_view message_type, std::string_view json_payload,
                              std::string_view headers_json);
    // Batch form: one GPU launch for all records, offered in order; each message gets its own uuid
    // and timestamp (msgs[i].uuid / .timestamp are ignored).  Returns the uuids.
    std::vector<std::string> publish_topic_batch(const std::vector<TopicMessageFields>& msgs);

private:
    OfferFn offer_;
};

// include/aeron_cluster/commit_manager.hpp:17-24
struct CommitOffset {
    std::string topic;
    std::string message_identifier;
    std::string message_id;
    std::uint64_t timestamp_nanos = 0;
    std::uint64_t sequence_number = 0;
};

class CommitManager {
public:
    // src/commit_manager.cpp:16-22
    static std::uint32_t topic_to_id(const std::string& topic);
    // src/commit_manager.cpp:107-132: a known topic → CommitOffsetLite (template 301) with topicId,
    // sequence, messageId, messageIdentifier; E109 → std::runtime_error.  The unknown-topic
    // fallback (a jsoncpp-formatted TopicMessage, :134-160) is not built: it throws.
    std::vector<std::uint8_t> build_commit_offset_message(const std::string& topic, const std::string& client_id,
                                                          const CommitOffset& offset) const;
    // Batch (one GPU launch); every offset's topic must be known.
    EncodedBatch build_commit_offset_batch(const std::vector<CommitOffset>& offsets) const;
};

// A decoded Lite record (CommitOffsetLite / OrderRequestLite / OrderNotificationLite flyweights).
struct LiteRecord {
    std::uint16_t template_id = 0;
    std::uint32_t topic_id = 0;
    std::uint64_t sequence = 0;
    std::vector<std::string> fields;  // var strings in wire order (2 or 3)
};
// Decoded with the generated flyweights' semantics; nullopt when the record is not a Lite
// template or a bounds check throws E100.
std::optional<LiteRecord> decode_lite(const std::uint8_t* data, std::size_t len);

// LocalFragmentReassembler (src/cluster_client.cpp:39-82) for batches of Aeron fragments: fragment
// i is data[frag_off[i], frag_off[i+1]) with header flags[i] (BEGIN 0x80, END 0x40).  Returns the
// delivered messages in order; a message whose END has not arrived yet is kept for the next call,
// exactly as the reference's accumulator.
class FragmentReassembler {
public:
    EncodedBatch on_fragments(const std::uint8_t* data, const std::uint64_t* frag_off, const std::uint8_t* flags,
                              std::size_t n);
    std::size_t pending_bytes() const { return acc_.size(); }

private:
    std::vector<std::uint8_t> acc_;
};

// include/aeron_cluster/order_types.hpp:16-66: the members Order::to_json and publish_order read
// (the reference class carries more; they play no part in the text).
struct Order {
    std::string id;
    std::string client_order_uuid;
    std::string base_token;
    std::string quote_token;
    std::string side;
    double quantity = 0.0;
    std::int64_t customer_id = 0;
    std::string status = "CREATED";
    std::int64_t timestamp = 0;
    std::string identifier;
    // src/order_types.cpp:122-181 (one-record batch on the GPU)
    std::string to_json() const;
};

// A batch of Orders → Order::to_json texts (payload) and the headers JSON publish_order builds
// beside them (src/cluster_client.cpp:308-323, messageId = message_ids[i]); record i of each is
// bytes[offsets[i], offsets[i+1]), ready to be TopicMessage payload / headers.
struct OrderJsonBatch {
    EncodedBatch payload;
    EncodedBatch headers;
};
OrderJsonBatch orders_to_json(const std::vector<Order>& orders, const std::vector<std::string>& message_ids);

// Feeds every encoded record of a batch to an offer_ingress-shaped sink in order; returns the
// number accepted before the first refusal.
std::size_t offer_batch(const EncodedBatch& batch, const OfferFn& offer);

// true when a gfx950 device is usable (all entry points above need one).
bool gpu_codec_available();
// threads (the caller's included) that stage batches and build ParseResults: AERON_AMD_HOST_THREADS,
// default min(16, cores)
unsigned host_threads();

// Stops the calling thread's small-batch serve kernel if it is resident (it exits after
// AERON_AMD_SERVE_IDLE_US without a call, default 1 ms; the next small call relaunches it).  While
// resident it holds a hardware queue that other streams of the process may share, and a
// device-wide synchronisation (hipDeviceSynchronize, torch.cuda.synchronize()) waits for it to go
// idle: call this before such a synchronisation, or before handing the GPU to other work.
void quiesce();

// Page-locks a long-lived host buffer (e.g. an Aeron term buffer mapped from /dev/shm) for the
// device's copy engines: batches decoded from registered (or hipHostMalloc'd) memory are copied to
// HBM in place, without the staging copy.  The memory stays registered until host_unregister.
void host_register(const void* p, std::size_t len);
void host_unregister(const void* p);

}  // namespace aeron_cluster
