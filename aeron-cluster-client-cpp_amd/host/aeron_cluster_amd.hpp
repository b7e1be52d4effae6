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
// entry point throws std::runtime_error("sbecodec: ...").
#pragma once

#include <cstdint>
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
constexpr std::uint16_t TOPIC_SCHEMA_ID = 1;
constexpr std::uint16_t SESSION_EVENT_TEMPLATE_ID = 2;
constexpr std::uint16_t TOPIC_MESSAGE_TEMPLATE_ID = 1;
constexpr std::uint16_t ACKNOWLEDGMENT_TEMPLATE_ID = 2;
}  // namespace SBEConstants

// include/aeron_cluster/sbe_messages.hpp:306-328 (fields), :332-377 (predicates)
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

// A packed batch of encoded records: record i = bytes[offsets[i], offsets[i+1]).
struct EncodedBatch {
    std::vector<std::uint8_t> bytes;
    std::vector<std::uint64_t> offsets;
    std::vector<std::uint8_t> status;  // SBE_ENC_* per record
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
};

class MessageParser {
public:
    static ParseResult parse_message(const std::uint8_t* data, std::size_t length);
    // Batch: records data[rec_off[i], rec_off[i+1]), one GPU launch.
    static std::vector<ParseResult> parse_batch(const std::uint8_t* data, const std::uint64_t* rec_off, std::size_t n);
};

std::optional<AckInfo> decode_ack(const std::uint8_t* data, std::size_t len);

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

}  // namespace aeron_cluster
