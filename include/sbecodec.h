/*
 * sbecodec.h — C ABI of the MI355X-native batch SBE record codec.
 *
 * This is the drop-in boundary for the wire codec of reverb-sys/aeron-cluster-client-cpp
 * (reference snapshot mounted at /root/reference; all file:line citations are relative to it).
 * Every entry point is plain C: pointers, sizes and integers only.  Device pointers are HIP
 * device (or host-pinned, device-visible) pointers; `stream` is a hipStream_t passed as void*
 * (NULL = the default stream).  Nothing here allocates, synchronises or copies on the host:
 * every call is an asynchronous launch on `stream` and returns after argument validation.
 *
 * Entry point                     replaces (reference)
 * ------------------------------  ------------------------------------------------------------
 * sbe_encode_topic_batch()        SBEEncoder::encode_topic_message   src/sbe_encoder.cpp:131-167
 *                                  (decl include/aeron_cluster/sbe_messages.hpp:158-164), its live
 *                                  twin SessionManager::Impl::create_topic_message
 *                                  src/session_manager.cpp:1050-1115 and the correct-length encoder
 *                                  inside ClusterClient::publish_topic src/cluster_client.cpp:1809-1864;
 *                                  output records are what ClusterClient::offer_ingress
 *                                  (include/aeron_cluster/cluster_client.hpp:409,
 *                                  src/cluster_client_offer.cpp:11-20) receives one by one.
 * sbe_encode_session_batch()      SessionManager::Impl::publish_message's frame: create_topic_message
 *                                  src/session_manager.cpp:1050-1115 behind the 32-B
 *                                  SessionMessageHeader that send_combined_message prepends
 *                                  (:936-967 build, :1018-1046 update, :1118-1144 combine).
 * sbe_encode_lite_batch()         CommitManager::build_commit_offset_message's CommitOffsetLite
 *                                  encoder src/commit_manager.cpp:107-132 (template 301) and the
 *                                  OrderRequestLite / OrderNotificationLite flyweights (201 / 202,
 *                                  include/model/OrderRequestLite.h:114-118, :1020-1050).
 * sbe_decode_batch(LITE)          the Lite templates' generated decode flyweights
 *                                  (wrapForDecode + fixed fields + getXAsString in order,
 *                                  include/model/CommitOffsetLite.h, OrderRequestLite.h,
 *                                  OrderNotificationLite.h).
 * sbe_reassemble_fragments()      LocalFragmentReassembler::onFragment src/cluster_client.cpp:39-82
 *                                  (BEGIN / END flag reassembly of Aeron fragments, before parse).
 * sbe_decode_batch(PARSE_MESSAGE) MessageParser::parse_message      src/sbe_encoder.cpp:513-551
 *                                  (+ parse_topic_message :724-831, decode_acknowledgment_with_sbe
 *                                  :833-954, decode_topic_message_with_sbe :957-1143,
 *                                  parse_session_event :618-647) → ParseResult
 *                                  include/aeron_cluster/sbe_messages.hpp:306-412
 * sbe_decode_batch(ON_EGRESS)     decode_ack  src/ack_decoder.cpp:29-105 (AckInfo
 *                                  include/aeron_cluster/ack_decoder.hpp:9-15) and
 *                                  MessageHandler::on_egress include/aeron_cluster/message_handler.hpp:35-68
 * sbe_order_to_json_batch()       Order::to_json src/order_types.cpp:122-181 and publish_order's
 *                                  headers JSON src/cluster_client.cpp:308-323 (the strings that
 *                                  become the TopicMessage payload / headers)
 * sbe_serve_*()                   the same encoders / decoders for small batches (one record per
 *                                  call, as the reference's per-message API is used: parse_message per
 *                                  fragment src/cluster_client.cpp:1185, publish_topic per message)
 *                                  through a resident serve kernel instead of a launch per call
 * sbe_gather_encoded()            no reference counterpart (its transport is Aeron,
 *                                  src/session_manager.cpp:1180): the RCCL gather of encoded shards
 *                                  to one ingress rank
 */
#ifndef SBECODEC_H
#define SBECODEC_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define SBECODEC_ABI_VERSION 8

/* ---- return codes of every entry point ---- */
#define SBE_OK 0
#define SBE_EINVAL (-1)    /* bad argument (null pointer, n too large, bad mode) */
#define SBE_EHIP (-2)      /* a HIP launch failed (hipGetLastError != hipSuccess) */
#define SBE_ENOSPC (-3)    /* workspace too small */
#define SBE_ENODEV (-4)    /* no gfx950 device visible */

/* ---- wire constants (include/model/MessageHeader.h:95-490, TopicMessage.h:114-118,
 *      Acknowledgment.h:114-118, include/aeron_cluster/config.hpp:169-199) ---- */
#define SBE_HEADER_LEN 8u
#define SBE_TM_BLOCK_LEN 16u
#define SBE_TM_TEMPLATE_ID 1u
#define SBE_ACK_TEMPLATE_ID 2u
#define SBE_TOPIC_SCHEMA_ID 1u
#define SBE_CLUSTER_SCHEMA_ID 111u
#define SBE_SESSION_EVENT_TEMPLATE_ID 2u
#define SBE_TM_FIELDS 5u           /* topic, messageType, uuid, payload, headers */
#define SBE_TM_WIRE_OVERHEAD 34u   /* 8 header + 16 block + 5 x u16 length */
#define SBE_TM_REF_OVERHEAD 26u    /* reference encode_topic_message emits 8 B less */
#define SBE_VAR_MAX_LEN 65534u     /* TopicMessage.h:1396-1428 (E109 above this) */
#define SBE_SESSION_HDR_LEN 32u    /* SessionMessageHeader {24,1,111,8} + termId, sessionId, ts=0
                                      (src/session_manager.cpp:936-967) */
#define SBE_SESSION_BLOCK_LEN 24u
#define SBE_SESSION_TEMPLATE_ID 1u
#define SBE_CLUSTER_SCHEMA_VERSION 8u
#define SBE_LITE_BLOCK_LEN 12u     /* u32 topicId @0, u64 sequence @4 (CommitOffsetLite.h:114, :337-420) */
#define SBE_ORDER_REQUEST_LITE_TEMPLATE_ID 201u      /* uuid, messageIdentifier, payload */
#define SBE_ORDER_NOTIFICATION_LITE_TEMPLATE_ID 202u /* uuid, messageIdentifier, payload */
#define SBE_COMMIT_OFFSET_LITE_TEMPLATE_ID 301u      /* messageId, messageIdentifier */

/* ===================================== encode ===================================== */

/* encode flags */
#define SBE_ENC_REF_TRUNCATE8 0x1u /* emit exactly what SBEEncoder::encode_topic_message returns:
                                      buffer.resize(encodedLength()) keeps only the first
                                      26+Σlen bytes of the wire record (src/sbe_encoder.cpp:163-164) */
#define SBE_ENC_PUBLISH_TOPIC 0x2u /* the encoder block of ClusterClient::publish_topic
                                      (src/cluster_client.cpp:1823-1858): wire length, and the
                                      put*(const char*, int) overloads (TopicMessage.h:515-529) that
                                      take the length as std::uint16_t: a field of L bytes writes
                                      length L mod 65536 followed by its first L mod 65536 bytes; no
                                      E109 (computeLength is never called).  Topic batches only; not
                                      with SBE_ENC_REF_TRUNCATE8.  The caller supplies the uuid
                                      ("pub_" + now_nanos(), :1818) and "{}" for empty headers (:1821),
                                      as the host mirror's publish_topic does. */

/* Lite records: 8 header {12, template, 1, 1} + 12 block + nf x (u16 length + bytes), nf = 2
 * (301) or 3 (201, 202).  Wire overhead 20 + 2 nf; no truncation (8 + encodedLength() is the
 * whole record, src/commit_manager.cpp:129-130). */
#define SBE_LITE_OVERHEAD(nf) (20u + 2u * (nf))

/* per-record encode status */
#define SBE_ENC_OK 0u
#define SBE_ENC_E109_TOPIC 1u        /* "topicLength too long for length type [E109]" */
#define SBE_ENC_E109_MESSAGE_TYPE 2u /* "messageTypeLength too long for length type [E109]" */
#define SBE_ENC_E109_UUID 3u         /* "uuidLength too long for length type [E109]" */
#define SBE_ENC_E109_PAYLOAD 4u      /* "payloadLength too long for length type [E109]" */
#define SBE_ENC_E109_HEADERS 5u      /* "headersLength too long for length type [E109]" */
#define SBE_ENC_OVERFLOW 6u          /* record does not fit in out_capacity (nothing written) */
/* Lite templates: status 1 + f = "<field f>Length too long for length type [E109]" with the
 * template's field names in wire order (computeLength, e.g. CommitOffsetLite.h:839-870). */

/* A batch of TopicMessages in struct-of-arrays form.  Field order per record is the wire order
 * topic, messageType, uuid, payload, headers (TopicMessage.h:515-1231).
 *   arena      string bytes.
 *   str_off    [n][5] byte offsets into arena, or NULL: "packed" — the strings of record 0..n-1
 *              lie back to back in arena in record-major, field-minor order from arena[0].
 *   str_len    [n][5] lengths (> 65534 → E109, the record emits no bytes).
 *   timestamp  [n]; 0 is replaced by ts_default (the reference substitutes the wall clock for 0,
 *              src/sbe_encoder.cpp:134-138; the caller passes that clock value). */
typedef struct sbe_tm_batch {
    const uint8_t* arena;
    const uint32_t* str_off;
    const uint32_t* str_len;
    const uint64_t* timestamp;
} sbe_tm_batch;

/* Bytes of device workspace sbe_encode_topic_batch needs for n records (look-back tile state). */
size_t sbe_encode_workspace_size(uint64_t n);

/* Optional: zero a workspace (hipMemsetAsync on `stream`).  The encoder needs no particular
 * workspace contents; a workspace serves one stream at a time. */
int sbe_encode_workspace_init(void* workspace, size_t workspace_bytes, void* stream);

/* Upper bound of the encoded stream for a batch whose strings total `string_bytes`. */
uint64_t sbe_encode_output_bound(uint64_t n, uint64_t string_bytes, uint32_t flags);

/* Encode n TopicMessages into one packed byte stream.
 *   out        device buffer of out_capacity bytes; record i is out[out_off[i] .. out_off[i+1]).
 *   out_off    [n+1] u64 device array (written).
 *   status     [n] u8 device array (written) or NULL.
 *   workspace  device memory of >= sbe_encode_workspace_size(n) bytes, 16-B aligned.
 *   alignment  out 16 B, out_off 8 B (arena, str_off, str_len, timestamp: natural alignment).
 * Records are independent; a failing record (E109, overflow) emits 0 bytes and the batch goes on. */
int sbe_encode_topic_batch(const sbe_tm_batch* in, uint64_t n, uint64_t ts_default, uint32_t flags,
                           uint8_t* out, uint64_t out_capacity, uint64_t* out_off, uint8_t* status,
                           void* workspace, size_t workspace_bytes, void* stream);

/* Session-framed encode: every record is the 32-B SessionMessageHeader
 *   {blockLength 24, templateId 1, schemaId 111, version 8, i64 leadershipTermId,
 *    i64 clusterSessionId, i64 timestamp 0}
 * followed by the TopicMessage exactly as sbe_encode_topic_batch emits it under `flags`
 * (SBE_ENC_REF_TRUNCATE8: the 26+Σlen bytes create_topic_message returns, which is what the live
 * publish path sends; 0: the wire-correct 34+Σlen).  Record i = out[out_off[i]..out_off[i+1]) is
 * one Publication::offer of send_combined_message.  Workspace, alignment and status as for
 * sbe_encode_topic_batch. */
int sbe_encode_session_batch(const sbe_tm_batch* in, uint64_t n, uint64_t ts_default, uint32_t flags,
                             int64_t leadership_term_id, int64_t cluster_session_id, uint8_t* out,
                             uint64_t out_capacity, uint64_t* out_off, uint8_t* status, void* workspace,
                             size_t workspace_bytes, void* stream);

/* A batch of Lite records (struct of arrays):
 *   arena, str_off ([n][nf] or NULL = packed), str_len [n][nf]: the var strings in wire order;
 *   topic_id [n]: u32 topicId; sequence [n]: u64 sequence. */
typedef struct sbe_lite_batch {
    const uint8_t* arena;
    const uint32_t* str_off;
    const uint32_t* str_len;
    const uint32_t* topic_id;
    const uint64_t* sequence;
} sbe_lite_batch;

/* Fields per record of a Lite template (2 or 3), 0 if template_id is not one of them. */
uint32_t sbe_lite_fields(uint32_t template_id);

/* Upper bound of the encoded stream of a Lite batch whose strings total `string_bytes`. */
uint64_t sbe_lite_output_bound(uint64_t n, uint64_t string_bytes, uint32_t template_id);

/* Encode n Lite records of template_id (201, 202 or 301).  Outputs, workspace and alignment as
 * for sbe_encode_topic_batch (the same workspace size). */
int sbe_encode_lite_batch(const sbe_lite_batch* in, uint64_t n, uint32_t template_id, uint8_t* out,
                          uint64_t out_capacity, uint64_t* out_off, uint8_t* status, void* workspace,
                          size_t workspace_bytes, void* stream);

/* ===================================== decode ===================================== */

#define SBE_DEC_PARSE_MESSAGE 0u /* MessageParser::parse_message semantics → ParseResult */
#define SBE_DEC_ON_EGRESS 1u     /* MessageHandler::on_egress semantics (decode_ack first) */
#define SBE_DEC_LITE 2u          /* Lite-template flyweight decode (201 / 202 / 301) */

/* per-record decode status.  Parse mode (0..31): */
#define SBE_ST_TM 0u                 /* TopicMessage: views topic,type,uuid,payload,headers */
#define SBE_ST_ACK 1u                /* Acknowledgment (printable-run heuristic): views 0..2 */
#define SBE_ST_SESSION_EVENT 2u      /* SessionEvent: view 3 = detail (u32-prefixed) */
#define SBE_ST_ERR_NULL_EMPTY 16u    /* "Null or empty data" */
#define SBE_ST_ERR_HEADER 17u        /* "Failed to decode message header" */
#define SBE_ST_ERR_UNKNOWN_TYPE 18u  /* "Unknown message type: template=T, schema=S" (hdr kept) */
#define SBE_ST_ERR_SESSION_EVENT 19u /* "Failed to decode SessionEvent" */
#define SBE_ST_ERR_SESSION_SHORT 20u /* "Session message too short to contain embedded message" */
#define SBE_ST_ERR_EMBEDDED_SHORT 21u /* "Embedded message too short" */
#define SBE_ST_ERR_EMBEDDED_TEMPLATE 22u /* "Unknown embedded message template_id: <param>" */
#define SBE_ST_ERR_EMBEDDED_SCHEMA 23u   /* "Unknown embedded message schema_id: <param>" */
#define SBE_ST_ERR_DIRECT_TEMPLATE 24u   /* "Unknown direct message template_id: <param>" */
#define SBE_ST_ERR_TM_E100 25u       /* "SBE TopicMessage decoding failed: buffer too short [E100]" */
#define SBE_ST_ERR_ACK_SHORT 26u     /* "Buffer too short for Acknowledgment message. Need at least
                                         16 bytes, got <param>" */
/* On-egress mode (32..): */
#define SBE_ST_EG_ACK_SIMPLE 32u     /* decode_ack simple 16-B control ack; ts = timestamp_nanos */
#define SBE_ST_EG_ACK 33u            /* decode_ack full ack; views messageId,topic,correlationId */
#define SBE_ST_EG_TM 34u             /* topic-message callback; views topic,type,uuid,payload,headers */
#define SBE_ST_EG_NONE 35u           /* on_egress returns without a callback */
#define SBE_ST_EG_THROW_E100 36u     /* on_egress throws std::runtime_error("buffer too short [E100]") */
/* Lite mode (48..): the generated flyweight sequence MessageHeader::wrap, wrapForDecode(buf, 8,
 * blockLength, version, len), topicId(), sequence(), getXAsString() per var field in order. */
#define SBE_ST_LITE 48u              /* decoded: ts = sequence, view_off[4] = topicId, views 0..nf-1 */
#define SBE_ST_LITE_E100 49u         /* a flyweight bounds check threw "buffer too short [E100]" (also:
                                         the 12 fixed bytes lie past the record) */
#define SBE_ST_LITE_NOT_LITE 50u     /* len < 8, schema != 1 or template not 201/202/301 (hdr kept
                                         when len >= 8) */

/* per-record decode flags */
#define SBE_FL_ID_DEFAULT 0x1u      /* ack: message_id = "ack_" + decimal(ts) */
#define SBE_FL_PAYLOAD_DEFAULT 0x2u /* ack: payload = "SUCCESS" */
#define SBE_FL_HEADERS_E100 0x4u    /* TM: headers read hit E100 and was swallowed (headers = "") */
#define SBE_FL_SEQ_KEY 0x8u         /* TM: payload (>= 16 B) contains the bytes "_sequence_number" */
#define SBE_FL_WRAPPED 0x10u        /* record was a schema-111 session message (embedded decode) */
#define SBE_FL_SEQ_ESC 0x20u        /* TM: payload (>= 16 B) contains a '\\' byte (a key spelled with
                                       \u escapes decodes to "_sequence_number" without containing it) */
/* A TM record without SEQ_KEY and SEQ_ESC has ParseResult.sequence_number == 0 under any JSON
 * parser; sbe_eval_sequence_numbers evaluates the others. */

/* Decoded records, struct of arrays, all device arrays of n (or n*4 / n*5) elements.
 *   hdr      [n][4] block_length, template_id, schema_id, version as ParseResult reports them.
 *   ts       [n] ParseResult.timestamp / AckInfo.timestamp_nanos.
 *   view_off [n][5], view_len [n][5]: byte ranges relative to the record's first byte.
 *            For statuses with a parameter, view_off[i*5] holds it. */
typedef struct sbe_decoded {
    uint8_t* status;
    uint8_t* flags;
    uint16_t* hdr;
    uint64_t* ts;
    uint32_t* view_off;
    uint32_t* view_len;
    uint64_t* seq; /* optional (NULL: skip), parse mode only: seq[i] = ParseResult.sequence_number of
                      every TopicMessage flagged SBE_FL_SEQ_KEY / SBE_FL_SEQ_ESC, evaluated in the same
                      launch (see sbe_eval_sequence_numbers); other entries are not written (8-B aligned) */
} sbe_decoded;

/* Decode n records; record i is in[rec_off[i] .. rec_off[i+1]) (rec_off: [n+1] device u64).
 * Record boundaries come from the transport (Aeron fragments, src/cluster_client.cpp:541-546):
 * the SBE header carries no total length.  Alignment: in 16 B, rec_off/hdr/ts 8 B, views 4 B. */
int sbe_decode_batch(const uint8_t* in, const uint64_t* rec_off, uint64_t n, uint32_t mode,
                     const sbe_decoded* out, void* stream);

/* sbe_decode_batch with the batch's total record bytes (rec_off[n] - rec_off[0]) as the caller
 * knows them, used only to pick the kernel shape (the LDS window of a 64-record tile, which caps
 * the workgroups per CU): records over 320 B on average (long payloads) 13 KiB windows, over 256 B
 * (session frames) 12 KiB (a tile takes two or more); up to 112 B 8 KiB; up to 204 B 15 KiB;
 * others 16 KiB.
 * in_bytes = 0: the 16 KiB kernel.  Outputs are identical either way. */
int sbe_decode_batch_sized(const uint8_t* in, const uint64_t* rec_off, uint64_t n, uint64_t in_bytes, uint32_t mode,
                           const sbe_decoded* out, void* stream);

/* ParseResult.sequence_number (src/sbe_encoder.cpp:1031-1125) as a separate launch, for
 * descriptors decoded with seq == NULL: for every record that
 * sbe_decode_batch(SBE_DEC_PARSE_MESSAGE) left with status SBE_ST_TM and flag SBE_FL_SEQ_KEY or
 * SBE_FL_SEQ_ESC, parse its payload with the semantics of jsoncpp 1.9.5's CharReaderBuilder
 * defaults (comments and trailing commas allowed, extra content after the root ignored, stack
 * limit 1000, UTF-8 BOM skipped) and write seq[i] = the first non-zero "_sequence_number" of
 * root, root.message, root.message.message, root.message.message.message (extractSequence:
 * integers as u64, other numbers through a correctly rounded double and the x86-64 cast, strings
 * through std::stoull), or 0 when the payload does not parse.  seq[i] of any other record is not
 * written: its sequence_number is 0.  in / rec_off / status / flags / view_* are the arguments and
 * outputs of that decode call; seq is a device u64[n] (8-B aligned).  Same stream order rules. */
int sbe_eval_sequence_numbers(const uint8_t* in, const uint64_t* rec_off, uint64_t n, const sbe_decoded* dec,
                              uint64_t* seq, void* stream);

/* MATERIALIZE: the five views of every decoded record copied out of the input into one arena, so
 * that the strings outlive the input buffer, as the reference's ParseResult owns its std::strings
 * (include/aeron_cluster/sbe_messages.hpp:306-328) and a poll callback's fragment dies with the
 * callback (src/cluster_client.cpp:541-546).  After sbe_decode_batch[_sized] on the same in /
 * rec_off (dec: its outputs), view k of record i goes to arena[arena_off[5 i + k] ..) with
 * view_len[i][k] bytes, views in record order and back to back (arena_off: device u64 [5 n + 1],
 * the last entry the total; a view of length 0, including the Lite topicId slot, takes no bytes).
 * A view that would end past arena_capacity is not written (arena_off still holds the full
 * layout, so the caller can size the arena from arena_off[5 n] and rerun); nothing is written past
 * arena_capacity.  Workspace: sbe_materialize_workspace_size(n) bytes (16-B aligned). */
size_t sbe_materialize_workspace_size(uint64_t n);
int sbe_materialize_views(const uint8_t* in, const uint64_t* rec_off, uint64_t n, const sbe_decoded* dec,
                          uint8_t* arena, uint64_t arena_capacity, uint64_t* arena_off, void* workspace,
                          size_t workspace_bytes, void* stream);

/* ============================ Aeron fragment reassembly ============================ */
/* Replaces LocalFragmentReassembler::onFragment (src/cluster_client.cpp:39-82) for a batch of
 * fragments, in arrival order:
 *   flags[i] & (BEGIN|END) == BEGIN|END   the fragment is a whole message;
 *   otherwise   BEGIN clears the accumulator, the fragment is appended, END delivers the
 *               accumulator as one message and clears it.
 * in[frag_off[i] .. frag_off[i+1]) is fragment i (frag_off: n + 1 device u64).
 * Outputs: the delivered messages back to back in delivery order, out[msg_off[j] .. msg_off[j+1])
 * for j < m; then the open accumulator ("carry", bytes of a message whose END has not arrived)
 * at out[msg_off[m] .. msg_off[m] + carry).  counts (device u64[2]) = {m, carry}.  To continue
 * with the next batch, pass the carry bytes as its first fragment with flags 0 (a middle
 * fragment appends exactly as the accumulator would).
 * out must hold frag_off[n] - frag_off[0] bytes, msg_off n + 1 entries. */
#define SBE_FRAG_BEGIN 0x80u
#define SBE_FRAG_END 0x40u
size_t sbe_reassemble_workspace_size(uint64_t n);
int sbe_reassemble_fragments(const uint8_t* in, const uint64_t* frag_off, const uint8_t* flags, uint64_t n,
                             uint8_t* out, uint64_t* msg_off, uint64_t* counts, void* workspace,
                             size_t workspace_bytes, void* stream);

/* ========================== Order JSON (publish_order payload) ========================== */
/* Replaces Order::to_json (src/order_types.cpp:122-181, jsoncpp StreamWriterBuilder with
 * indentation "" → compact, keys sorted) and the headers JSON publish_order builds beside it
 * (src/cluster_client.cpp:308-323), for a batch of Orders, so the strings feed
 * sbe_encode_topic_batch as payload / headers without a host round trip.
 * A batch of Orders (struct of arrays; order_types.hpp:16-66):
 *   arena, str_off ([n][8] or NULL = packed), str_len [n][8]: the string members
 *     0 client_order_uuid, 1 identifier, 2 base_token, 3 quote_token, 4 side, 5 id,
 *     6 message_id (OrderUtils::generate_message_id's value, made by the caller),
 *     7 status (selects messageType: "UPDATED" / "CANCELLED" → UPDATE_ORDER, else CREATE_ORDER);
 *   customer_id [n], timestamp [n] (ns; create_ts = timestamp / 1000000), quantity [n] (f64).
 * Number text follows glibc printf on the exact binary value: "%.17g" (jsoncpp valueToString,
 * ".0" appended when there is no '.' or 'e'; NaN → null, ±inf → ±1e+9999) and "%f"
 * (std::to_string); strings are escaped as jsoncpp 1.9.5 valueToQuotedStringN with emitUTF8
 * false (\" \\ \b \f \n \r \t, other controls and every non-ASCII code point as lower-case \uXXXX,
 * invalid UTF-8 as �); identifier is cut at its first NUL (.c_str(), order_types.cpp:138). */
#define SBE_ORDER_FIELDS 8u
#define SBE_JSON_ORDER_PAYLOAD 0u   /* Order::to_json() */
#define SBE_JSON_PUBLISH_HEADERS 1u /* {"messageId":…,"messageType":…,"orderId":…} */
#define SBE_JSON_OK 0u
#define SBE_JSON_OVERFLOW 6u        /* record ends past out_capacity (nothing written) */
typedef struct sbe_order_batch {
    const uint8_t* arena;
    const uint32_t* str_off;
    const uint32_t* str_len;
    const int64_t* customer_id;
    const int64_t* timestamp;
    const double* quantity;
} sbe_order_batch;

/* Bytes of device workspace sbe_order_to_json_batch needs for n records. */
size_t sbe_order_json_workspace_size(uint64_t n);

/* Write the JSON text of n Orders back to back: record i = out[out_off[i] .. out_off[i+1]).
 * out_off (n + 1 device u64) always holds the full sizes; a record past out_capacity is not
 * written and gets status SBE_JSON_OVERFLOW (status: n device u8 or NULL).  On `stream`: a
 * sizing launch, a one-block scan of its per-block sums and the writing launch (packed arena:
 * first a per-block string-bytes launch and its scan). */
int sbe_order_to_json_batch(const sbe_order_batch* in, uint64_t n, uint32_t what, uint8_t* out,
                            uint64_t out_capacity, uint64_t* out_off, uint8_t* status, void* workspace,
                            size_t workspace_bytes, void* stream);

/* ======================= multi-GPU gather of encoded shards (RCCL) ======================= */
/* A batch sharded over the GPUs of one node (records [lo_r, hi_r) on rank r, contiguous, in rank
 * order) is encoded per rank with no collective; sbe_gather_encoded then assembles on one rank the
 * stream and offsets a single-GPU encode of the whole batch produces, over RCCL (xGMI inside a
 * node).  The reference has no counterpart: its only transport is Aeron
 * (src/session_manager.cpp:1180); the gathered stream is what one ingress publisher offers
 * record by record (ClusterClient::offer_ingress, include/aeron_cluster/cluster_client.hpp:409).
 * One process per GPU; a communicator serves one stream at a time. */
#define SBE_ECOMM (-5)       /* an RCCL call failed (sbe_last_error names it) */
#define SBE_COMM_ID_BYTES 128u
typedef struct sbe_comm sbe_comm;

/* A fresh communicator id (ncclGetUniqueId), made on one rank and passed to every rank out of band. */
int sbe_comm_unique_id(uint8_t id[SBE_COMM_ID_BYTES]);
/* Collective over the `world` processes: create this rank's communicator on the current HIP device. */
int sbe_comm_init(sbe_comm** comm, int world, int rank, const uint8_t id[SBE_COMM_ID_BYTES]);
int sbe_comm_destroy(sbe_comm* comm);

/* Collective over the communicator.  Every rank passes its shard: out (its encoded stream, 16-B
 * aligned) with out_off [n+1] (device u64, out_off[0] == 0) as sbe_encode_*_batch wrote them.
 * The root receives the shards back to back in rank order into dst (dst_capacity bytes) and the
 * rebased offsets into dst_off (dst_off_capacity device u64 entries; N + 1 are written, N = Σ n_r:
 * record j of rank r at Σ_{q<r} bytes_q + out_off_r[j]); other ranks pass dst = dst_off = NULL and
 * capacities 0.  totals (host u64[2], or NULL) = {Σ bytes, N} on every rank.  On `stream`: an
 * all-gather of the ranks' {bytes, n, root capacities}, one 32-B-per-rank device→host copy and a
 * synchronisation of `stream` (the root sizes its receives from it), the plan of sbe_gather_plan,
 * then one group of ncclSend / ncclRecv at the prefix offsets (RCCL has no gatherv) and the root's
 * offset rebase; returns once those are enqueued.  SBE_ENOSPC on every rank (nothing sent) when the
 * root's dst or dst_off is too small.  RCCL is loaded on the first sbe_comm_* call (the RCCL the
 * process already holds, else librccl.so.1); nothing else in this library needs it. */
int sbe_gather_encoded(sbe_comm* comm, int root, const uint8_t* out, const uint64_t* out_off, uint64_t n,
                       uint8_t* dst, uint64_t dst_capacity, uint64_t* dst_off, uint64_t dst_off_capacity,
                       uint64_t* totals, void* stream);

/* The same gather for a caller that already knows every rank's shard size (fixed-size records:
 * bytes = records x record size; or the host size plan the C++ mirror keeps for every encode):
 * sizes (host u64 [world][2]) = {bytes, records} of each rank's shard, identical on every rank.
 * No size all-gather and no host synchronisation: it enqueues the grouped ncclSend / ncclRecv and
 * the root's rebase on `stream` and returns, so a rank can go on to encode its next shard while
 * this one travels.  dst_capacity / dst_off_capacity are the ROOT's capacities, passed on every
 * rank (non-roots pass dst = dst_off = NULL), so every rank reaches the same SBE_ENOSPC verdict
 * before anything is sent; dst_off_capacity 0 is SBE_EINVAL (N + 1 >= 1 offsets are always
 * written), and a rank that passes other capacities than the root's can leave the root blocked in
 * its receives, so the Python binding refuses zero capacities on every rank.  The sizes are trusted as a planned encode's tile sums are: they must
 * equal out_off[n] and n of the shard each rank encoded (a wrong plan moves the wrong bytes; it
 * never writes past the root's capacities). */
int sbe_gather_encoded_sized(sbe_comm* comm, int root, const uint64_t* sizes, const uint8_t* out,
                             const uint64_t* out_off, uint8_t* dst, uint64_t dst_capacity, uint64_t* dst_off,
                             uint64_t dst_off_capacity, uint64_t* totals, void* stream);

/* The gather's plan (host only, no device): from every rank's {bytes, records, dst_capacity,
 * dst_off_capacity} (ranks: host u64 [world][4], the capacities read from the root's entry) the
 * byte and record base of each rank's shard on the root (byte_base / rec_base: host u64
 * [world + 1], exclusive prefix sums; the last entry is the total) and totals {Σ bytes, Σ records}
 * (or NULL).  SBE_ENOSPC when the root's dst holds fewer than Σ bytes or its dst_off fewer than
 * Σ records + 1 entries; SBE_EINVAL on a bad world / root. */
int sbe_gather_plan(const uint64_t* ranks, int world, int root, uint64_t* byte_base, uint64_t* rec_base,
                    uint64_t* totals);

/* ============================ small-batch serve kernel ============================ */
/* A one-record call through the batch entry points pays a kernel launch and a completion wait
 * (≈12 us round trip on MI355X, profiles/r04_launch_probe.log) on top of its few microseconds of
 * work: the reference's per-message calls (SBEEncoder::encode_topic_message,
 * src/sbe_encoder.cpp:131-181; SBEDecoder/parse_message, src/sbe_encoder.cpp:183-318 and
 * 915-1029; ClusterClient::publish_topic, src/cluster_client.cpp:1850-1857) cost well under that
 * on a CPU.  A server is one resident workgroup on its own HIP stream that polls a page-locked
 * request slot and runs each small batch as it arrives (no launch per request, ≈3 us round
 * trip), then exits after `idle_us` without a request; the next request relaunches it.
 * Every sbe_serve_* call is synchronous: it returns when the outputs are written (or with the
 * error the batch entry point would return, checked on the host before posting).  Outputs are
 * byte-identical to the batch entry points'.  Pointers are device-visible addresses (device
 * memory, or page-locked host memory's device pointer); encodes take packed input only
 * (str_off == NULL); n <= SBE_SERVE_MAX_RECORDS (one workgroup walks the batch tile by tile, so
 * large batches belong on the batch entry points).  A server is used by one host thread at a time. */
#define SBE_SERVE_MAX_RECORDS 4096u
typedef struct sbe_server sbe_server;
/* idle_us: how long the resident kernel waits for a request before it exits (0: 1000).  Keep it
 * short: see sbe_server_quiesce on what a resident server holds up. */
int sbe_server_create(sbe_server** srv, uint32_t idle_us);
/* A server of `workgroups` resident workgroups (1..SBE_SERVE_MAX_WORKGROUPS): workgroup 0 polls the
 * slot and republishes a request of several tiles to the others through device memory; a decode
 * of T tiles (64 records each) then runs on min(T, workgroups) of them, as does a planned encode
 * (below).  One-tile requests run on workgroup 0 alone, as with sbe_server_create. */
#define SBE_SERVE_MAX_WORKGROUPS 64u
int sbe_server_create_wide(sbe_server** srv, uint32_t idle_us, uint32_t workgroups);
/* Stops the kernel (a shutdown request, then the stream is synchronised) and frees the server.
 * A request that times out (10 s) or finds the server's stream failed returns SBE_EHIP and leaves
 * the server failed: every later request returns SBE_EHIP at once, and destroy only waits for the
 * kernel to leave (it exits idle_us after its last request) before freeing.  That wait is bounded
 * (idle_us + 10 s): a kernel still running then is left with its buffers (never freed under it)
 * and destroy returns SBE_EHIP. */
int sbe_server_destroy(sbe_server* srv);
int sbe_serve_encode_topic(sbe_server* srv, const sbe_tm_batch* in, uint64_t n, uint64_t ts_default, uint32_t flags,
                           uint8_t* out, uint64_t out_capacity, uint64_t* out_off, uint8_t* status);
int sbe_serve_encode_session(sbe_server* srv, const sbe_tm_batch* in, uint64_t n, uint64_t ts_default,
                             uint32_t flags, int64_t leadership_term_id, int64_t cluster_session_id, uint8_t* out,
                             uint64_t out_capacity, uint64_t* out_off, uint8_t* status);
int sbe_serve_encode_lite(sbe_server* srv, const sbe_lite_batch* in, uint64_t n, uint32_t template_id, uint8_t* out,
                          uint64_t out_capacity, uint64_t* out_off, uint8_t* status);
/* sbe_decode_batch's modes and outputs (seq evaluated in the same request when non-NULL). */
int sbe_serve_decode(sbe_server* srv, const uint8_t* in, const uint64_t* rec_off, uint64_t n, uint32_t mode,
                     const sbe_decoded* out);
/* The same with the inputs in host memory (any memory the calling thread reads; packed strings,
 * no alignment needed): they are copied into the server's request slot, and the kernel moves them
 * to device scratch in the round trip that fetches the request, so its dependent reads (offsets,
 * then records; lengths, then strings) hit the L2 instead of crossing PCIe twice.  At most
 * SBE_SERVE_INLINE_BYTES of inputs per request, laid out 16-B aligned: decode
 * 8 (n + 1) + (rec_off[n] - rec_off[0]); encode Σlen + 4 nf n + 8 n (+ 4 n Lite topicIds).
 * SBE_EINVAL when they do not fit.  Outputs are device-visible pointers, as above. */
#define SBE_SERVE_INLINE_BYTES 16384u
int sbe_serve_encode_topic_host(sbe_server* srv, const sbe_tm_batch* in, uint64_t n, uint64_t ts_default,
                                uint32_t flags, uint8_t* out, uint64_t out_capacity, uint64_t* out_off,
                                uint8_t* status);
int sbe_serve_encode_session_host(sbe_server* srv, const sbe_tm_batch* in, uint64_t n, uint64_t ts_default,
                                  uint32_t flags, int64_t leadership_term_id, int64_t cluster_session_id,
                                  uint8_t* out, uint64_t out_capacity, uint64_t* out_off, uint8_t* status);
int sbe_serve_encode_lite_host(sbe_server* srv, const sbe_lite_batch* in, uint64_t n, uint32_t template_id,
                               uint8_t* out, uint64_t out_capacity, uint64_t* out_off, uint8_t* status);
int sbe_serve_decode_host(sbe_server* srv, const uint8_t* in, const uint64_t* rec_off, uint64_t n, uint32_t mode,
                          const sbe_decoded* out);
/* Planned encodes: device-visible inputs (packed) plus the tile sums sbe_encode_*_batch's first
 * launch would compute, supplied by a caller that knows every record's sizes (the C++ mirror
 * does): tile_sums [T][2] = output / input bytes before tile t inside its superblock, sb_sums
 * [S][2] = output / input bytes of superblock s, with T = ceil(n / R) tiles of R =
 * sbe_encode_tile_records(layout) records and superblocks of 128 R records; a record's output
 * bytes are 0 for an E109 record, its input bytes the sum of its string lengths.  The tile loop
 * of the batch kernel then runs on min(T, workgroups) workgroups.  Outputs are byte-identical.
 * The sums are trusted as the lengths are: output stores stay inside out_capacity whatever they
 * say, but input reads follow them, so sums that do not match the lengths read past the arena
 * (undefined, as lengths that overrun the arena are for every encode entry point). */
#define SBE_LAYOUT_TOPIC 0u
#define SBE_LAYOUT_SESSION 1u
#define SBE_LAYOUT_LITE 2u
uint32_t sbe_encode_tile_records(uint32_t layout);
int sbe_serve_encode_topic_planned(sbe_server* srv, const sbe_tm_batch* in, uint64_t n, uint64_t ts_default,
                                   uint32_t flags, uint8_t* out, uint64_t out_capacity, uint64_t* out_off,
                                   uint8_t* status, const uint64_t* tile_sums, const uint64_t* sb_sums);
int sbe_serve_encode_session_planned(sbe_server* srv, const sbe_tm_batch* in, uint64_t n, uint64_t ts_default,
                                     uint32_t flags, int64_t leadership_term_id, int64_t cluster_session_id,
                                     uint8_t* out, uint64_t out_capacity, uint64_t* out_off, uint8_t* status,
                                     const uint64_t* tile_sums, const uint64_t* sb_sums);
int sbe_serve_encode_lite_planned(sbe_server* srv, const sbe_lite_batch* in, uint64_t n, uint32_t template_id,
                                  uint8_t* out, uint64_t out_capacity, uint64_t* out_off, uint8_t* status,
                                  const uint64_t* tile_sums, const uint64_t* sb_sums);
/* Makes a resident server exit now (a shutdown request, then its stream is synchronised) and
 * keeps it usable: the next request relaunches it.  SBE_OK at once when it is not running.
 *
 * WHY THIS MATTERS.  While its kernel is resident (from a request until idle_us after the last
 * one), a server occupies a HIP hardware queue, and HIP maps streams onto GPU_MAX_HW_QUEUES
 * queues (4 by default) shared by every stream of the process.  Work on a stream that shares the
 * server's queue, and any device-wide synchronisation (hipDeviceSynchronize,
 * torch.cuda.synchronize()), waits until the server exits: up to idle_us after its last request,
 * and for as long as its owner keeps it busy.  Quiesce the thread's server before such a
 * synchronisation or before enqueueing large work; keep idle_us short (the C++ mirror's default is
 * 1 ms, and the mirror quiesces its own server before every batch it launches). */
int sbe_server_quiesce(sbe_server* srv);
/* Requests this server ran and kernel launches it took (a launch per idle exit). */
int sbe_server_stats(const sbe_server* srv, uint64_t* requests, uint64_t* launches);

/* ================================== profiling ================================== */
/* Optional (off by default; thread-local): sbe_profile_enable(every) with every >= 1 makes every
 * `every`-th sbe_encode_topic_batch / sbe_decode_batch call of this thread carry a pair of HIP
 * events on its main kernel's dispatch (kernel 0 = the encode pack kernel, 1 = the decode
 * kernel; hipExtLaunchKernel timestamps), kept in a ring of the last 256 per kernel; 0 turns it
 * off.  Each call resets the rings and launch counters (the first enabling call creates the events,
 * so none is created inside a timed region; SBE_EHIP when they cannot be created, e.g. no device).  sbe_profile_read copies the elapsed
 * milliseconds of up to `max` most recent sampled launches (oldest first) into ms[], clears the
 * ring and returns the count; the caller synchronises the streams first.  Used by bench.py to
 * time the dominant kernel inside its timed region (a timed dispatch costs the GPU several us,
 * hence the sampling). */
int sbe_profile_enable(int every);
int sbe_profile_read(int kernel, float* ms, int max);

/* ===================================== misc ===================================== */
int sbe_abi_version(void);
/* 1 if a gfx950 device is visible to HIP, 0 if not, <0 on HIP error. */
int sbe_device_ready(void);
/* Name of the last HIP error seen by this library (thread-local), "" if none. */
const char* sbe_last_error(void);

#ifdef __cplusplus
}
#endif
#endif /* SBECODEC_H */
