/*
 * sbe_oracle.h — TEST INFRASTRUCTURE ONLY.
 *
 * CPU restatement (plain C) of the reference codec semantics, used as the parity checker by
 * tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg.  Never linked into, loaded
 * by or called from the product library (libsbecodec.so) or its host mirror.
 *
 * Pinned by: tests/golden/ fixtures produced by oracle/_ref (the reference's own SBE-generated
 * flyweights, compiled from the model headers under /root/reference/include by oracle/Makefile) and the
 * reference probe observations recorded in SURVEY.md Appendix B.  See DESIGN.md §Oracle.
 *
 * The batch entry points produce exactly the device output layout of include/sbecodec.h.
 */
#ifndef SBE_ORACLE_H
#define SBE_ORACLE_H

#include <stddef.h>
#include <stdint.h>

#include "../include/sbecodec.h"

#ifdef __cplusplus
extern "C" {
#endif

/* One TopicMessage, SBEEncoder::encode_topic_message (src/sbe_encoder.cpp:131-167).
 * s[f]/len[f] field f of topic,messageType,uuid,payload,headers.  Writes the record to out
 * (capacity >= 34 + Σlen) and returns its byte count; returns 0 and sets *status on E109. */
uint64_t orc_encode_one(const uint8_t* const s[5], const uint32_t len[5], uint64_t ts,
                        uint32_t flags, uint8_t* out, uint8_t* status);

/* Batch encode with the exact semantics/outputs of sbe_encode_topic_batch (no capacity limit:
 * out must hold sbe_encode_output_bound bytes).  nthreads > 1 uses OpenMP (two passes). */
int orc_encode_batch(const uint8_t* arena, const uint32_t* str_off, const uint32_t* str_len,
                     const uint64_t* timestamp, uint64_t n, uint64_t ts_default, uint32_t flags,
                     uint8_t* out, uint64_t* out_off, uint8_t* status, int nthreads);

/* Session-framed batch encode, the semantics/outputs of sbe_encode_session_batch. */
int orc_encode_session_batch(const uint8_t* arena, const uint32_t* str_off, const uint32_t* str_len,
                             const uint64_t* timestamp, uint64_t n, uint64_t ts_default, uint32_t flags,
                             int64_t leadership_term_id, int64_t cluster_session_id, uint8_t* out,
                             uint64_t* out_off, uint8_t* status, int nthreads);

/* Lite-template batch encode (201 / 202 / 301), the semantics/outputs of sbe_encode_lite_batch.
 * str_off / str_len are [n][nf].  Returns -1 for an unknown template. */
int orc_encode_lite_batch(const uint8_t* arena, const uint32_t* str_off, const uint32_t* str_len,
                          const uint32_t* topic_id, const uint64_t* sequence, uint64_t n,
                          uint32_t template_id, uint8_t* out, uint64_t* out_off, uint8_t* status,
                          int nthreads);

/* One record, MessageParser::parse_message (mode 0), MessageHandler::on_egress (mode 1) or the
 * Lite flyweight decode (mode 2).
 * Writes the descriptor fields of record slot 0 of the given arrays. */
void orc_decode_one(const uint8_t* rec, uint64_t len, uint32_t mode, uint8_t* status,
                    uint8_t* flags, uint16_t hdr[4], uint64_t* ts, uint32_t view_off[5],
                    uint32_t view_len[5]);

/* Batch decode: same outputs as sbe_decode_batch (host arrays). */
int orc_decode_batch(const uint8_t* in, const uint64_t* rec_off, uint64_t n, uint32_t mode,
                     uint8_t* status, uint8_t* flags, uint16_t* hdr, uint64_t* ts,
                     uint32_t* view_off, uint32_t* view_len, int nthreads);

/* Fragment reassembly with the semantics/outputs of sbe_reassemble_fragments (host arrays; out
 * and acc_buf hold frag_off[n] - frag_off[0] bytes, msg_off n + 1 entries). */
int orc_reassemble(const uint8_t* in, const uint64_t* frag_off, const uint8_t* flags, uint64_t n,
                   uint8_t* out, uint64_t* msg_off, uint64_t counts[2], uint8_t* acc_buf);

/* ParseResult.sequence_number of a payload (src/sbe_encoder.cpp:1031-1125 over jsoncpp 1.9.5's
 * CharReaderBuilder defaults; jsoncpp is absent here: PARITY UNPINNED, restated). */
uint64_t orc_seq_eval(const uint8_t* payload, uint64_t n);

/* sbe_eval_sequence_numbers over host arrays (the outputs of orc_decode_batch in parse mode). */
int orc_seq_batch(const uint8_t* in, const uint64_t* rec_off, uint64_t n, const uint8_t* status,
                  const uint8_t* flags, const uint32_t* view_off, const uint32_t* view_len, uint64_t* seq,
                  int nthreads);

/* Order::to_json (src/order_types.cpp:122-181) / publish_order headers JSON
 * (src/cluster_client.cpp:308-323) of one Order: fields s[0..7] as in sbe_order_batch.  Returns
 * the text length and writes it when out != NULL.  jsoncpp absent: PARITY UNPINNED, restated. */
uint64_t orc_order_json_one(const uint8_t* const s[8], const uint32_t len[8], int64_t customer_id,
                            int64_t timestamp, double quantity, uint32_t what, uint8_t* out);

/* sbe_order_to_json_batch over host arrays (out holds the whole text). */
int orc_order_json_batch(const uint8_t* arena, const uint32_t* str_off, const uint32_t* str_len,
                         const int64_t* customer_id, const int64_t* timestamp, const double* quantity,
                         uint64_t n, uint32_t what, uint8_t* out, uint64_t* out_off, int nthreads);

/* SBEDecoder::decode_session_event (src/sbe_encoder.cpp:183-238): 1 (true) / 0 (false); *got = 1
 * when the u32-prefixed detail was assigned, its bytes at rec[*off .. *off + *len). */
int orc_sbedecoder_session_event(const uint8_t* rec, uint64_t len, uint32_t* off, uint32_t* len_out, uint32_t* got);
/* SBEDecoder::decode_acknowledgment (:240-282): 1 / 0; *got bit k = string k (messageId, status,
 * error) assigned at rec[off[k] .. off[k] + slen[k]), bit 3 = *ts written. */
int orc_sbedecoder_ack(const uint8_t* rec, uint64_t len, uint32_t off[3], uint32_t slen[3], uint32_t* got, int64_t* ts);

/* protocol.hpp:37-42 */
uint64_t orc_to_nanos_auto(uint64_t ts);

#ifdef __cplusplus
}
#endif
#endif
