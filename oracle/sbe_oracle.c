/*
 * sbe_oracle.c — TEST INFRASTRUCTURE ONLY (see sbe_oracle.h).
 *
 * Plain-C restatement of the reference wire codec.  Every function cites the reference lines it
 * restates (paths relative to /root/reference).  Bounds are checked BEFORE any read (the
 * reference's getXAsString builds the string before its E100 check, TopicMessage.h:539-541;
 * that read is discarded on the throw, so checking first changes no output).
 */
#include "sbe_oracle.h"

#include <stdlib.h>
#include <string.h>
#ifdef _OPENMP
#include <omp.h>
#endif

static inline uint16_t rd16(const uint8_t* p) { return (uint16_t)(p[0] | (p[1] << 8)); }
static inline uint32_t rd32(const uint8_t* p) {
    return (uint32_t)p[0] | ((uint32_t)p[1] << 8) | ((uint32_t)p[2] << 16) | ((uint32_t)p[3] << 24);
}
static inline uint64_t rd64(const uint8_t* p) { return (uint64_t)rd32(p) | ((uint64_t)rd32(p + 4) << 32); }
static inline void wr16(uint8_t* p, uint16_t v) { p[0] = (uint8_t)v; p[1] = (uint8_t)(v >> 8); }
static inline void wr64(uint8_t* p, uint64_t v) {
    for (int i = 0; i < 8; ++i) p[i] = (uint8_t)(v >> (8 * i));
}

/* include/aeron_cluster/protocol.hpp:37-42 */
uint64_t orc_to_nanos_auto(uint64_t ts) { return ts < 100000000000000ULL ? ts * 1000000ULL : ts; }

/* ------------------------------------------------------------------------------------------
 * Encode.  SBEEncoder::encode_topic_message, src/sbe_encoder.cpp:131-167:
 *   computeLength() checks each field in wire order and throws E109 above 65534
 *   (TopicMessage.h:1382-1434); wrapAndApplyHeader writes {blockLength 16, templateId 1,
 *   schemaId 1, version 1} (TopicMessage.h:221-238); timestamp @+0, sequenceNumber(0) @+8
 *   (:362-374, :425-437); putX writes u16 LE length then the bytes (:515-529 ...);
 *   buffer.resize(encodedLength()) with encodedLength = position - m_offset and m_offset = 8
 *   (:281-284), i.e. the wire record minus its last 8 bytes.
 * ------------------------------------------------------------------------------------------ */
uint64_t orc_encode_one(const uint8_t* const s[5], const uint32_t len_in[5], uint64_t ts,
                        uint32_t flags, uint8_t* out, uint8_t* status) {
    /* SBE_ENC_PUBLISH_TOPIC: ClusterClient::publish_topic (src/cluster_client.cpp:1850-1854) calls
     * putX(const char*, int); the int converts to the std::uint16_t parameter (TopicMessage.h:515),
     * so length and copied bytes are L mod 65536 and computeLength (E109) is never called */
    const int pub = (flags & SBE_ENC_PUBLISH_TOPIC) != 0;
    uint32_t len[5];
    for (int f = 0; f < 5; ++f) len[f] = pub ? (len_in[f] & 0xffffu) : len_in[f];
    for (int f = 0; f < 5 && !pub; ++f) {
        if (len[f] > SBE_VAR_MAX_LEN) { /* TopicMessage.h:1396-1428 */
            if (status) *status = (uint8_t)(SBE_ENC_E109_TOPIC + f);
            return 0;
        }
    }
    uint64_t total = SBE_TM_WIRE_OVERHEAD;
    for (int f = 0; f < 5; ++f) total += len[f];
    uint64_t emit = (flags & SBE_ENC_REF_TRUNCATE8) ? total - 8 : total;
    /* build the wire record, then keep the first `emit` bytes */
    uint8_t head[24];
    wr16(head + 0, SBE_TM_BLOCK_LEN);
    wr16(head + 2, SBE_TM_TEMPLATE_ID);
    wr16(head + 4, SBE_TOPIC_SCHEMA_ID);
    wr16(head + 6, 1); /* schema version, TopicMessage.h:117 */
    wr64(head + 8, ts);
    wr64(head + 16, 0);
    uint64_t pos = 0;
#define PUT(src, n)                                        \
    do {                                                   \
        uint64_t n_ = (n);                                 \
        uint64_t k_ = pos + n_ <= emit ? n_ : emit - pos;  \
        if (pos < emit && k_) memcpy(out + pos, (src), k_); \
        pos += n_;                                         \
    } while (0)
    PUT(head, 24);
    for (int f = 0; f < 5; ++f) {
        uint8_t l2[2];
        wr16(l2, (uint16_t)len[f]);
        PUT(l2, 2);
        if (len[f]) PUT(s[f], len[f]);
    }
#undef PUT
    if (status) *status = SBE_ENC_OK;
    return emit;
}

/* One record of any layout: `lit` (nlit bytes: session header, SBE header, fixed block), then
 * nf u16-length-prefixed strings; the last `cut` bytes of the wire record are dropped
 * (REF_TRUNCATE8).  E109 on the first field above 65534 in wire order (computeLength). */
static uint64_t enc_record(const uint8_t* lit, uint32_t nlit, int nf, const uint8_t* const* s,
                           const uint32_t* len_in, uint32_t cut, int wrap16, uint8_t* out, uint8_t* status) {
    uint32_t len[5];
    for (int f = 0; f < nf; ++f) len[f] = wrap16 ? (len_in[f] & 0xffffu) : len_in[f];
    for (int f = 0; f < nf && !wrap16; ++f) {
        if (len[f] > SBE_VAR_MAX_LEN) {
            if (status) *status = (uint8_t)(SBE_ENC_E109_TOPIC + f);
            return 0;
        }
    }
    uint64_t total = nlit + 2u * (uint64_t)nf;
    for (int f = 0; f < nf; ++f) total += len[f];
    const uint64_t emit = total - cut;
    uint64_t pos = 0;
#define PUT(src, n)                                        \
    do {                                                   \
        uint64_t n_ = (n);                                 \
        uint64_t k_ = pos + n_ <= emit ? n_ : emit - pos;  \
        if (pos < emit && k_) memcpy(out + pos, (src), k_); \
        pos += n_;                                         \
    } while (0)
    PUT(lit, nlit);
    for (int f = 0; f < nf; ++f) {
        uint8_t l2[2];
        wr16(l2, (uint16_t)len[f]);
        PUT(l2, 2);
        if (len[f]) PUT(s[f], len[f]);
    }
#undef PUT
    if (status) *status = SBE_ENC_OK;
    return emit;
}

enum { LAY_TM = 0, LAY_TM_SESSION = 1, LAY_LITE = 2 };
typedef struct {
    int kind, nf;
    uint32_t cut, tmpl;
    int wrap16; /* SBE_ENC_PUBLISH_TOPIC: lengths mod 65536, no E109 (see orc_encode_one) */
    int64_t term, sess;
    uint64_t ts_default;
    const uint64_t* ts;   /* timestamp / sequence */
    const uint32_t* tid;
} layout_t;

/* the literal prefix of record i; returns its length */
static uint32_t lay_prefix(const layout_t* L, uint64_t i, uint8_t* lit) {
    uint32_t o = 0;
    if (L->kind == LAY_TM_SESSION) {
        /* SessionManager::Impl::create_session_message_header_buffer / update_session_header
         * (src/session_manager.cpp:936-967, :1018-1046), prepended by send_combined_message
         * (:1118-1144) */
        wr16(lit + 0, SBE_SESSION_BLOCK_LEN);
        wr16(lit + 2, SBE_SESSION_TEMPLATE_ID);
        wr16(lit + 4, SBE_CLUSTER_SCHEMA_ID);
        wr16(lit + 6, SBE_CLUSTER_SCHEMA_VERSION);
        wr64(lit + 8, (uint64_t)L->term);
        wr64(lit + 16, (uint64_t)L->sess);
        wr64(lit + 24, 0);
        o = 32;
    }
    if (L->kind == LAY_LITE) {
        /* wrapAndApplyHeader {12, T, 1, 1}; topicId @0, sequence @4 (src/commit_manager.cpp:120-124,
         * include/model/CommitOffsetLite.h:114-118, :337-420) */
        wr16(lit + 0, SBE_LITE_BLOCK_LEN);
        wr16(lit + 2, (uint16_t)L->tmpl);
        wr16(lit + 4, 1);
        wr16(lit + 6, 1);
        const uint32_t t = L->tid[i];
        lit[8] = (uint8_t)t; lit[9] = (uint8_t)(t >> 8); lit[10] = (uint8_t)(t >> 16); lit[11] = (uint8_t)(t >> 24);
        wr64(lit + 12, L->ts[i]);
        return 20;
    }
    /* TopicMessage: header {16,1,1,1}, timestamp (0 → the caller's clock), sequenceNumber 0 */
    wr16(lit + o + 0, SBE_TM_BLOCK_LEN);
    wr16(lit + o + 2, SBE_TM_TEMPLATE_ID);
    wr16(lit + o + 4, SBE_TOPIC_SCHEMA_ID);
    wr16(lit + o + 6, 1);
    wr64(lit + o + 8, L->ts[i] ? L->ts[i] : L->ts_default);
    wr64(lit + o + 16, 0);
    return o + 24;
}

static int encode_batch_lay(const layout_t* Ly, const uint8_t* arena, const uint32_t* str_off,
                            const uint32_t* str_len, uint64_t n, uint8_t* out, uint64_t* out_off,
                            uint8_t* status, int nthreads) {
    const int nf = Ly->nf;
    const uint64_t nlit = Ly->kind == LAY_LITE ? 20u : (Ly->kind == LAY_TM_SESSION ? 56u : 24u);
    const uint64_t ovh = nlit + 2u * (uint64_t)nf - Ly->cut;
    /* pass 1: record sizes (0 for E109) */
    uint64_t acc = 0;
    for (uint64_t i = 0; i < n; ++i) {
        const uint32_t* L = str_len + (uint64_t)nf * i;
        uint64_t sum = 0;
        int bad = 0;
        for (int f = 0; f < nf; ++f) {
            sum += Ly->wrap16 ? (L[f] & 0xffffu) : L[f];
            if (!Ly->wrap16 && L[f] > SBE_VAR_MAX_LEN) bad = 1;
        }
        out_off[i] = acc;
        acc += bad ? 0 : ovh + sum;
    }
    out_off[n] = acc;
    if (nthreads < 1) nthreads = 1;
    /* packed: string bytes of record i start at Σ_{j<i} Σlen_j (E109 records included).  Split
     * into nthreads contiguous chunks; each chunk first sums its predecessors' string bytes. */
    int nt = nthreads;
    uint64_t chunk = (n + (uint64_t)nt - 1) / (uint64_t)nt;
#ifdef _OPENMP
#pragma omp parallel for schedule(static, 1) num_threads(nt)
#endif
    for (int t = 0; t < nt; ++t) {
        uint64_t lo = (uint64_t)t * chunk, hi = lo + chunk < n ? lo + chunk : n;
        if (lo >= hi) continue;
        uint64_t ib = 0;
        if (!str_off)
            for (uint64_t j = 0; j < lo * (uint64_t)nf; ++j) ib += str_len[j];
        for (uint64_t i = lo; i < hi; ++i) {
            const uint32_t* L = str_len + (uint64_t)nf * i;
            const uint8_t* s[5];
            for (int f = 0; f < nf; ++f) {
                s[f] = arena + (str_off ? str_off[(uint64_t)nf * i + f] : ib);
                if (!str_off) ib += L[f];
            }
            uint8_t lit[64], st;
            const uint32_t nlit = lay_prefix(Ly, i, lit);
            enc_record(lit, nlit, nf, s, L, Ly->cut, Ly->wrap16, out + out_off[i], &st);
            if (status) status[i] = st;
        }
    }
    return 0;
}

int orc_encode_batch(const uint8_t* arena, const uint32_t* str_off, const uint32_t* str_len,
                     const uint64_t* timestamp, uint64_t n, uint64_t ts_default, uint32_t flags,
                     uint8_t* out, uint64_t* out_off, uint8_t* status, int nthreads) {
    if ((flags & SBE_ENC_PUBLISH_TOPIC) && (flags & SBE_ENC_REF_TRUNCATE8)) return -1;
    layout_t Ly = {LAY_TM, 5, (flags & SBE_ENC_REF_TRUNCATE8) ? 8u : 0u, 0, (flags & SBE_ENC_PUBLISH_TOPIC) != 0,
                   0, 0, ts_default, timestamp, NULL};
    return encode_batch_lay(&Ly, arena, str_off, str_len, n, out, out_off, status, nthreads);
}

int orc_encode_session_batch(const uint8_t* arena, const uint32_t* str_off, const uint32_t* str_len,
                             const uint64_t* timestamp, uint64_t n, uint64_t ts_default, uint32_t flags,
                             int64_t leadership_term_id, int64_t cluster_session_id, uint8_t* out,
                             uint64_t* out_off, uint8_t* status, int nthreads) {
    if (flags & SBE_ENC_PUBLISH_TOPIC) return -1;
    layout_t Ly = {LAY_TM_SESSION, 5, (flags & SBE_ENC_REF_TRUNCATE8) ? 8u : 0u, 0, 0,
                   leadership_term_id, cluster_session_id, ts_default, timestamp, NULL};
    return encode_batch_lay(&Ly, arena, str_off, str_len, n, out, out_off, status, nthreads);
}

static int lite_fields(uint32_t t) {
    return t == SBE_COMMIT_OFFSET_LITE_TEMPLATE_ID ? 2
         : (t == SBE_ORDER_REQUEST_LITE_TEMPLATE_ID || t == SBE_ORDER_NOTIFICATION_LITE_TEMPLATE_ID) ? 3 : 0;
}

int orc_encode_lite_batch(const uint8_t* arena, const uint32_t* str_off, const uint32_t* str_len,
                          const uint32_t* topic_id, const uint64_t* sequence, uint64_t n,
                          uint32_t template_id, uint8_t* out, uint64_t* out_off, uint8_t* status,
                          int nthreads) {
    const int nf = lite_fields(template_id);
    if (!nf) return -1;
    layout_t Ly = {LAY_LITE, nf, 0, template_id, 0, 0, 0, 0, sequence, topic_id};
    return encode_batch_lay(&Ly, arena, str_off, str_len, n, out, out_off, status, nthreads);
}

/* ------------------------------------------------------------------------------------------
 * Decode.  Descriptor conventions: see include/sbecodec.h (views relative to record start).
 * ------------------------------------------------------------------------------------------ */
typedef struct {
    uint8_t status, flags;
    uint16_t hdr[4]; /* block_length, template_id, schema_id, version */
    uint64_t ts;
    uint32_t off[5], len[5];
} desc_t;

static void set_view(desc_t* d, int k, uint64_t off, uint64_t len) {
    d->off[k] = (uint32_t)off;
    d->len[k] = (uint32_t)len;
}

static void fail(desc_t* d, uint8_t st, uint32_t param) {
    memset(d, 0, sizeof(*d));
    d->status = st;
    d->off[0] = param;
}

static void set_hdr(desc_t* d, const uint8_t* p) {
    d->hdr[0] = rd16(p + 0);
    d->hdr[1] = rd16(p + 2);
    d->hdr[2] = rd16(p + 4);
    d->hdr[3] = rd16(p + 6);
}

/* Does [p, p+n) contain "_sequence_number"?  With SBE_FL_SEQ_ESC, marks the payloads whose
 * sequence_number needs the JSON evaluation below (src/sbe_encoder.cpp:1031-1125). */
static int has_seq_key(const uint8_t* p, uint64_t n) {
    static const char key[] = "_sequence_number";
    const uint64_t k = sizeof(key) - 1;
    if (n < k) return 0;
    for (uint64_t i = 0; i + k <= n; ++i)
        if (p[i] == '_' && memcmp(p + i, key, k) == 0) return 1;
    return 0;
}

/* MessageParser::decode_topic_message_with_sbe, src/sbe_encoder.cpp:957-1143.
 * rec = embedded record at byte `base` of the original record. */
static void dec_tm_parse(const uint8_t* rec, uint64_t len, uint64_t base, desc_t* d) {
    /* MessageHeader::wrap(buf,0,0,len) cannot throw here: len >= 8 by dispatch (:521-526, :772) */
    const uint16_t blk = rd16(rec + 0), ver = rd16(rec + 6);
    /* template/schema are 1/1 by dispatch (:792, :814), so :976-983 never fails */
    /* wrapForDecode(buf, 8, blk, ver, len): sbeCheckPosition(8 + blk) (TopicMessage.h:240-254) */
    uint64_t pos = 8u + blk;
    if (pos > len) { fail(d, SBE_ST_ERR_TM_E100, 0); return; }
    desc_t r;
    memset(&r, 0, sizeof(r));
    /* getTopicAsString, getMessageTypeAsString, getUuidAsString, getPayloadAsString (:1006-1009):
     * sbePosition(pos+2) then sbePosition(pos+2+L), each throws E100 past len (:529-543) */
    for (int f = 0; f < 4; ++f) {
        if (pos + 2 > len) { fail(d, SBE_ST_ERR_TM_E100, 0); return; }
        uint64_t L = rd16(rec + pos);
        if (pos + 2 + L > len) { fail(d, SBE_ST_ERR_TM_E100, 0); return; }
        set_view(&r, f, base + pos + 2, L);
        pos += 2 + L;
    }
    r.status = SBE_ST_TM;
    r.hdr[0] = blk;  /* block_length = acting_block_length (:1025) */
    r.hdr[1] = 1;    /* template_id (:1022) */
    r.hdr[2] = 1;    /* schema_id (:1023) */
    r.hdr[3] = ver;  /* version = acting_version (:1024) */
    r.ts = rd64(rec + 8); /* in bounds: success implies len >= 16 + blk */
    if (base) r.flags |= SBE_FL_WRAPPED;
    if (has_seq_key(rec + (r.off[3] - base), r.len[3])) r.flags |= SBE_FL_SEQ_KEY;
    if (r.len[3] >= 16 && memchr(rec + (r.off[3] - base), '\\', r.len[3])) r.flags |= SBE_FL_SEQ_ESC;
    /* headers in their own try: E100 → headers = "" and success stays (:1127-1135) */
    if (pos + 2 > len || pos + 2 + (uint64_t)rd16(rec + pos) > len) {
        r.flags |= SBE_FL_HEADERS_E100;
    } else {
        uint64_t L = rd16(rec + pos);
        set_view(&r, 4, base + pos + 2, L);
    }
    *d = r;
}

/* MessageParser::decode_acknowledgment_with_sbe, src/sbe_encoder.cpp:833-954 */
static void dec_ack_heuristic(const uint8_t* rec, uint64_t len, uint64_t base, desc_t* d) {
    /* len < 8 ("Buffer too short for SBE header", :842-845) is unreachable: every caller has
     * already required 8 bytes (:521-526, :772).  template/schema are 2/1 by dispatch. */
    if (len < 16) { fail(d, SBE_ST_ERR_ACK_SHORT, (uint32_t)len); return; } /* :868-874 */
    desc_t r;
    memset(&r, 0, sizeof(r));
    set_hdr(&r, rec); /* :916-920 */
    r.status = SBE_ST_ACK;
    r.ts = rd64(rec + 8); /* :880 */
    if (base) r.flags |= SBE_FL_WRAPPED;
    /* maximal runs of bytes in [32,126] over [16,len); runs of >= 3 kept; first three
     * become message_id, payload, headers (:890-933) */
    int nruns = 0;
    uint64_t run_start = 0, run_len = 0;
    for (uint64_t i = 16; i < len && nruns < 3; ++i) {
        uint8_t c = rec[i];
        if (c >= 32 && c <= 126) {
            if (run_len == 0) run_start = i;
            ++run_len;
        } else {
            if (run_len >= 3) set_view(&r, nruns++, base + run_start, run_len);
            run_len = 0;
        }
    }
    if (nruns < 3 && run_len >= 3) set_view(&r, nruns++, base + run_start, run_len);
    if (nruns < 1) r.flags |= SBE_FL_ID_DEFAULT;      /* "ack_" + to_string(ts) (:936-938) */
    if (nruns < 2) r.flags |= SBE_FL_PAYLOAD_DEFAULT; /* "SUCCESS" (:939-941) */
    *d = r;
}

/* MessageParser::parse_session_event + SBEDecoder::decode_session_event,
 * src/sbe_encoder.cpp:618-647, :183-238, :285-318 */
static void dec_session_event(const uint8_t* rec, uint64_t len, desc_t* d) {
    if (len < 8 + 32) { fail(d, SBE_ST_ERR_SESSION_EVENT, 0); return; } /* :185-187 */
    desc_t r;
    memset(&r, 0, sizeof(r));
    r.status = SBE_ST_SESSION_EVENT;
    set_hdr(&r, rec); /* :639-644 */
    /* detail: u32-prefixed string at 40 if it fits (extract_variable_string :285-318) */
    uint64_t rem = len - 40;
    if (rem >= 4) {
        uint64_t L = rd32(rec + 40);
        if (!(L > rem - 4 || L > 10u * 1024u * 1024u) && L > 0) set_view(&r, 3, 44, L);
    }
    *d = r;
}

/* MessageParser::parse_topic_message, src/sbe_encoder.cpp:724-831 */
static void dec_topic_dispatch(const uint8_t* rec, uint64_t len, desc_t* d) {
    const uint16_t blk = rd16(rec + 0), tmpl = rd16(rec + 2), schema = rd16(rec + 4);
    if (schema == SBE_CLUSTER_SCHEMA_ID) {
        uint64_t shs = 8u + blk; /* :756 */
        if (len <= shs) { fail(d, SBE_ST_ERR_SESSION_SHORT, 0); return; }
        const uint8_t* emb = rec + shs;
        uint64_t elen = len - shs;
        if (elen < 8) { fail(d, SBE_ST_ERR_EMBEDDED_SHORT, 0); return; }
        uint16_t etmpl = rd16(emb + 2), eschema = rd16(emb + 4);
        if (eschema == 1) {
            if (etmpl == 1) { dec_tm_parse(emb, elen, shs, d); return; }
            if (etmpl == 2) { dec_ack_heuristic(emb, elen, shs, d); return; }
            fail(d, SBE_ST_ERR_EMBEDDED_TEMPLATE, etmpl);
            return;
        }
        fail(d, SBE_ST_ERR_EMBEDDED_SCHEMA, eschema);
        return;
    }
    /* schema == 1 here (parse_message only dispatches schema 1 or 111 to this function) */
    if (tmpl == 1) { dec_tm_parse(rec, len, 0, d); return; }
    if (tmpl == 2) { dec_ack_heuristic(rec, len, 0, d); return; }
    fail(d, SBE_ST_ERR_DIRECT_TEMPLATE, tmpl); /* :820-823 */
}

/* MessageParser::parse_message, src/sbe_encoder.cpp:513-551, with the ParseResult predicates
 * of include/aeron_cluster/sbe_messages.hpp:332-377 (message_type is still empty here, so the
 * string clauses of is_topic_message never fire). */
static void dec_parse_message(const uint8_t* rec, uint64_t len, desc_t* d) {
    if (!rec || len == 0) { fail(d, SBE_ST_ERR_NULL_EMPTY, 0); return; }
    if (len < 8) { fail(d, SBE_ST_ERR_HEADER, 0); return; } /* :174-181, :523-526 */
    const uint16_t tmpl = rd16(rec + 2), schema = rd16(rec + 4);
    if (tmpl == 2 && schema == SBE_CLUSTER_SCHEMA_ID) { dec_session_event(rec, len, d); return; }
    int is_topic = (tmpl == 1 && schema == 1) || (schema == SBE_CLUSTER_SCHEMA_ID && tmpl == 1) ||
                   (schema == 1 && tmpl == 2);
    if (is_topic) { dec_topic_dispatch(rec, len, d); return; }
    /* is_acknowledgment() (2/1) is covered by the third is_topic clause: never reached */
    fail(d, SBE_ST_ERR_UNKNOWN_TYPE, 0); /* :546-549, header fields kept */
    set_hdr(d, rec);
}

/* decode_ack, src/ack_decoder.cpp:29-105.  Returns 1 and fills d on success. */
static int dec_ack_full(const uint8_t* rec, uint64_t len, desc_t* d) {
    if (len < 8) return 0;
    const uint16_t blk = rd16(rec + 0), tmpl = rd16(rec + 2), schema = rd16(rec + 4);
    if (schema != 1 || tmpl != 2) return 0; /* :40-42 */
    desc_t r;
    memset(&r, 0, sizeof(r));
    set_hdr(&r, rec);
    if (len == 16 && blk == 8) { /* simple control ack :46-52 */
        r.status = SBE_ST_EG_ACK_SIMPLE;
        r.ts = orc_to_nanos_auto(rd64(rec + 8));
        *d = r;
        return 1;
    }
    /* Acknowledgment::wrapForDecode(data, 8, blk, ver, len - 8): the "len-8 bug" (:67) */
    const uint64_t lim = len - 8;
    uint64_t pos = 8u + blk;
    if (pos > lim) return 0;
    /* getXLength() peeks the u16 at the position (in bounds: pos <= len-8); getX() is called
     * only for a non-zero length and then advances past 2+L with E100 checks (:71-96,
     * Acknowledgment.h:410-450); a zero length leaves the position where it was. */
    for (int f = 0; f < 3; ++f) {
        uint64_t L = rd16(rec + pos);
        if (L > 0) {
            if (pos + 2 + L > lim) return 0; /* E100 → catch(...) → nullopt (:99-101) */
            set_view(&r, f, pos + 2, L);
            pos += 2 + L;
        }
    }
    r.status = SBE_ST_EG_ACK;
    r.ts = orc_to_nanos_auto(rd64(rec + 8)); /* len >= 16 + blk here */
    *d = r;
    return 1;
}

/* MessageHandler::on_egress, include/aeron_cluster/message_handler.hpp:35-68 */
static void dec_on_egress(const uint8_t* rec, uint64_t len, desc_t* d) {
    memset(d, 0, sizeof(*d));
    if (!rec || len < 8) { d->status = SBE_ST_EG_NONE; return; }
    if (dec_ack_full(rec, len, d)) return;
    const uint16_t blk = rd16(rec + 0), tmpl = rd16(rec + 2), schema = rd16(rec + 4);
    set_hdr(d, rec);
    if (!(tmpl == 1 && schema == 1)) { d->status = SBE_ST_EG_NONE; return; } /* :74-79 */
    /* TopicMessage::wrapForDecode(data, 8, blk, ver, len - 8) — no try/catch: E100 escapes */
    const uint64_t lim = len - 8;
    uint64_t pos = 8u + blk;
    if (pos > lim) { d->status = SBE_ST_EG_THROW_E100; return; }
    /* read_var_string: xLength() peek; getter only if len > 0 (:81-89) */
    for (int f = 0; f < 5; ++f) {
        uint64_t L = rd16(rec + pos);
        if (L > 0) {
            if (pos + 2 + L > lim) {
                memset(d->off, 0, sizeof d->off);
                memset(d->len, 0, sizeof d->len);
                d->status = SBE_ST_EG_THROW_E100;
                return;
            }
            set_view(d, f, pos + 2, L);
            pos += 2 + L;
        }
    }
    if (d->len[0] == 0) { /* empty topic → return (:63) */
        memset(d->off, 0, sizeof d->off);
        memset(d->len, 0, sizeof d->len);
        d->status = SBE_ST_EG_NONE;
        return;
    }
    d->status = SBE_ST_EG_TM;
}

/* The Lite templates' generated decode flyweights, in field order: MessageHeader::wrap,
 * wrapForDecode(buf, 8, blockLength, version, len) → sbeCheckPosition(8 + blockLength)
 * (CommitOffsetLite.h:240-254, :268-276), topicId() @8, sequence() @12 (:337-420: no bounds
 * check; records shorter than 20 B would read past the buffer, reported as E100 here), then
 * getXAsString() per var field: sbePosition(pos + 2), then sbePosition(pos + 2 + L)
 * (:528-540), each throwing "buffer too short [E100]" past len. */
static void dec_lite(const uint8_t* rec, uint64_t len, desc_t* d) {
    memset(d, 0, sizeof(*d));
    if (!rec || len < 8) { d->status = SBE_ST_LITE_NOT_LITE; return; }
    set_hdr(d, rec);
    const uint16_t blk = rd16(rec + 0), tmpl = rd16(rec + 2), schema = rd16(rec + 4);
    const int nf = lite_fields(tmpl);
    if (schema != 1 || !nf) { d->status = SBE_ST_LITE_NOT_LITE; return; }
    uint64_t pos = 8u + blk;
    if (pos > len || len < 20) { d->status = SBE_ST_LITE_E100; return; }
    for (int f = 0; f < nf; ++f) {
        if (pos + 2 > len) { memset(d->off, 0, sizeof d->off); memset(d->len, 0, sizeof d->len);
                             d->status = SBE_ST_LITE_E100; return; }
        const uint64_t L = rd16(rec + pos);
        pos += 2;
        if (pos + L > len) { memset(d->off, 0, sizeof d->off); memset(d->len, 0, sizeof d->len);
                             d->status = SBE_ST_LITE_E100; return; }
        set_view(d, f, pos, L);
        pos += L;
    }
    d->status = SBE_ST_LITE;
    d->ts = rd64(rec + 12);
    d->off[4] = rd32(rec + 8);
}

static void decode_into(const uint8_t* rec, uint64_t len, uint32_t mode, desc_t* d) {
    if (mode == SBE_DEC_LITE)
        dec_lite(rec, len, d);
    else if (mode == SBE_DEC_ON_EGRESS)
        dec_on_egress(rec, len, d);
    else
        dec_parse_message(rec, len, d);
}

void orc_decode_one(const uint8_t* rec, uint64_t len, uint32_t mode, uint8_t* status,
                    uint8_t* flags, uint16_t hdr[4], uint64_t* ts, uint32_t view_off[5],
                    uint32_t view_len[5]) {
    desc_t d;
    decode_into(rec, len, mode, &d);
    *status = d.status;
    *flags = d.flags;
    memcpy(hdr, d.hdr, sizeof d.hdr);
    *ts = d.ts;
    memcpy(view_off, d.off, sizeof d.off);
    memcpy(view_len, d.len, sizeof d.len);
}

int orc_decode_batch(const uint8_t* in, const uint64_t* rec_off, uint64_t n, uint32_t mode,
                     uint8_t* status, uint8_t* flags, uint16_t* hdr, uint64_t* ts,
                     uint32_t* view_off, uint32_t* view_len, int nthreads) {
    if (nthreads < 1) nthreads = 1;
#ifdef _OPENMP
#pragma omp parallel for schedule(static) num_threads(nthreads)
#endif
    for (int64_t i = 0; i < (int64_t)n; ++i) {
        desc_t d;
        uint64_t a = rec_off[i], b = rec_off[i + 1];
        decode_into(b > a ? in + a : NULL, b - a, mode, &d);
        status[i] = d.status;
        flags[i] = d.flags;
        memcpy(hdr + 4 * i, d.hdr, sizeof d.hdr);
        ts[i] = d.ts;
        memcpy(view_off + 5 * i, d.off, sizeof d.off);
        memcpy(view_len + 5 * i, d.len, sizeof d.len);
    }
    return 0;
}

/* ------------------------------------------------------------------------------------------
 * Aeron fragment reassembly: LocalFragmentReassembler::onFragment, src/cluster_client.cpp:39-82,
 * one call per fragment in order:
 *   BEGIN|END (0xC0)     deliver the fragment itself (the accumulator is untouched, :52-56);
 *   otherwise            BEGIN clears the accumulator (:59-62), the fragment is appended (:63),
 *                        END delivers the accumulator and clears it (:66-73).
 * Outputs as sbe_reassemble_fragments: messages back to back, msg_off[0..m], then the open
 * accumulator ("carry") right after the last message; counts = {m, carry bytes}.
 * ------------------------------------------------------------------------------------------ */
int orc_reassemble(const uint8_t* in, const uint64_t* frag_off, const uint8_t* flags, uint64_t n,
                   uint8_t* out, uint64_t* msg_off, uint64_t counts[2], uint8_t* acc_buf) {
    uint64_t m = 0, at = 0, acc = 0;
    msg_off[0] = 0;
    for (uint64_t i = 0; i < n; ++i) {
        const uint8_t f = flags[i];
        const uint8_t* src = in + frag_off[i];
        const uint64_t len = frag_off[i + 1] - frag_off[i];
        if ((f & (SBE_FRAG_BEGIN | SBE_FRAG_END)) == (SBE_FRAG_BEGIN | SBE_FRAG_END)) {
            memcpy(out + at, src, len);
            at += len;
            msg_off[++m] = at;
            continue;
        }
        if (f & SBE_FRAG_BEGIN) acc = 0;
        memcpy(acc_buf + acc, src, len);
        acc += len;
        if (f & SBE_FRAG_END) {
            memcpy(out + at, acc_buf, acc);
            at += acc;
            msg_off[++m] = at;
            acc = 0;
        }
    }
    memcpy(out + at, acc_buf, acc);
    counts[0] = m;
    counts[1] = acc;
    return 0;
}

/* ------------------------------------------------------------------------------------------
 * ParseResult.sequence_number (src/sbe_encoder.cpp:1031-1125): parse the payload with jsoncpp's
 * CharReaderBuilder defaults (jsoncpp 1.9: comments allowed, trailing commas allowed, extra
 * content after the root ignored, no single quotes / numeric keys / special floats, stack limit
 * 1000; OurReader's tokenizer: a NUL byte outside a string ends the stream), then look up
 * "_sequence_number" in the root object, root.message, root.message.message and
 * root.message.message.message, first value > 0 wins (extractSequence: UInt64, Int64, other
 * numbers through double, strings through std::stoull, else 0).  Any parse failure or exception
 * gives 0.  jsoncpp is absent from this image: PARITY UNPINNED (restated from its published
 * algorithm; decimal → double is exact only on the Clinger fast path, ≤ 19 significant digits).
 * ------------------------------------------------------------------------------------------ */
typedef struct {
    const uint8_t* p;
    uint64_t n, i;
} jcur;

enum { JT_OBEG, JT_OEND, JT_ABEG, JT_AEND, JT_STR, JT_NUM, JT_TRUE, JT_FALSE, JT_NULL, JT_COMMA, JT_COLON,
       JT_COMMENT, JT_EOS, JT_ERR };

static int jc_get(jcur* c) { return c->i < c->n ? c->p[c->i++] : 0; }

static void jc_skip_spaces(jcur* c) {
    while (c->i < c->n) {
        const uint8_t ch = c->p[c->i];
        if (ch == ' ' || ch == '\t' || ch == '\r' || ch == '\n') ++c->i;
        else break;
    }
}

/* OurReader::readToken; *s, *e: the token's bytes */
static int jc_token(jcur* c, uint64_t* s, uint64_t* e) {
    jc_skip_spaces(c);
    *s = c->i;
    const int ch = jc_get(c);
    int t = JT_ERR;
    switch (ch) {
        case '{': t = JT_OBEG; break;
        case '}': t = JT_OEND; break;
        case '[': t = JT_ABEG; break;
        case ']': t = JT_AEND; break;
        case ',': t = JT_COMMA; break;
        case ':': t = JT_COLON; break;
        case 0: t = JT_EOS; break;
        case '"': { /* readString: to the next unescaped quote */
            int q = 0;
            while (c->i < c->n) {
                const int x = jc_get(c);
                if (x == '\\') jc_get(c);
                else if (x == '"') { q = 1; break; }
            }
            t = q ? JT_STR : JT_ERR;
            break;
        }
        case '/': { /* readComment */
            const int x = jc_get(c);
            if (x == '*') { /* readCStyleComment: stops one byte early, then needs '/' */
                int ok = 0;
                while (c->i + 1 < c->n) {
                    const int y = jc_get(c);
                    if (y == '*' && c->p[c->i] == '/') break;
                }
                ok = jc_get(c) == '/';
                t = ok ? JT_COMMENT : JT_ERR;
            } else if (x == '/') {
                while (c->i < c->n) {
                    const int y = jc_get(c);
                    if (y == '\n') break;
                    if (y == '\r') { if (c->i < c->n && c->p[c->i] == '\n') ++c->i; break; }
                }
                t = JT_COMMENT;
            } else {
                t = JT_ERR;
            }
            break;
        }
        case 't': t = (c->n - c->i >= 3 && memcmp(c->p + c->i, "rue", 3) == 0) ? (c->i += 3, JT_TRUE) : JT_ERR; break;
        case 'f': t = (c->n - c->i >= 4 && memcmp(c->p + c->i, "alse", 4) == 0) ? (c->i += 4, JT_FALSE) : JT_ERR; break;
        case 'n': t = (c->n - c->i >= 3 && memcmp(c->p + c->i, "ull", 3) == 0) ? (c->i += 3, JT_NULL) : JT_ERR; break;
        default:
            if (ch == '-' && c->i < c->n && c->p[c->i] == 'I') { /* readNumber(checkInf): -Infinity, not allowed */
                ++c->i;
                t = JT_ERR;
            } else if ((ch >= '0' && ch <= '9') || ch == '-') { /* readNumber */
                uint64_t k = c->i;
                int x = '0';
#define NX() (x = (c->i = k) < c->n ? c->p[k++] : 0)
                while (x >= '0' && x <= '9') NX();
                if (x == '.') { NX(); while (x >= '0' && x <= '9') NX(); }
                if (x == 'e' || x == 'E') { NX(); if (x == '+' || x == '-') NX(); while (x >= '0' && x <= '9') NX(); }
#undef NX
                t = JT_NUM;
            }
            break;
    }
    *e = c->i;
    return t;
}

/* Reader::decodeString into out (up to cap bytes kept; *len = full decoded length); 0 on error */
static void jc_utf8(uint32_t cp, uint8_t* out, uint64_t cap, uint64_t* len) {
    uint8_t b[4];
    int k = 0;
    if (cp <= 0x7f) b[k++] = (uint8_t)cp;
    else if (cp <= 0x7ff) { b[k++] = (uint8_t)(0xc0 | (cp >> 6)); b[k++] = (uint8_t)(0x80 | (cp & 0x3f)); }
    else if (cp <= 0xffff) { b[k++] = (uint8_t)(0xe0 | (cp >> 12)); b[k++] = (uint8_t)(0x80 | ((cp >> 6) & 0x3f)); b[k++] = (uint8_t)(0x80 | (cp & 0x3f)); }
    else if (cp <= 0x10ffff) { b[k++] = (uint8_t)(0xf0 | (cp >> 18)); b[k++] = (uint8_t)(0x80 | ((cp >> 12) & 0x3f)); b[k++] = (uint8_t)(0x80 | ((cp >> 6) & 0x3f)); b[k++] = (uint8_t)(0x80 | (cp & 0x3f)); }
    for (int j = 0; j < k; ++j) { if (*len < cap) out[*len] = b[j]; ++*len; }
}
static int jc_hex4(const uint8_t* p, uint64_t avail, uint32_t* v) {
    if (avail < 4) return 0;
    uint32_t r = 0;
    for (int j = 0; j < 4; ++j) {
        const uint8_t h = p[j];
        r <<= 4;
        if (h >= '0' && h <= '9') r |= h - '0';
        else if (h >= 'a' && h <= 'f') r |= h - 'a' + 10;
        else if (h >= 'A' && h <= 'F') r |= h - 'A' + 10;
        else return 0;
    }
    *v = r;
    return 1;
}
static int jc_decode_string(const uint8_t* p, uint64_t s, uint64_t e, uint8_t* out, uint64_t cap, uint64_t* len) {
    *len = 0;
    uint64_t i = s + 1, end = e - 1; /* inside the quotes */
    while (i < end) {
        const uint8_t ch = p[i++];
        if (ch == '"') break;
        if (ch == '\\') {
            if (i == end) return 0; /* "Empty escape sequence in string" */
            const uint8_t x = p[i++];
            uint8_t o = 0;
            switch (x) {
                case '"': o = '"'; break;
                case '/': o = '/'; break;
                case '\\': o = '\\'; break;
                case 'b': o = '\b'; break;
                case 'f': o = '\f'; break;
                case 'n': o = '\n'; break;
                case 'r': o = '\r'; break;
                case 't': o = '\t'; break;
                case 'u': {
                    uint32_t cp;
                    if (!jc_hex4(p + i, end - i, &cp)) return 0;
                    i += 4;
                    if (cp >= 0xD800 && cp <= 0xDBFF) { /* surrogate pair: another \uXXXX must follow */
                        if (end - i < 6) return 0;
                        if (p[i] != '\\' || p[i + 1] != 'u') return 0;
                        uint32_t lo;
                        if (!jc_hex4(p + i + 2, end - i - 2, &lo)) return 0;
                        i += 6;
                        cp = 0x10000 + ((cp & 0x3FF) << 10) + (lo & 0x3FF);
                    }
                    jc_utf8(cp, out, cap, len);
                    continue;
                }
                default: return 0; /* "Bad escape sequence in string" */
            }
            if (*len < cap) out[*len] = o;
            ++*len;
        } else {
            if (*len < cap) out[*len] = ch;
            ++*len;
        }
    }
    return 1;
}

/* decoded value of one number token: kind 1 int64, 2 uint64, 3 double; 0 on error */
static int jc_decode_number(const uint8_t* p, uint64_t s, uint64_t e, int64_t* iv, uint64_t* uv, double* dv) {
    uint64_t i = s;
    const int neg = p[i] == '-';
    if (neg) ++i;
    const uint64_t maxv = neg ? (uint64_t)1 << 63 : ~0ull;
    const uint64_t thr = maxv / 10, lastd = maxv % 10;
    uint64_t v = 0;
    int dbl = 0;
    for (; i < e; ++i) {
        const uint8_t ch = p[i];
        if (ch < '0' || ch > '9') { dbl = 1; break; }
        const uint64_t dg = ch - '0';
        if (v >= thr && (v > thr || i + 1 != e || dg > lastd)) { dbl = 1; break; }
        v = v * 10 + dg;
    }
    if (!dbl) {
        if (neg) { *iv = (int64_t)(0 - v); return 1; }
        if (v <= (uint64_t)INT64_MAX) { *iv = (int64_t)v; return 1; }
        *uv = v;
        return 2;
    }
    /* decodeDouble: istringstream >> double over the token.  libstdc++'s num_get hands the
     * accumulated characters to strtod and fails unless all of them convert; an overflow
     * (±HUGE_VAL) becomes ±max with failbit, which jsoncpp turns back into ±infinity.  The token
     * grammar (readNumber) admits only digits, '-', '.', 'e', 'E', '+', so strtod over the whole
     * token is the same conversion (glibc strtod is correctly rounded). */
    char sbuf[128];
    const uint64_t tl = e - s;
    char* tb = tl < sizeof sbuf ? sbuf : (char*)malloc(tl + 1);
    if (!tb) return 0;
    memcpy(tb, p + s, tl);
    tb[tl] = 0;
    char* endp = NULL;
    const double d = strtod(tb, &endp);
    const int full = endp == tb + tl && tl > 0;
    if (tb != sbuf) free(tb);
    if (!full) return 0; /* "'...' is not a number." */
    *dv = d;
    return 3;
}

/* extractSequence on a realValue d (jsoncpp 1.9.5 json_value.cpp): isUInt64 (integral, 0 <= d < 2^64)
 * → asUInt64; isInt64 (integral, -2^63 <= d < 2^63) → asInt64; else static_cast<uint64_t>(asDouble())
 * as x86-64 gcc compiles it: d < 2^63 → cvttsd2si(d), else cvttsd2si(d - 2^63) ^ 2^63, where
 * cvttsd2si gives 0x8000000000000000 out of range (so d >= 2^64, +inf included, gives 0). */
static uint64_t jc_real_seq(double d) {
    if (d != d) return 0x8000000000000000ull;
    if (d >= 18446744073709551616.0) return 0;
    if (d >= 9223372036854775808.0) return (uint64_t)d; /* integral: exact */
    if (d < -9223372036854775808.0) return 0x8000000000000000ull;
    return (uint64_t)(int64_t)d; /* truncation toward zero */
}

/* std::stoull(s) (base 10) with 0 for the exceptions the reference catches */
static uint64_t jc_stoull(const uint8_t* s, uint64_t n) {
    uint64_t i = 0;
    while (i < n && (s[i] == ' ' || (s[i] >= 9 && s[i] <= 13))) ++i;
    if (i < n && s[i] == 0) return 0;
    int neg = 0;
    if (i < n && (s[i] == '+' || s[i] == '-')) { neg = s[i] == '-'; ++i; }
    uint64_t v = 0;
    int any = 0, ovf = 0;
    for (; i < n && s[i] >= '0' && s[i] <= '9'; ++i) {
        any = 1;
        const uint64_t dg = s[i] - '0';
        if (v > (~0ull - dg) / 10) ovf = 1;
        else v = v * 10 + dg;
    }
    if (!any || ovf) return 0; /* invalid_argument / out_of_range */
    return neg ? 0 - v : v;
}

#define J_MAX_DEPTH 1000
#define J_KEYCAP 32
uint64_t orc_seq_eval(const uint8_t* p, uint64_t n) {
    jcur c = {p, n, 0};
    if (n >= 3 && p[0] == 0xEF && p[1] == 0xBB && p[2] == 0xBF) c.i = 3; /* skipBom (jsoncpp 1.9.5) */
    uint8_t stk[J_MAX_DEPTH + 2]; /* 1 object, 2 array */
    int depth = 0;                /* containers open */
    int chain = 0;                /* containers [0, chain) are the root / message chain objects */
    uint64_t res[4] = {0, 0, 0, 0};
    int hobj[4] = {0, 0, 0, 0};
    int root_obj = 0;
    /* the member whose value comes next: 0 other, 1 "_sequence_number", 2 "message" (of a chain object) */
    int pend_kind = 0, pend_level = 0;
    uint64_t s, e;
    int t;
    enum { S_VALUE, S_KEY, S_COLON, S_OAFTER, S_AFIRST, S_AAFTER } st = S_VALUE;
    for (;;) {
        if (st == S_VALUE || st == S_AFIRST) {
            if (st == S_AFIRST) { /* readArray: ']' right after '[' or a ',' (spaces only) */
                jc_skip_spaces(&c);
                if (c.i < c.n && c.p[c.i] == ']') {
                    ++c.i;
                    --depth;
                    goto value_done;
                }
            }
            if (depth >= J_MAX_DEPTH) return 0; /* "Exceeded stackLimit in readValue()" */
            do t = jc_token(&c, &s, &e); while (t == JT_COMMENT);
            const int kind = pend_kind, level = pend_level;
            pend_kind = 0;
            switch (t) {
                case JT_OBEG:
                    stk[depth++] = 1;
                    if (depth == 1) { root_obj = 1; chain = 1; }
                    else if (kind == 2 && depth - 1 == level + 1 && chain == level + 1) { chain = depth; hobj[level + 1] = 1; }
                    if (kind == 1) res[level] = 0;
                    st = S_KEY;
                    continue;
                case JT_ABEG:
                    stk[depth++] = 2;
                    if (kind == 1) res[level] = 0;
                    st = S_AFIRST;
                    continue;
                case JT_NUM: {
                    int64_t iv = 0;
                    uint64_t uv = 0;
                    double dv = 0;
                    const int k = jc_decode_number(c.p, s, e, &iv, &uv, &dv);
                    if (!k) return 0;
                    if (kind == 1) {
                        if (k == 1) res[level] = (uint64_t)iv; /* isUInt64 / isInt64 */
                        else if (k == 2) res[level] = uv;
                        else res[level] = jc_real_seq(dv);
                    }
                    break;
                }
                case JT_STR: {
                    uint8_t buf[64];
                    uint64_t len;
                    if (!jc_decode_string(c.p, s, e, buf, sizeof buf, &len)) return 0;
                    if (kind == 1) {
                        /* c_str(): stops at an embedded NUL */
                        uint64_t m = len < sizeof buf ? len : sizeof buf;
                        for (uint64_t j = 0; j < m; ++j) if (buf[j] == 0) { m = j; break; }
                        res[level] = len <= sizeof buf ? jc_stoull(buf, m) : 0;
                        if (len > sizeof buf) { /* long strings: decode fully (rare) */
                            uint8_t* big = (uint8_t*)__builtin_alloca(len);
                            jc_decode_string(c.p, s, e, big, len, &len);
                            uint64_t mm = len;
                            for (uint64_t j = 0; j < len; ++j) if (big[j] == 0) { mm = j; break; }
                            res[level] = jc_stoull(big, mm);
                        }
                    }
                    break;
                }
                case JT_TRUE: case JT_FALSE: case JT_NULL:
                    if (kind == 1) res[level] = 0;
                    break;
                default:
                    return 0; /* "Syntax error: value, object or array expected." */
            }
        value_done:
            if (depth == 0) break; /* root done: extra content is ignored */
            st = stk[depth - 1] == 1 ? S_OAFTER : S_AAFTER;
            continue;
        }
        if (st == S_KEY) { /* key or '}' (empty object or trailing comma) */
            do t = jc_token(&c, &s, &e); while (t == JT_COMMENT);
            if (t == JT_OEND) {
                if (depth == chain) chain = depth - 1;
                --depth;
                goto value_done;
            }
            if (t != JT_STR) return 0;
            uint8_t key[J_KEYCAP];
            uint64_t klen;
            if (!jc_decode_string(c.p, s, e, key, J_KEYCAP, &klen)) return 0;
            if (depth == chain && depth <= 4) {
                const int level = depth - 1;
                if (klen == 16 && memcmp(key, "_sequence_number", 16) == 0) { pend_kind = 1; pend_level = level; }
                else if (klen == 7 && memcmp(key, "message", 7) == 0 && level < 3) {
                    pend_kind = 2;
                    pend_level = level;
                    for (int k = level + 1; k < 4; ++k) { res[k] = 0; hobj[k] = 0; }
                }
            }
            do t = jc_token(&c, &s, &e); while (0);
            if (t != JT_COLON) return 0; /* "Missing ':' after object member name" */
            st = S_VALUE;
            continue;
        }
        if (st == S_OAFTER) {
            t = jc_token(&c, &s, &e);
            if (t != JT_OEND && t != JT_COMMA && t != JT_COMMENT) return 0;
            if (t == JT_COMMENT) { /* after comments, the next token is taken as the separator */
                while (t == JT_COMMENT) t = jc_token(&c, &s, &e);
                if (t == JT_ERR && s == e) return 0;
            }
            if (t == JT_OEND) {
                if (depth == chain) chain = depth - 1;
                --depth;
                goto value_done;
            }
            st = S_KEY;
            continue;
        }
        if (st == S_AAFTER) {
            do t = jc_token(&c, &s, &e); while (t == JT_COMMENT);
            if (t == JT_AEND) { --depth; goto value_done; }
            if (t != JT_COMMA) return 0; /* "Missing ',' or ']' in array declaration" */
            st = S_AFIRST;
            continue;
        }
    }
    if (!root_obj) return 0; /* isMember on a non-object root throws (or is false for null) */
    if (res[0]) return res[0];
    for (int k = 1; k < 4; ++k) {
        if (!hobj[k]) break;
        if (res[k]) return res[k];
    }
    return 0;
}

int orc_seq_batch(const uint8_t* in, const uint64_t* rec_off, uint64_t n, const uint8_t* status,
                  const uint8_t* flags, const uint32_t* view_off, const uint32_t* view_len, uint64_t* seq,
                  int nthreads) {
    if (nthreads < 1) nthreads = 1;
#ifdef _OPENMP
#pragma omp parallel for schedule(dynamic, 64) num_threads(nthreads)
#endif
    for (int64_t i = 0; i < (int64_t)n; ++i) {
        if (status[i] != SBE_ST_TM || !(flags[i] & (SBE_FL_SEQ_KEY | SBE_FL_SEQ_ESC))) continue;
        seq[i] = orc_seq_eval(in + rec_off[i] + view_off[5 * i + 3], view_len[5 * i + 3]);
    }
    return 0;
}

/* ------------------------------------------------------------------------------------------
 * Order JSON: Order::to_json (src/order_types.cpp:122-181) and publish_order's headers JSON
 * (src/cluster_client.cpp:308-323).  Both go through jsoncpp's StreamWriterBuilder with
 * indentation "" (compact: no newlines, colon ":"), whose object members come out in std::map
 * order (Value::CZString::operator<: memcmp of the common prefix, then the shorter first).
 * jsoncpp 1.9.5 is absent here: the writer logic below is restated from its published source
 * (PARITY UNPINNED against jsoncpp itself); the number text is glibc snprintf, the same
 * function jsoncpp (valueToString) and libstdc++ (std::to_string) call.
 * ------------------------------------------------------------------------------------------ */
#include <math.h>
#include <stdio.h>

typedef struct {
    uint8_t* out; /* NULL: count only */
    uint64_t n;
} jw;

static void jw_put(jw* w, const char* s, uint64_t n) {
    if (w->out) memcpy(w->out + w->n, s, n);
    w->n += n;
}
static void jw_lit(jw* w, const char* s) { jw_put(w, s, strlen(s)); }

/* jsoncpp json_writer.cpp utf8ToCodepoint: lead byte decides the length, continuation bytes
 * are not checked, overlong / surrogate / truncated → U+FFFD (a truncated one consumes 1 byte). */
static uint32_t orc_utf8_cp(const uint8_t** s, const uint8_t* e) {
    const uint8_t* p = *s;
    uint32_t b = p[0], c;
    if (b < 0x80) return b;
    if (b < 0xE0) {
        if (e - p < 2) return 0xFFFD;
        c = ((b & 0x1F) << 6) | (p[1] & 0x3F);
        *s = p + 1;
        return c < 0x80 ? 0xFFFD : c;
    }
    if (b < 0xF0) {
        if (e - p < 3) return 0xFFFD;
        c = ((b & 0x0F) << 12) | ((uint32_t)(p[1] & 0x3F) << 6) | (p[2] & 0x3F);
        *s = p + 2;
        if (c >= 0xD800 && c <= 0xDFFF) return 0xFFFD;
        return c < 0x800 ? 0xFFFD : c;
    }
    if (b < 0xF8) {
        if (e - p < 4) return 0xFFFD;
        c = ((b & 0x07) << 18) | ((uint32_t)(p[1] & 0x3F) << 12) | ((uint32_t)(p[2] & 0x3F) << 6) | (p[3] & 0x3F);
        *s = p + 3;
        return c < 0x10000 ? 0xFFFD : c;
    }
    return 0xFFFD;
}

static void jw_hex(jw* w, uint32_t v) { /* appendHex: "\\u" + 4 lower-case hex digits */
    static const char hx[] = "0123456789abcdef";
    char b[6] = {'\\', 'u', hx[(v >> 12) & 15], hx[(v >> 8) & 15], hx[(v >> 4) & 15], hx[v & 15]};
    jw_put(w, b, 6);
}

/* jsoncpp valueToQuotedStringN(str, len, emitUTF8=false) */
static void jw_quoted(jw* w, const uint8_t* s, uint64_t n) {
    const uint8_t* e = s + n;
    jw_put(w, "\"", 1);
    for (const uint8_t* c = s; c < e; ++c) {
        switch (*c) {
            case '"': jw_put(w, "\\\"", 2); break;
            case '\\': jw_put(w, "\\\\", 2); break;
            case '\b': jw_put(w, "\\b", 2); break;
            case '\f': jw_put(w, "\\f", 2); break;
            case '\n': jw_put(w, "\\n", 2); break;
            case '\r': jw_put(w, "\\r", 2); break;
            case '\t': jw_put(w, "\\t", 2); break;
            default: {
                uint32_t cp = orc_utf8_cp(&c, e);
                if (cp < 0x20) jw_hex(w, cp);
                else if (cp < 0x80) { char ch = (char)cp; jw_put(w, &ch, 1); }
                else if (cp < 0x10000) jw_hex(w, cp);
                else {
                    cp -= 0x10000;
                    jw_hex(w, 0xD800 + ((cp >> 10) & 0x3FF));
                    jw_hex(w, 0xDC00 + (cp & 0x3FF));
                }
            }
        }
    }
    jw_put(w, "\"", 1);
}

static void jw_key(jw* w, const char* k) { /* "key": (keys here need no escaping) */
    jw_put(w, "\"", 1);
    jw_lit(w, k);
    jw_put(w, "\":", 2);
}

/* jsoncpp valueToString(double, useSpecialFloats=false, precision=17, significantDigits) */
static void jw_double(jw* w, double v) {
    char b[64];
    if (!isfinite(v)) {
        jw_lit(w, isnan(v) ? "null" : (v < 0 ? "-1e+9999" : "1e+9999"));
        return;
    }
    int n = snprintf(b, sizeof b, "%.*g", 17, v);
    jw_put(w, b, (uint64_t)n);
    if (!strchr(b, '.') && !strchr(b, 'e')) jw_lit(w, ".0");
}

/* std::to_string(double) = "%f"; std::to_string(long) = "%ld" */
static void jw_fixed6(jw* w, double v) {
    char b[400];
    int n = snprintf(b, sizeof b, "%f", v);
    jw_put(w, b, (uint64_t)n);
}
static void jw_i64(jw* w, int64_t v) {
    char b[24];
    int n = snprintf(b, sizeof b, "%lld", (long long)v);
    jw_put(w, b, (uint64_t)n);
}

static void jw_qstr_i64(jw* w, int64_t v) {
    jw_put(w, "\"", 1);
    jw_i64(w, v);
    jw_put(w, "\"", 1);
}

static uint64_t orc_cstr_len(const uint8_t* s, uint64_t n) { /* std::string(x.c_str()) */
    const uint8_t* z = memchr(s, 0, n);
    return z ? (uint64_t)(z - s) : n;
}

static int orc_eq(const uint8_t* s, uint64_t n, const char* lit) {
    return n == strlen(lit) && memcmp(s, lit, n) == 0;
}

/* One Order's JSON text (what = SBE_JSON_*); returns its length, writes it when out != NULL. */
uint64_t orc_order_json_one(const uint8_t* const s[8], const uint32_t len[8], int64_t customer_id,
                            int64_t timestamp, double quantity, uint32_t what, uint8_t* out) {
    jw w = {out, 0};
    if (what == SBE_JSON_PUBLISH_HEADERS) {
        /* cluster_client.cpp:308-323: message_type from order.status; keys sorted */
        const int upd = orc_eq(s[7], len[7], "UPDATED") || orc_eq(s[7], len[7], "CANCELLED");
        jw_lit(&w, "{");
        jw_key(&w, "messageId");
        jw_quoted(&w, s[6], len[6]);
        jw_lit(&w, ",");
        jw_key(&w, "messageType");
        jw_lit(&w, upd ? "\"UPDATE_ORDER\"" : "\"CREATE_ORDER\"");
        jw_lit(&w, ",");
        jw_key(&w, "orderId");
        jw_quoted(&w, s[5], len[5]);
        jw_lit(&w, "}");
        return w.n;
    }
    /* order_types.cpp:122-181, members in sorted order at every level */
    jw_lit(&w, "{\"message\":{\"headers\":{\"auth_token\":\"Bearer xxx\",\"connection_uuid\":\"130032\",");
    jw_key(&w, "create_ts");
    jw_qstr_i64(&w, timestamp / 1000000);
    jw_lit(&w, ",");
    jw_key(&w, "customer_id");
    jw_qstr_i64(&w, customer_id);
    jw_lit(&w, ",\"ip_address\":\"10.37.62.251\",\"origin\":\"fix\",");
    jw_key(&w, "origin_id");
    jw_quoted(&w, s[1], orc_cstr_len(s[1], len[1]));
    jw_lit(&w, ",\"origin_name\":\"FIX_GATEWAY\"},\"message\":{\"action\":\"CREATE\",\"order_details\":{");
    jw_key(&w, "client_order_id");
    jw_quoted(&w, s[0], len[0]);
    jw_lit(&w, ",\"order_type\":\"market\",\"quantity\":{");
    jw_key(&w, "token");
    jw_quoted(&w, s[2], len[2]);
    jw_lit(&w, ",");
    jw_key(&w, "value");
    jw_double(&w, quantity);
    jw_lit(&w, "},");
    jw_key(&w, "quantity_value_str");
    jw_put(&w, "\"", 1);
    jw_fixed6(&w, quantity);
    jw_put(&w, "\"", 1);
    jw_lit(&w, ",");
    jw_key(&w, "side");
    jw_quoted(&w, s[4], len[4]);
    jw_lit(&w, ",\"token_pair\":{");
    jw_key(&w, "base_token");
    jw_quoted(&w, s[2], len[2]);
    jw_lit(&w, ",");
    jw_key(&w, "quote_token");
    jw_quoted(&w, s[3], len[3]);
    jw_lit(&w, "}}}},\"msg_type\":\"D\",");
    jw_key(&w, "uuid");
    jw_quoted(&w, s[0], len[0]);
    jw_lit(&w, "}");
    return w.n;
}

/* sbe_order_to_json_batch over host arrays (no capacity limit: out holds the full text). */
int orc_order_json_batch(const uint8_t* arena, const uint32_t* str_off, const uint32_t* str_len,
                         const int64_t* customer_id, const int64_t* timestamp, const double* quantity,
                         uint64_t n, uint32_t what, uint8_t* out, uint64_t* out_off, int nthreads) {
    if (what > SBE_JSON_PUBLISH_HEADERS) return SBE_EINVAL;
    if (nthreads < 1) nthreads = 1;
    uint64_t* base = (uint64_t*)malloc(sizeof(uint64_t) * (n + 1));
    if (!base) return SBE_EINVAL;
    /* string bases for packed input */
    uint64_t acc = 0;
    for (uint64_t i = 0; i < n; ++i) {
        base[i] = acc;
        if (!str_off)
            for (int f = 0; f < 8; ++f) acc += str_len[8 * i + f];
    }
    for (int pass = 0; pass < 2; ++pass) {
#ifdef _OPENMP
#pragma omp parallel for schedule(static) num_threads(nthreads)
#endif
        for (int64_t i = 0; i < (int64_t)n; ++i) {
            const uint8_t* s[8];
            uint32_t l[8];
            uint64_t at = base[i];
            for (int f = 0; f < 8; ++f) {
                l[f] = str_len[8 * i + f];
                if (str_off) s[f] = arena + str_off[8 * i + f];
                else { s[f] = arena + at; at += l[f]; }
            }
            uint64_t m = orc_order_json_one(s, l, customer_id[i], timestamp[i], quantity[i], what,
                                            pass ? out + out_off[i] : NULL);
            if (!pass) out_off[i + 1] = m;
        }
        if (!pass) {
            out_off[0] = 0;
            for (uint64_t i = 0; i < n; ++i) out_off[i + 1] += out_off[i];
        }
    }
    free(base);
    return 0;
}

/* ---- SBEDecoder's one-record struct readers (src/sbe_encoder.cpp:174-323) ---------------- */

/* SBEDecoder::extract_variable_string, src/sbe_encoder.cpp:285-318: u32 length prefix at `off`
 * of a region of `rem` bytes; returns the end offset, 0 when nothing was assigned (prefix past the
 * region, length past the region or above 10 MiB).  *s_off / *s_len: the string assigned. */
static uint64_t sbedec_extract(const uint8_t* p, uint64_t off, uint64_t rem, uint32_t* s_off, uint32_t* s_len) {
    if (off + 4 > rem) return 0;                                   /* :287-290 */
    uint64_t L = rd32(p + off);                                    /* :295-296 */
    off += 4;
    /* :302-305 checks L > rem - 4 whatever the offset, so the reference reads past the record
     * when a later field's length overruns it (undefined); the defined reading: the string must
     * end inside the record (same result for every in-bounds record) */
    if (L > rem - off || L > 10u * 1024u * 1024u) return 0;
    *s_off = (uint32_t)off;
    *s_len = (uint32_t)L;                                          /* :308-315 (0: clear) */
    return off + L;
}

/* SBEDecoder::decode_session_event, src/sbe_encoder.cpp:183-238 */
int orc_sbedecoder_session_event(const uint8_t* rec, uint64_t len, uint32_t* d_off, uint32_t* d_len, uint32_t* got) {
    *got = 0;
    if (!rec || len < 8 + 32) return 0;                            /* :185-187 */
    if (!(rd16(rec + 2) == 2 && rd16(rec + 4) == SBE_CLUSTER_SCHEMA_ID)) return 0; /* :216-223, :320-323 */
    uint64_t rem = len - 40;                                       /* :232 */
    if (rem > 0) {
        uint32_t o = 0, l = 0;
        if (sbedec_extract(rec + 40, 0, rem, &o, &l)) {            /* :233-235 */
            *d_off = 40 + o;
            *d_len = l;
            *got = 1;
        }
    }
    return 1;
}

/* SBEDecoder::decode_acknowledgment, src/sbe_encoder.cpp:240-282.  got: bit k = string k
 * (messageId, status, error) assigned at rec[off[k] .. off[k] + slen[k]); bit 3 = *ts written. */
int orc_sbedecoder_ack(const uint8_t* rec, uint64_t len, uint32_t off[3], uint32_t slen[3], uint32_t* got, int64_t* ts) {
    *got = 0;
    if (!rec || len < 8 + 8) return 0;                             /* :243-245 */
    if (!(rd16(rec + 2) == 2 && rd16(rec + 4) == 1)) return 0;     /* :253-256 */
    *ts = (int64_t)rd64(rec + 8);                                  /* :259-260 */
    *got |= 8;
    const uint8_t* p = rec + 16;
    uint64_t rem = len - 16, o = 0;                                /* :264-265 */
    uint32_t so, sl;
    o = sbedec_extract(p, o, rem, &so, &sl);                       /* :268-270 */
    if (o == 0) return 0;
    off[0] = 16 + so, slen[0] = sl, *got |= 1;
    o = sbedec_extract(p, o, rem, &so, &sl);                       /* :272-274 */
    if (o == 0) return 0;
    off[1] = 16 + so, slen[1] = sl, *got |= 2;
    if (o < rem && sbedec_extract(p, o, rem, &so, &sl)) {          /* :277-279 */
        off[2] = 16 + so, slen[2] = sl, *got |= 4;
    }
    return 1;
}
