// ref_flyweights.cpp — TEST INFRASTRUCTURE ONLY.
//
// Drives the reference's own SBE-generated flyweights (/root/reference/include/model/*.h,
// compiled unmodified from where they lie; nothing is copied) through the call sequences the
// reference codec uses, so the oracle restatement can be checked against the reference code
// itself.  Built by oracle/Makefile into oracle/_ref/libsbe_ref_fw.so (git-ignored).
//
// What is and is not covered:
//  * src/sbe_encoder.cpp includes <json/json.h> (jsoncpp, absent from this image) and
//    src/ack_decoder.cpp includes "sbe/*.h" headers that do not exist and calls accessors the
//    generated code does not have.  Building either would need stand-ins, so they
//    are treated as unbuildable here.  Their flyweight call sequences are driven below instead;
//    the hand-written dispatch around them is pinned by SURVEY Appendix B observations.
#include <cstdint>
#include <cstring>
#include <stdexcept>
#include <string>
#include <string_view>
#include <vector>

#include "model/Acknowledgment.h"
#include "model/CommitOffsetLite.h"
#include "model/MessageHeader.h"
#include "model/OrderNotificationLite.h"
#include "model/OrderRequestLite.h"
#include "model/TopicMessage.h"

namespace {

int e109_field(const std::runtime_error& e) {
    static const char* names[5] = {"topicLength", "messageTypeLength", "uuidLength", "payloadLength",
                                   "headersLength"};
    const std::string w = e.what();
    for (int f = 0; f < 5; ++f)
        if (w.rfind(names[f], 0) == 0) return f + 1;
    return 99;
}

void put_out(uint8_t* buf, uint64_t& at, uint32_t* flen, int f, const std::string& s) {
    flen[f] = (uint32_t)s.size();
    std::memcpy(buf + at, s.data(), s.size());
    at += s.size();
}

// Lite encode in CommitManager::build_commit_offset_message's call order
// (src/commit_manager.cpp:114-130): computeLength, wrapAndApplyHeader, topicId, sequence, putX
// per var field, 8 + encodedLength().
template <class M>
int lite_encode(const std::string* f, uint32_t tid, uint64_t seq, uint8_t* out, uint64_t cap, uint64_t* out_len);

int lite_e109(const std::runtime_error& e, const char* const* names, int nf) {
    const std::string w = e.what();
    for (int k = 0; k < nf; ++k)
        if (w.rfind(names[k], 0) == 0) return k + 1;
    return 99;
}

template <>
int lite_encode<sbe::CommitOffsetLite>(const std::string* f, uint32_t tid, uint64_t seq, uint8_t* out, uint64_t cap,
                                       uint64_t* out_len) {
    static const char* names[2] = {"messageIdLength", "messageIdentifierLength"};
    size_t total;
    try {
        total = sbe::MessageHeader::encodedLength() + sbe::CommitOffsetLite::computeLength(f[0].size(), f[1].size());
    } catch (const std::runtime_error& e) {
        *out_len = 0;
        return lite_e109(e, names, 2);
    }
    std::string buf(total, '\0');
    sbe::CommitOffsetLite m;
    m.wrapAndApplyHeader(&buf[0], 0, buf.size());
    m.topicId(tid);
    m.sequence(seq);
    m.putMessageId(f[0].c_str(), static_cast<std::uint16_t>(f[0].size()));
    m.putMessageIdentifier(f[1].c_str(), static_cast<std::uint16_t>(f[1].size()));
    const uint64_t n = sbe::MessageHeader::encodedLength() + m.encodedLength();
    if (n > cap) return 98;
    std::memcpy(out, buf.data(), n);
    *out_len = n;
    return 0;
}

template <class M>
int lite3_encode(const std::string* f, uint32_t tid, uint64_t seq, uint8_t* out, uint64_t cap, uint64_t* out_len) {
    static const char* names[3] = {"uuidLength", "messageIdentifierLength", "payloadLength"};
    size_t total;
    try {
        total = sbe::MessageHeader::encodedLength() + M::computeLength(f[0].size(), f[1].size(), f[2].size());
    } catch (const std::runtime_error& e) {
        *out_len = 0;
        return lite_e109(e, names, 3);
    }
    std::string buf(total, '\0');
    M m;
    m.wrapAndApplyHeader(&buf[0], 0, buf.size());
    m.topicId(tid);
    m.sequence(seq);
    m.putUuid(f[0].c_str(), static_cast<std::uint16_t>(f[0].size()));
    m.putMessageIdentifier(f[1].c_str(), static_cast<std::uint16_t>(f[1].size()));
    m.putPayload(f[2].c_str(), static_cast<std::uint16_t>(f[2].size()));
    const uint64_t n = sbe::MessageHeader::encodedLength() + m.encodedLength();
    if (n > cap) return 98;
    std::memcpy(out, buf.data(), n);
    *out_len = n;
    return 0;
}

// Lite decode with the generated flyweights: wrapForDecode(buf, 8, blockLength, version, len),
// topicId(), sequence(), getXAsString() in field order.
template <class M>
int lite_decode(char* p, uint64_t len, const sbe::MessageHeader& h, uint32_t* tid, uint64_t* seq, uint32_t* flen,
                uint8_t* fbuf);

template <>
int lite_decode<sbe::CommitOffsetLite>(char* p, uint64_t len, const sbe::MessageHeader& h, uint32_t* tid,
                                       uint64_t* seq, uint32_t* flen, uint8_t* fbuf) {
    sbe::CommitOffsetLite m;
    uint64_t at = 0;
    m.wrapForDecode(p, 8, h.blockLength(), h.version(), len);
    *tid = m.topicId();
    *seq = m.sequence();
    put_out(fbuf, at, flen, 0, m.getMessageIdAsString());
    put_out(fbuf, at, flen, 1, m.getMessageIdentifierAsString());
    return 0;
}

template <class M>
int lite3_decode(char* p, uint64_t len, const sbe::MessageHeader& h, uint32_t* tid, uint64_t* seq, uint32_t* flen,
                 uint8_t* fbuf) {
    M m;
    uint64_t at = 0;
    m.wrapForDecode(p, 8, h.blockLength(), h.version(), len);
    *tid = m.topicId();
    *seq = m.sequence();
    put_out(fbuf, at, flen, 0, m.getUuidAsString());
    put_out(fbuf, at, flen, 1, m.getMessageIdentifierAsString());
    put_out(fbuf, at, flen, 2, m.getPayloadAsString());
    return 0;
}

}  // namespace

extern "C" {

// Lite encode (template 301, 201 or 202).  Returns 0, 1..nf = E109 on that field, 97 = unknown
// template, 98 = capacity.
int ref_lite_encode(uint32_t tmpl, const uint8_t* const* s, const uint32_t* len, uint32_t tid, uint64_t seq,
                    uint8_t* out, uint64_t cap, uint64_t* out_len) {
    std::string f[3];
    const int nf = tmpl == 301 ? 2 : 3;
    for (int i = 0; i < nf; ++i) f[i].assign(reinterpret_cast<const char*>(s[i]), len[i]);
    switch (tmpl) {
        case 301: return lite_encode<sbe::CommitOffsetLite>(f, tid, seq, out, cap, out_len);
        case 201: return lite3_encode<sbe::OrderRequestLite>(f, tid, seq, out, cap, out_len);
        case 202: return lite3_encode<sbe::OrderNotificationLite>(f, tid, seq, out, cap, out_len);
        default: return 97;
    }
}

// Lite decode of a record whose header says template 301 / 201 / 202, schema 1 (the caller
// checks the header; len >= 20).  Returns 0 (fields out) or 1 (E100 thrown).
int ref_lite_decode(const uint8_t* rec, uint64_t len, uint32_t* tid, uint64_t* seq, uint32_t* flen, uint8_t* fbuf) {
    char* p = const_cast<char*>(reinterpret_cast<const char*>(rec));
    try {
        sbe::MessageHeader h;
        h.wrap(p, 0, 1, len);
        switch (h.templateId()) {
            case 301: return lite_decode<sbe::CommitOffsetLite>(p, len, h, tid, seq, flen, fbuf);
            case 201: return lite3_decode<sbe::OrderRequestLite>(p, len, h, tid, seq, flen, fbuf);
            case 202: return lite3_decode<sbe::OrderNotificationLite>(p, len, h, tid, seq, flen, fbuf);
            default: return 2;
        }
    } catch (const std::exception&) {
        return 1;
    }
}

// The sequence of SBEEncoder::encode_topic_message (src/sbe_encoder.cpp:141-164) when wire == 0;
// wire == 1 returns the same record at its wire length (8 + encodedLength(), the length
// ClusterClient::publish_topic emits, src/cluster_client.cpp:1857).
// Returns 0, or 1..5 = E109 on field 1..5 (computeLength throws first, TopicMessage.h:1382-1434).
int ref_tm_encode(const uint8_t* const* s, const uint32_t* len, uint64_t ts, int wire, uint8_t* out,
                  uint64_t cap, uint64_t* out_len) {
    std::string f[5];
    for (int i = 0; i < 5; ++i) f[i].assign(reinterpret_cast<const char*>(s[i]), len[i]);
    size_t total;
    try {
        total = sbe::TopicMessage::sbeBlockAndHeaderLength() +
                sbe::TopicMessage::computeLength(f[0].size(), f[1].size(), f[2].size(), f[3].size(),
                                                 f[4].size());
    } catch (const std::runtime_error& e) {
        *out_len = 0;
        return e109_field(e);
    }
    std::string buffer(total, '\0');
    sbe::TopicMessage tm;
    tm.wrapAndApplyHeader(&buffer[0], 0, buffer.size());
    tm.timestamp(ts);
    tm.sequenceNumber(0);
    tm.putTopic(f[0]);
    tm.putMessageType(f[1]);
    tm.putUuid(f[2]);
    tm.putPayload(f[3]);
    tm.putHeaders(f[4]);
    uint64_t n = tm.encodedLength() + (wire ? sbe::MessageHeader::encodedLength() : 0);
    if (n > cap) return 98;
    std::memcpy(out, buffer.data(), n);
    *out_len = n;
    return 0;
}

// ref_tm_encode over a packed batch (record i's strings back to back after record i-1's), for the
// CPU baseline: the reference's own flyweight sequence per record, records spread over nthreads
// OpenMP threads.  out holds the records back to back at out_off[i] (n + 1 entries, computed by the
// caller from the lengths: wire ? 34 : 26 + Σlen).  Returns the number of records that failed.
int ref_tm_encode_batch(const uint8_t* arena, const uint32_t* str_len, const uint64_t* ts, uint64_t n, int wire,
                        uint8_t* out, const uint64_t* out_off, const uint64_t* in_off, int nthreads) {
    int bad = 0;
#pragma omp parallel for schedule(static) num_threads(nthreads > 0 ? nthreads : 1) reduction(+ : bad)
    for (int64_t i = 0; i < (int64_t)n; ++i) {
        const uint8_t* s[5];
        uint64_t at = in_off[i];
        for (int k = 0; k < 5; ++k) {
            s[k] = arena + at;
            at += str_len[5 * i + k];
        }
        uint64_t len = 0;
        bad += ref_tm_encode(s, str_len + 5 * i, ts[i], wire, out + out_off[i], out_off[i + 1] - out_off[i], &len) != 0;
    }
    return bad;
}

// The encoder block of ClusterClient::publish_topic (src/cluster_client.cpp:1823-1858) in its call
// order, with the protocol.hpp:8-12 constants: buffer of 8+8+Σ+128 zero bytes, MessageHeader
// wrap(buf, 0, SBE_VERSION, size) and the four setters, TopicMessage wrapForEncode(buf, 8,
// size - 8), timestamp, sequenceNumber(0), putX(const char*, static_cast<int>(size)) per field
// (the int becomes put*'s std::uint16_t), resize to 8 + encodedLength().  uuid / headers are the
// caller's ("pub_" + now_nanos(), "{}" for empty headers: :1818-1821).  Returns 0, or 2 if a
// flyweight bounds check threw (never, for these buffer sizes).
int ref_publish_topic(const uint8_t* const* s, const uint32_t* len, uint64_t ts, uint8_t* out, uint64_t cap,
                      uint64_t* out_len) {
    std::string_view f[5];
    for (int i = 0; i < 5; ++i) f[i] = std::string_view(reinterpret_cast<const char*>(s[i]), len[i]);
    std::vector<std::uint8_t> buf;
    buf.resize(8 + 8 + f[0].size() + f[1].size() + f[2].size() + f[3].size() + f[4].size() + 128);
    try {
        sbe::MessageHeader hdr;
        hdr.wrap(reinterpret_cast<char*>(buf.data()), 0, 1, static_cast<std::uint64_t>(buf.size()));
        hdr.blockLength(16);
        hdr.templateId(1);
        hdr.schemaId(1);
        hdr.version(1);
        sbe::TopicMessage msg;
        msg.wrapForEncode(reinterpret_cast<char*>(buf.data()), 8, static_cast<std::uint64_t>(buf.size() - 8));
        msg.timestamp(ts);
        msg.sequenceNumber(0);
        msg.putTopic(f[0].data(), static_cast<int>(f[0].size()));
        msg.putMessageType(f[1].data(), static_cast<int>(f[1].size()));
        msg.putUuid(f[2].data(), static_cast<int>(f[2].size()));
        msg.putPayload(f[3].data(), static_cast<int>(f[3].size()));
        msg.putHeaders(f[4].data(), static_cast<int>(f[4].size()));
        const int encodedLen = 8 + msg.encodedLength();
        buf.resize(encodedLen);
    } catch (const std::exception&) {
        *out_len = 0;
        return 2;
    }
    if (buf.size() > cap) return 98;
    std::memcpy(out, buf.data(), buf.size());
    *out_len = buf.size();
    return 0;
}

// The flyweight part of MessageParser::decode_topic_message_with_sbe (src/sbe_encoder.cpp:966-1135).
// Returns 0 (fields out), 1 = E100 from the main block (→ failure result).  *headers_ok = 0 when
// the separate headers read threw (→ headers "").
int ref_tm_decode_parse(const uint8_t* rec, uint64_t len, uint64_t* ts, uint64_t* seq, uint32_t* flen,
                        uint8_t* fbuf, int* headers_ok) {
    char* p = const_cast<char*>(reinterpret_cast<const char*>(rec));
    uint64_t at = 0;
    try {
        sbe::MessageHeader h;
        h.wrap(p, 0, 0, len);
        sbe::TopicMessage tm;
        tm.wrapForDecode(p, sbe::MessageHeader::encodedLength(), h.blockLength(), h.version(), len);
        *ts = tm.timestamp();
        put_out(fbuf, at, flen, 0, tm.getTopicAsString());
        put_out(fbuf, at, flen, 1, tm.getMessageTypeAsString());
        put_out(fbuf, at, flen, 2, tm.getUuidAsString());
        put_out(fbuf, at, flen, 3, tm.getPayloadAsString());
        *seq = tm.sequenceNumber();
        try {
            put_out(fbuf, at, flen, 4, tm.getHeadersAsString());
            *headers_ok = 1;
        } catch (const std::exception&) {
            flen[4] = 0;
            *headers_ok = 0;
        }
        return 0;
    } catch (const std::exception&) {
        return 1;
    }
}

// The flyweight part of decode_ack's full-ack branch (src/ack_decoder.cpp:55-101):
// wrapForDecode(data, 8, blockLength, version, len - 8) and the three varStrings read only when
// their peeked length is non-zero.  Returns 0 (fields out) or 1 (exception → nullopt).
int ref_ack_decode(const uint8_t* rec, uint64_t len, uint64_t* ts, uint32_t* flen, uint8_t* fbuf) {
    char* p = const_cast<char*>(reinterpret_cast<const char*>(rec));
    uint64_t at = 0;
    try {
        sbe::MessageHeader h;
        h.wrap(p, 0, 1, len);
        sbe::Acknowledgment ack;
        ack.wrapForDecode(p, 8, h.blockLength(), h.version(), len - 8);
        *ts = ack.timestamp();
        std::string s;
        uint16_t l = ack.messageIdLength();
        s.assign(l, '\0');
        if (l > 0) ack.getMessageId(&s[0], l);
        put_out(fbuf, at, flen, 0, l > 0 ? s : std::string());
        l = ack.topicLength();
        s.assign(l, '\0');
        if (l > 0) ack.getTopic(&s[0], l);
        put_out(fbuf, at, flen, 1, l > 0 ? s : std::string());
        l = ack.correlationIdLength();
        s.assign(l, '\0');
        if (l > 0) ack.getCorrelationId(&s[0], l);
        put_out(fbuf, at, flen, 2, l > 0 ? s : std::string());
        return 0;
    } catch (...) {
        return 1;
    }
}

// The flyweight part of MessageHandler::on_egress for a TopicMessage
// (include/aeron_cluster/message_handler.hpp:47-60): wrapForDecode(data, 8, blk, ver, len - 8)
// and read_var_string (getter only for a positive peeked length).  Returns 0 or 1 (throws E100).
int ref_egress_tm(const uint8_t* rec, uint64_t len, uint32_t* flen, uint8_t* fbuf) {
    char* p = const_cast<char*>(reinterpret_cast<const char*>(rec));
    uint64_t at = 0;
    try {
        sbe::MessageHeader h;
        h.wrap(p, 0, 1, len);
        sbe::TopicMessage tm;
        tm.wrapForDecode(p, 8, h.blockLength(), h.version(), len - 8);
        int l;
        std::string s;
#define RVS(f, LEN, GET)                                    \
    l = (int)tm.LEN();                                      \
    if (l > 0) {                                            \
        s.assign((size_t)l, '\0');                          \
        tm.GET(&s[0], (uint64_t)l);                         \
    } else {                                                \
        s.clear();                                          \
    }                                                       \
    put_out(fbuf, at, flen, f, s);
        RVS(0, topicLength, getTopic)
        RVS(1, messageTypeLength, getMessageType)
        RVS(2, uuidLength, getUuid)
        RVS(3, payloadLength, getPayload)
        RVS(4, headersLength, getHeaders)
#undef RVS
        return 0;
    } catch (const std::exception&) {
        return 1;
    }
}

}  // extern "C"
