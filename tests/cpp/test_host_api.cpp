// GPU test of the C++ host mirror (aeron-cluster-client-cpp_amd/host): the reference-shaped API
// against SURVEY Appendix B probe observations and against the oracle (oracle/liboracle.so).
#include <cfloat>
#include <cstdio>
#include <cstring>
#include <iomanip>
#include <iostream>
#include <random>
#include <sstream>
#include <stdexcept>
#include <string>
#include <vector>

#include "aeron_cluster_amd.hpp"
#include "../../oracle/sbe_oracle.h"

using namespace aeron_cluster;

static int failures = 0;
#define CHECK(c)                                                            \
    do {                                                                    \
        if (!(c)) {                                                         \
            std::fprintf(stderr, "FAIL %s:%d: %s\n", __FILE__, __LINE__, #c); \
            ++failures;                                                     \
        }                                                                   \
    } while (0)

static std::string hex(const std::vector<uint8_t>& v) {
    std::string s;
    char b[3];
    for (auto c : v) {
        std::snprintf(b, 3, "%02x", c);
        s += b;
    }
    return s;
}

static std::vector<uint8_t> wire_tm(const std::vector<std::string>& f, uint64_t ts, uint16_t blk = 16) {
    std::vector<uint8_t> b = {(uint8_t)blk, (uint8_t)(blk >> 8), 1, 0, 1, 0, 1, 0};
    for (int i = 0; i < 8; ++i) b.push_back((uint8_t)(ts >> (8 * i)));
    for (int i = 0; i < 8; ++i) b.push_back(0);
    for (auto& s : f) {
        b.push_back((uint8_t)s.size());
        b.push_back((uint8_t)(s.size() >> 8));
        b.insert(b.end(), s.begin(), s.end());
    }
    return b;
}

static bool same(const ParseResult& a, const ParseResult& b) {
    return a.success == b.success && a.error_message == b.error_message && a.message_type == b.message_type &&
           a.message_id == b.message_id && a.payload == b.payload && a.headers == b.headers && a.timestamp == b.timestamp &&
           a.sequence_number == b.sequence_number && a.template_id == b.template_id && a.schema_id == b.schema_id &&
           a.version == b.version && a.block_length == b.block_length && a.correlation_id == b.correlation_id &&
           a.session_id == b.session_id && a.leader_member_id == b.leader_member_id && a.event_code == b.event_code &&
           a.leadership_term_id == b.leadership_term_id;
}

static void put_le(std::vector<uint8_t>& b, uint64_t v, int bytes) {
    for (int i = 0; i < bytes; ++i) b.push_back((uint8_t)(v >> (8 * i)));
}

// SessionEvent (template 2 / schema 111, sbe_messages.hpp:43-54) with a u32-prefixed detail
static std::vector<uint8_t> session_event(int64_t corr, int64_t sess, int64_t term, int32_t leader, int32_t code,
                                          const std::string& detail) {
    std::vector<uint8_t> b = {32, 0, 2, 0, 111, 0, 8, 0};
    put_le(b, (uint64_t)corr, 8);
    put_le(b, (uint64_t)sess, 8);
    put_le(b, (uint64_t)term, 8);
    put_le(b, (uint32_t)leader, 4);
    put_le(b, (uint32_t)code, 4);
    if (!detail.empty()) {
        put_le(b, detail.size(), 4);
        b.insert(b.end(), detail.begin(), detail.end());
    }
    return b;
}

// a schema-111 session message {24,1,111,8} + 24 block bytes around an embedded record
static std::vector<uint8_t> wrapped(const std::vector<uint8_t>& inner) {
    std::vector<uint8_t> b = {24, 0, 1, 0, 111, 0, 8, 0};
    put_le(b, 7, 8);
    put_le(b, 9, 8);
    put_le(b, 0, 8);
    b.insert(b.end(), inner.begin(), inner.end());
    return b;
}

// The fields the predicates and get_description read, from the oracle restatement's descriptor of
// the record (independent of the mirror's materialisation).
static ParseResult oracle_fields(const std::vector<uint8_t>& rec) {
    uint8_t st = 0, fl = 0;
    uint16_t h[4] = {0, 0, 0, 0};
    uint64_t ts = 0;
    uint32_t vo[5] = {0}, vl[5] = {0};
    orc_decode_one(rec.data(), rec.size(), SBE_DEC_PARSE_MESSAGE, &st, &fl, h, &ts, vo, vl);
    ParseResult r;
    auto v = [&](int k) { return std::string(reinterpret_cast<const char*>(rec.data()) + vo[k], vl[k]); };
    if (st == SBE_ST_TM || st == SBE_ST_ACK || st == SBE_ST_SESSION_EVENT || st == SBE_ST_ERR_UNKNOWN_TYPE) {
        r.template_id = h[1];
        r.schema_id = h[2];
    }
    r.success = st < SBE_ST_ERR_NULL_EMPTY;
    if (st == SBE_ST_TM) {
        r.message_type = v(1);
        r.message_id = v(2);
        r.payload = v(3);
        r.headers = v(4);
    } else if (st == SBE_ST_ACK) {
        r.message_type = "Acknowledgment";
        r.message_id = (fl & SBE_FL_ID_DEFAULT) ? "ack_" + std::to_string(ts) : v(0);
        r.payload = (fl & SBE_FL_PAYLOAD_DEFAULT) ? std::string("SUCCESS") : v(1);
        r.headers = v(2);
    } else if (st == SBE_ST_SESSION_EVENT) {
        r.message_type = "SessionEvent";
        r.payload = v(3);
        std::memcpy(&r.event_code, rec.data() + 36, 4);
    }
    return r;
}

// examples/basic_client_example.cpp:272-329, the message callback of BASELINE config #1: which
// branch a ParseResult takes (1 order, 2 acknowledgment, 3 other topic message, 0 none)
static int callback_branch(const ParseResult& r) {
    if (r.is_order_message()) return 1;
    if (r.is_acknowledgment()) return 2;
    if (r.is_topic_message()) return 3;
    return 0;
}

static void surface_tests(const std::vector<std::string>& f5, const std::vector<uint8_t>& wire,
                          const std::vector<uint8_t>& sack, const std::vector<uint8_t>& ack45) {
    auto tm = [&](const std::string& type, const std::string& uuid, const std::string& payload) {
        return wire_tm({"orders", type, uuid, payload, "{\"h\":1}"}, 1760000000000000001ULL);
    };
    std::vector<uint8_t> ack_qty = {8, 0, 2, 0, 1, 0, 1, 0};
    put_le(ack_qty, 1700000000000ULL, 8);
    for (std::string s : {"id_77", "quantity", "x"}) {
        ack_qty.push_back((uint8_t)s.size());
        ack_qty.push_back(0);
        ack_qty.insert(ack_qty.end(), s.begin(), s.end());
    }
    std::vector<uint8_t> ack12 = {8, 0, 2, 0, 1, 0, 1, 0, 1, 2, 3, 4};
    std::vector<uint8_t> t9 = wire;
    t9[2] = 9;
    std::vector<uint8_t> emb_t5 = wire, emb_s7 = wire;
    emb_t5[2] = 5;
    emb_s7[4] = 7;
    struct Case {
        std::vector<uint8_t> rec;
        int branch;
        std::string description;
    };
    const std::vector<Case> cases = {
        {wire, 1, "TopicMessage (type: CREATE_ORDER) [ID: msg_1...]"},
        {tm("REPLAY_COMPLETE", "uuid-abcdefgh", "{\"x\":1}"), 3, "TopicMessage (type: REPLAY_COMPLETE) [ID: uuid-abc...]"},
        {tm("TRADE", "t1", "{\"side\":\"BUY\"}"), 1, "TopicMessage (type: TRADE) [ID: t1...]"},
        {tm("CANCEL_ORDER", "", "{}"), 1, "TopicMessage (type: CANCEL_ORDER)"},
        {wire_tm(f5, 5, 8), 3, "TopicMessage"},
        {sack, 2, "Acknowledgment (type: Acknowledgment) [ID: ack_1000...]"},
        {ack45, 2, "Acknowledgment (type: Acknowledgment) [ID: msg_1...]"},
        {ack_qty, 1, "Acknowledgment (type: Acknowledgment) [ID: id_77...]"},  // payload run "quantity"
        {session_event(0x1122334455667788LL, 5, 6, 1, 0, ""), 0, "SessionEvent (code: OK)"},
        {session_event(1, 5, 6, 2, 2, "10.0.0.2:9002"), 0, "SessionEvent (code: REDIRECT)"},
        {session_event(1, 5, 6, 2, 9, "x"), 0, "SessionEvent (code: UNKNOWN(9))"},
        {wrapped(wire), 1, "TopicMessage (type: CREATE_ORDER) [ID: msg_1...]"},
        {wrapped(sack), 2, "Acknowledgment (type: Acknowledgment) [ID: ack_1000...]"},
        {std::vector<uint8_t>(wire.begin(), wire.begin() + 3), 0, "Parse Error: Failed to decode message header"},
        {t9, 0, "Parse Error: Unknown message type: template=9, schema=1"},
        {std::vector<uint8_t>(wire.begin(), wire.begin() + 50), 0,
         "Parse Error: SBE TopicMessage decoding failed: buffer too short [E100]"},
        {std::vector<uint8_t>({32, 0, 2, 0, 111, 0, 8, 0, 1, 2, 3, 4}), 0, "Parse Error: Failed to decode SessionEvent"},
        {wrapped({}), 0, "Parse Error: Session message too short to contain embedded message"},
        {wrapped({1, 0, 1, 0, 1}), 0, "Parse Error: Embedded message too short"},
        {wrapped(emb_t5), 0, "Parse Error: Unknown embedded message template_id: 5"},
        {wrapped(emb_s7), 0, "Parse Error: Unknown embedded message schema_id: 7"},
        {ack12, 0, "Parse Error: Buffer too short for Acknowledgment message. Need at least 16 bytes, got 12"},
        {wrapped(ack12), 0, "Parse Error: Buffer too short for Acknowledgment message. Need at least 16 bytes, got 12"},
        {{}, 0, "Parse Error: Null or empty data"},
    };
    std::vector<uint8_t> all;
    std::vector<uint64_t> off{0};
    std::vector<ParseResult> single;
    for (const Case& c : cases) {
        const ParseResult r = MessageParser::parse_message(c.rec.empty() ? nullptr : c.rec.data(), c.rec.size());
        single.push_back(r);
        const std::string d = r.get_description();
        if (d != c.description) std::fprintf(stderr, "  description '%s' != '%s'\n", d.c_str(), c.description.c_str());
        CHECK(d == c.description);
        CHECK(callback_branch(r) == c.branch);
        if (!c.rec.empty()) {  // the same branch from the oracle restatement's decode
            const ParseResult o = oracle_fields(c.rec);
            CHECK(callback_branch(o) == c.branch);
            CHECK(o.success == r.success && o.message_type == r.message_type && o.message_id == r.message_id &&
                  o.payload == r.payload && o.template_id == r.template_id && o.schema_id == r.schema_id &&
                  o.event_code == r.event_code);
        }
        all.insert(all.end(), c.rec.begin(), c.rec.end());
        off.push_back(all.size());
    }
    // the session event's fields (sbe_encoder.cpp:629-637)
    CHECK(single[8].correlation_id == 0x1122334455667788LL && single[8].session_id == 5 &&
          single[8].leadership_term_id == 6 && single[8].leader_member_id == 1 && single[9].payload == "10.0.0.2:9002");
    // batch paths == single-record path, record by record
    const auto batch = MessageParser::parse_batch(all.data(), off.data(), cases.size());
    const ParsedBatch pb = MessageParser::decode_batch(all.data(), off.data(), cases.size());
    CHECK(batch.size() == cases.size() && pb.size() == cases.size());
    ParseResult into;  // one object rewritten record after record (every kind over every other)
    for (size_t i = 0; i < cases.size(); ++i) {
        CHECK(same(batch[i], single[i]));
        CHECK(same(pb.result(i), single[i]));
        pb.result_into(i, into);
        CHECK(same(into, single[i]));
        CHECK(pb.success(i) == single[i].success && pb.template_id(i) == single[i].template_id &&
              pb.schema_id(i) == single[i].schema_id && pb.timestamp(i) == single[i].timestamp &&
              pb.sequence_number(i) == single[i].sequence_number);
        if (pb.status(i) == SBE_ST_TM)
            CHECK(pb.view(i, 1) == single[i].message_type && pb.view(i, 2) == single[i].message_id &&
                  pb.view(i, 3) == single[i].payload && pb.view(i, 4) == single[i].headers);
    }
    {  // the same batch from registered (page-locked) memory: decoded in place, same results
        std::vector<uint8_t> reg(all.begin(), all.end());
        reg.resize(reg.size() + 4096);
        host_register(reg.data(), reg.size());
        const auto rb = MessageParser::parse_batch(reg.data(), off.data(), cases.size());
        host_unregister(reg.data());
        for (size_t i = 0; i < cases.size(); ++i) CHECK(same(rb[i], single[i]));
    }
    {  // into a reused vector: the same batch, then the records in reverse order over the old
       // results (every field of a session event / Ack / error result rewritten by another kind)
        std::vector<ParseResult> reuse;
        MessageParser::parse_batch(all.data(), off.data(), cases.size(), reuse);
        CHECK(reuse.size() == cases.size());
        for (size_t i = 0; i < cases.size(); ++i) CHECK(same(reuse[i], single[i]));
        std::vector<uint8_t> rev;
        std::vector<uint64_t> roff{0};
        for (size_t k = cases.size(); k-- > 0;) {
            rev.insert(rev.end(), all.begin() + off[k], all.begin() + off[k + 1]);
            roff.push_back(rev.size());
        }
        MessageParser::parse_batch(rev.data(), roff.data(), cases.size(), reuse);
        for (size_t i = 0; i < cases.size(); ++i) CHECK(same(reuse[i], single[cases.size() - 1 - i]));
        MessageParser::parse_batch(all.data(), off.data(), 2, reuse);  // shrinks to n
        CHECK(reuse.size() == 2 && same(reuse[1], single[1]));
    }
    size_t visited = 0;
    pb.for_each([&](size_t i, const ParseResult& r) {
        CHECK(i == visited && same(r, single[i]));
        ++visited;
    });
    CHECK(visited == cases.size());

    // BatchingParser: the cases repeated, fed in polls of 1-100 fragments (the reference's
    // per-poll limit), delivered in order with results equal to parse_message's, under small
    // batches (many hand-offs, more batches in flight than are kept), the byte limit, the
    // deadline, an explicit flush and the destructor's flush, 2 to 64 batches kept, with and
    // without spinning waits
    {
        const size_t N = 5000;
        struct Setting {
            size_t max_records, max_bytes;
            int delay_us;
            size_t batches;
            int spin_us;
        };
        for (const Setting st : {Setting{7, 1u << 20, 1000000, 4, 200}, Setting{4096, 1u << 20, 200, 4, 200},
                                 Setting{8192, 3000, 1000000, 4, 200}, Setting{1, 1u << 20, 0, 4, 200},
                                 Setting{5, 1u << 20, 1000000, 2, 0}, Setting{3, 1u << 20, 0, 8, 50},
                                 Setting{64, 1u << 20, 1000000, 64, 200}}) {
            size_t got = 0;
            bool ok = true;
            {
                BatchingParser::Options o;
                o.max_records = st.max_records;
                o.max_bytes = st.max_bytes;
                o.max_delay = std::chrono::microseconds(st.delay_us);
                o.batches = st.batches;
                o.spin = std::chrono::microseconds(st.spin_us);
                BatchingParser bp([&](const ParseResult& r) { ok = ok && same(r, single[got++ % cases.size()]); }, o);
                uint64_t seed = 12345;
                size_t fed = 0;
                while (fed < N) {
                    seed = seed * 6364136223846793005ULL + 1442695040888963407ULL;
                    const size_t poll = 1 + (size_t)((seed >> 33) % 100);
                    for (size_t k = 0; k < poll && fed < N; ++k, ++fed) {
                        const Case& c = cases[fed % cases.size()];
                        bp.on_fragment(c.rec.empty() ? nullptr : c.rec.data(), c.rec.size());
                    }
                    (void)bp.poll();
                    CHECK(got + bp.pending() == fed);
                }
                if (st.max_records != 7) {
                    const size_t before = got;
                    CHECK(bp.flush() == N - before);
                    CHECK(got == N && bp.pending() == 0 && bp.delivered() == N);
                }
            }  // destructor: flush
            CHECK(ok && got == N);
            if (!(ok && got == N))
                std::fprintf(stderr, "  BatchingParser max_records %zu batches %zu: %zu of %zu delivered, ok %d\n",
                             st.max_records, st.batches, got, N, (int)ok);
        }
        // a handler that throws: the exception leaves the poll / flush that delivered
        // the record; the records after it come with the next calls, in order, none twice
        for (const size_t batches : {size_t(2), size_t(4)}) {
            const size_t M = 3000;
            size_t got = 0, throws = 0;
            bool ok = true;
            BatchingParser::Options o;
            o.max_records = 64;
            o.max_delay = std::chrono::microseconds(0);
            o.batches = batches;
            BatchingParser bp(
                [&](const ParseResult& r) {
                    const size_t k = got++;
                    ok = ok && same(r, single[k % cases.size()]);
                    if (k % 997 == 500) throw std::runtime_error("handler failure");
                },
                o);
            size_t fed = 0;
            while (fed < M) {
                for (size_t k = 0; k < 50 && fed < M; ++k, ++fed) {
                    const Case& c = cases[fed % cases.size()];
                    try {
                        bp.on_fragment(c.rec.empty() ? nullptr : c.rec.data(), c.rec.size());
                    } catch (const std::runtime_error&) {
                        ++throws;
                    }
                }
                try {
                    (void)bp.poll();
                } catch (const std::runtime_error&) {
                    ++throws;
                }
            }
            for (int t = 0; t < 10; ++t) {
                try {
                    (void)bp.flush();
                    break;
                } catch (const std::runtime_error&) {
                    ++throws;
                }
            }
            CHECK(ok && got == M && throws == 3 && bp.delivered() == M && bp.pending() == 0);
            if (!(ok && got == M && throws == 3))
                std::fprintf(stderr, "  BatchingParser throwing handler, batches %zu: %zu of %zu, %zu throws, ok %d\n",
                             batches, got, M, throws, (int)ok);
        }
    }

    // MessageParser's other public statics (sbe_messages.hpp:423-450, sbe_encoder.cpp:554-616)
    CHECK(same(MessageParser::decode_topic_message_with_sbe(wire.data(), wire.size()),
               MessageParser::parse_message(wire.data(), wire.size())));
    CHECK(MessageParser::decode_topic_message_with_sbe(sack.data(), sack.size()).error_message ==
          "Not a TopicMessage (got template_id=2, schema_id=1)");
    const auto wtm = wrapped(wire);
    CHECK(MessageParser::decode_topic_message_with_sbe(wtm.data(), wtm.size()).error_message ==
          "Not a TopicMessage (got template_id=1, schema_id=111)");
    auto e107 = MessageParser::decode_topic_message_with_sbe(wire.data(), 5);
    CHECK(!e107.success && e107.template_id == 0 &&
          e107.error_message == "SBE TopicMessage decoding failed: buffer too short for flyweight [E107]");
    CHECK(same(MessageParser::decode_acknowledgment_with_sbe(ack45.data(), ack45.size()),
               MessageParser::parse_message(ack45.data(), ack45.size())));
    CHECK(MessageParser::decode_acknowledgment_with_sbe(wire.data(), wire.size()).error_message ==
          "Message is not an Acknowledgment. Expected: template_id=2, schema_id=1. Got: template_id=1, schema_id=1");
    CHECK(MessageParser::decode_acknowledgment_with_sbe(wire.data(), 3).error_message == "Buffer too short for SBE header");
    CHECK(MessageParser::decode_acknowledgment_with_sbe(ack12.data(), ack12.size()).error_message ==
          "Buffer too short for Acknowledgment message. Need at least 16 bytes, got 12");
    CHECK(MessageParser::get_message_type(wire.data(), wire.size()) == "TopicMessage");
    CHECK(MessageParser::get_message_type(sack.data(), sack.size()) == "Acknowledgment");
    CHECK(MessageParser::get_message_type(wire.data(), 7) == "INVALID");
    CHECK(MessageParser::get_message_type(cases[8].rec.data(), 8) == "SessionEvent");
    const uint8_t h_conn[8] = {16, 0, 3, 0, 111, 0, 8, 0}, h_c9[8] = {0, 0, 9, 0, 111, 0, 0, 0},
                  h_t9[8] = {0, 0, 9, 0, 1, 0, 0, 0}, h_s7[8] = {0, 0, 1, 0, 7, 0, 0, 0};
    CHECK(MessageParser::get_message_type(h_conn, 8) == "SessionConnectRequest");
    CHECK(MessageParser::get_message_type(h_c9, 8) == "UnknownClusterMessage(9)");
    CHECK(MessageParser::get_message_type(h_t9, 8) == "UnknownTopicMessage(9)");
    CHECK(MessageParser::get_message_type(h_s7, 8) == "UnknownSchema(7,1)");
    CHECK(MessageParser::extract_correlation_id(cases[8].rec.data(), cases[8].rec.size()) == 0x1122334455667788LL);
    CHECK(MessageParser::extract_correlation_id(cases[8].rec.data(), 15) == 0);
    CHECK(MessageParser::extract_correlation_id(wire.data(), wire.size()) == 0);
    CHECK(MessageParser::is_acknowledgment_for(ack45.data(), ack45.size(), "msg_1"));
    CHECK(MessageParser::is_acknowledgment_for(ack45.data(), ack45.size(), "orders"));  // payload holds it
    CHECK(!MessageParser::is_acknowledgment_for(ack45.data(), ack45.size(), "zzz"));
    CHECK(!MessageParser::is_acknowledgment_for(wire.data(), wire.size(), "msg_1"));  // a TopicMessage
    {  // parse_message_debug: the hex dump of records up to 200 bytes goes to stdout (:557-559)
        std::ostringstream cap;
        std::streambuf* old = std::cout.rdbuf(cap.rdbuf());
        const ParseResult r = MessageParser::parse_message_debug(wire.data(), wire.size(), "p");
        std::cout.rdbuf(old);
        CHECK(same(r, MessageParser::parse_message(wire.data(), wire.size())));
        CHECK(cap.str().rfind("p  0000: 10 00 01 00 01 00 01 00  88 77 66 55 44 33 22 11  |.........wfUD3\".|\n", 0) == 0);
        // 71 bytes, 64 shown (max_bytes 64), then the rest counted
        CHECK(cap.str().find("p  0040: ") == std::string::npos && cap.str().find("p  ... (7 more bytes)\n") != std::string::npos);
        std::cout << std::setfill(' ');
        std::vector<uint8_t> big = wire_tm({"orders", "CREATE_ORDER", "u", std::string(300, 'p'), "h"}, 3);
        cap.str("");
        old = std::cout.rdbuf(cap.rdbuf());
        (void)MessageParser::parse_message_debug(big.data(), big.size());
        std::cout.rdbuf(old);
        CHECK(cap.str().empty());
    }
    // SBEUtils (src/sbe_encoder.cpp:370-485)
    CHECK(SBEUtils::format_timestamp(1760000000123456789LL) == "2025-10-09 08:53:20 UTC.123456789");
    CHECK(SBEUtils::is_valid_sbe_message(wire.data(), wire.size()) && !SBEUtils::is_valid_sbe_message(wire.data(), 20) &&
          !SBEUtils::is_valid_sbe_message(h_s7, 8));
    const auto strs = SBEUtils::extract_readable_strings(ack45.data(), ack45.size(), 3);
    CHECK(strs.size() == 3 && strs[0] == "msg_1" && strs[1] == "orders" && strs[2] == "corr");
    CHECK(SBEUtils::get_session_event_code_string(3) == "AUTHENTICATION_REJECTED" &&
          SBEUtils::get_session_event_code_string(4) == "CLOSED" && SBEUtils::get_session_event_code_string(1) == "ERROR");
    CHECK(SBEUtils::generate_correlation_id() > 0 && SBEUtils::is_valid_correlation_id(1) &&
          !SBEUtils::is_valid_correlation_id(0));
}

int main() {
    if (!gpu_codec_available()) {
        std::fprintf(stderr, "no gfx950 device\n");
        return 2;
    }
    const std::vector<std::string> f5 = {"orders", "CREATE_ORDER", "msg_1", "{\"a\":1}", "{\"h\":2}"};
    // --- SBEEncoder::encode_topic_message
    auto e = SBEEncoder::encode_topic_message(f5[0], f5[1], f5[2], f5[3], f5[4], 0x1122334455667788LL);
    CHECK(e.size() == 63);
    CHECK(hex(e).rfind("100001000100010088776655443322110000000000000000", 0) == 0);
    CHECK(hex(e).size() >= 20 && hex(e).substr(hex(e).size() - 20) == "07007b2261223a317d07");
    CHECK(SBEEncoder::encode_topic_message("", "", "", "", "", 1).size() == 26);
    CHECK(SBEEncoder::encode_topic_message(f5[0], f5[1], f5[2], f5[3], "", 1).size() == 56);
    try {
        SBEEncoder::encode_topic_message(std::string(65535, 'x'), "a", "b", "c", "d", 1);
        CHECK(false);
    } catch (const std::runtime_error& ex) {
        CHECK(std::string(ex.what()) == "topicLength too long for length type [E109]");
    }
    // timestamp 0 → wall clock milliseconds
    auto z = SBEEncoder::encode_topic_message("t", "m", "u", "p", "h", 0);
    uint64_t zts = 0;
    for (int i = 7; i >= 0; --i) zts = (zts << 8) | z[8 + i];
    CHECK(zts > 1700000000000ULL && zts < 100000000000000ULL);

    // --- MessageParser::parse_message probes
    auto wire = wire_tm(f5, 0x1122334455667788ULL);
    auto pr = MessageParser::parse_message(e.data(), e.size());
    CHECK(pr.success && pr.message_type == "CREATE_ORDER" && pr.message_id == "msg_1" && pr.payload == "{\"a\":1}" &&
          pr.headers.empty());
    CHECK(pr.is_topic_message());
    std::vector<uint8_t> cut(wire.begin(), wire.begin() + 50);
    pr = MessageParser::parse_message(cut.data(), cut.size());
    CHECK(!pr.success && pr.template_id == 0 && pr.error_message == "SBE TopicMessage decoding failed: buffer too short [E100]");
    // sequence_number: the payload's "_sequence_number", evaluated on the device (jsoncpp 1.9.5
    // semantics; src/sbe_encoder.cpp:1031-1125), against the oracle restatement
    {
        const std::vector<std::string> pays = {
            "{\"_sequence_number\":17}", "{\"message\":{\"_sequence_number\":\"4\"}}",
            "{\"\\u005fsequence_number\": 9}", "/* c */ {\"_sequence_number\": 2.5,}", "{\"_sequence_number\": -1}",
            "{\"_sequence_number\": 5", "[{\"_sequence_number\": 5}]", "{\"a\": \"\\\"q\\\"\"}"};
        const uint64_t want[] = {17, 4, 9, 2, ~0ULL, 0, 0, 0};
        for (size_t k = 0; k < pays.size(); ++k) {
            auto f = f5;
            f[3] = pays[k];
            auto w = wire_tm(f, 7);
            auto p = MessageParser::parse_message(w.data(), w.size());
            const uint64_t o = orc_seq_eval(reinterpret_cast<const uint8_t*>(pays[k].data()), pays[k].size());
            CHECK(p.success && p.payload == pays[k] && p.sequence_number == want[k] && o == want[k]);
        }
    }
    auto t9 = wire;
    t9[2] = 9;
    pr = MessageParser::parse_message(t9.data(), t9.size());
    CHECK(!pr.success && pr.template_id == 9 && pr.schema_id == 1 &&
          pr.error_message == "Unknown message type: template=9, schema=1");
    auto b8 = wire_tm(f5, 0x1122334455667788ULL, 8);
    pr = MessageParser::parse_message(b8.data(), b8.size());
    CHECK(pr.success && pr.message_type.empty() && pr.message_id.empty() && pr.payload.empty() && pr.headers == "orders");
    pr = MessageParser::parse_message(wire.data(), 3);
    CHECK(!pr.success && pr.error_message == "Failed to decode message header");
    pr = MessageParser::parse_message(nullptr, 0);
    CHECK(!pr.success && pr.error_message == "Null or empty data");
    std::vector<uint8_t> sack = {8, 0, 2, 0, 1, 0, 1, 0};
    const uint64_t ms = 1000000000000ULL;
    for (int i = 0; i < 8; ++i) sack.push_back((uint8_t)(ms >> (8 * i)));
    pr = MessageParser::parse_message(sack.data(), sack.size());
    CHECK(pr.success && pr.message_type == "Acknowledgment" && pr.message_id == "ack_1000000000000" &&
          pr.payload == "SUCCESS" && pr.timestamp == 1000000000000LL);

    // --- decode_ack / on_egress probes
    auto a = decode_ack(sack.data(), sack.size());
    CHECK(a && a->simple_control_ack && a->timestamp_nanos == 1000000000000000000ULL);
    std::vector<uint8_t> ack37 = {8, 0, 2, 0, 1, 0, 1, 0};
    for (int i = 0; i < 8; ++i) ack37.push_back((uint8_t)(1700000000000ULL >> (8 * i)));
    for (std::string s : {"msg_1", "orders", "corr"}) {
        ack37.push_back((uint8_t)s.size());
        ack37.push_back(0);
        ack37.insert(ack37.end(), s.begin(), s.end());
    }
    CHECK(ack37.size() == 37 && !decode_ack(ack37.data(), ack37.size()));
    auto ack45 = ack37;
    ack45.resize(45, 0);
    a = decode_ack(ack45.data(), ack45.size());
    CHECK(a && !a->simple_control_ack && a->message_id == "msg_1" && a->topic == "orders" && a->correlation_id == "corr" &&
          a->timestamp_nanos == 1700000000000000000ULL);
    MessageHandler h;
    int acks = 0, tms = 0;
    h.set_ack_callback([&](const AckInfo&) { ++acks; });
    h.set_topic_message_callback([&](std::string_view t, std::string_view, std::string_view, std::string_view,
                                     std::string_view hd) {
        ++tms;
        CHECK(t == "orders" && hd == "{\"h\":2}");
    });
    bool threw = false;
    try {
        h.on_egress(wire.data(), wire.size());
    } catch (const std::runtime_error& ex) {
        threw = std::string(ex.what()) == "buffer too short [E100]";
    }
    CHECK(threw);
    h.on_egress(ack37.data(), ack37.size());
    CHECK(acks == 0 && tms == 0);
    h.on_egress(ack45.data(), ack45.size());
    auto wire8 = wire;
    wire8.resize(wire.size() + 8, 0);
    h.on_egress(wire8.data(), wire8.size());
    CHECK(acks == 1 && tms == 1);

    // --- batch encode / parse vs the oracle on random records
    std::mt19937_64 rng(42);
    std::vector<std::vector<std::string>> recs(5000);
    std::vector<TopicMessageFields> msgs;
    std::string arena;
    std::vector<uint32_t> lens;
    std::vector<uint64_t> tss;
    for (auto& r : recs) {
        for (int k = 0; k < 5; ++k) {
            std::string s(rng() % 90, ' ');
            for (auto& c : s) c = (char)(32 + rng() % 95);
            r.push_back(s);
            arena += s;
            lens.push_back((uint32_t)s.size());
        }
        tss.push_back(rng() | 1);
    }
    for (size_t i = 0; i < recs.size(); ++i)
        msgs.push_back({recs[i][0], recs[i][1], recs[i][2], recs[i][3], recs[i][4], (int64_t)tss[i]});
    for (auto len : {EncodeLength::Wire, EncodeLength::Reference}) {
        EncodedBatch b = SBEEncoder::encode_topic_batch(msgs, len);
        std::vector<uint8_t> eo(arena.size() + 34 * recs.size() + 16);
        std::vector<uint64_t> eoff(recs.size() + 1);
        std::vector<uint8_t> est(recs.size());
        orc_encode_batch(reinterpret_cast<const uint8_t*>(arena.data()), nullptr, lens.data(), tss.data(), recs.size(), 0,
                         len == EncodeLength::Reference ? SBE_ENC_REF_TRUNCATE8 : 0u, eo.data(), eoff.data(), est.data(), 1);
        CHECK(b.offsets == eoff);
        CHECK(b.bytes.size() == eoff.back() && std::memcmp(b.bytes.data(), eo.data(), b.bytes.size()) == 0);
        size_t offered = 0;
        CHECK(offer_batch(b, [&](const uint8_t*, size_t) { ++offered; return true; }) == recs.size());
        CHECK(offered == recs.size());
        auto prs = MessageParser::parse_batch(b.bytes.data(), b.offsets.data(), recs.size());
        for (size_t i = 0; i < recs.size(); ++i) {
            // the reference-length form drops the last 8 bytes: with headers shorter than 6 bytes
            // that cuts into the payload and parse_message fails with E100
            if (len == EncodeLength::Reference && recs[i][4].size() < 6) {
                CHECK(!prs[i].success &&
                      prs[i].error_message == "SBE TopicMessage decoding failed: buffer too short [E100]");
                continue;
            }
            CHECK(prs[i].success && prs[i].message_type == recs[i][1] && prs[i].message_id == recs[i][2] &&
                  prs[i].payload == recs[i][3] && (int64_t)tss[i] == prs[i].timestamp);
            CHECK(prs[i].headers == (len == EncodeLength::Wire ? recs[i][4] : std::string()));
            if (failures > 20) break;
        }
    }
    // --- every field length 0..80 in every field position, against hand-built wire bytes: covers
    // each size class of the staging copy (1..3, 4..7, 8..15, 16..64 overlapping moves, >64 memcpy)
    // independently of the oracle, then parses the same records back into a reused vector
    {
        std::vector<TopicMessageFields> fm;
        std::vector<std::vector<std::string>> fr;
        for (int f = 0; f < 5; ++f)
            for (int L = 0; L <= 80; ++L) {
                std::vector<std::string> r(5);
                for (int k = 0; k < 5; ++k) {
                    size_t n = k == f ? (size_t)L : (size_t)((L * 7 + k * 13) % 81);
                    r[k].resize(n);
                    for (size_t j = 0; j < n; ++j) r[k][j] = (char)('A' + (j * 31 + k * 7 + L) % 58);
                }
                fr.push_back(r);
            }
        // the fields are views: into fr, once it no longer grows
        for (size_t i = 0; i < fr.size(); ++i)
            fm.push_back({fr[i][0], fr[i][1], fr[i][2], fr[i][3], fr[i][4],
                          (int64_t)(1700000000000000000LL + 1000003 * (int64_t)(i % 81) + (int64_t)(i / 81))});
        EncodedBatch b = SBEEncoder::encode_topic_batch(fm, EncodeLength::Wire);
        std::vector<uint8_t> want;
        std::vector<uint64_t> woff{0};
        auto put = [&](uint64_t v, int nb) { for (int j = 0; j < nb; ++j) want.push_back((uint8_t)(v >> (8 * j))); };
        for (size_t i = 0; i < fr.size(); ++i) {
            put(16, 2), put(1, 2), put(1, 2), put(1, 2);
            put((uint64_t)fm[i].timestamp, 8), put(0, 8);
            for (int k = 0; k < 5; ++k) {
                put(fr[i][k].size(), 2);
                want.insert(want.end(), fr[i][k].begin(), fr[i][k].end());
            }
            woff.push_back(want.size());
        }
        CHECK(b.offsets == woff);
        CHECK(b.bytes == want);
        std::vector<ParseResult> prs(3);  // reused: more records than the vector holds
        MessageParser::parse_batch(b.bytes.data(), b.offsets.data(), fr.size(), prs);
        CHECK(prs.size() == fr.size());
        for (size_t i = 0; i < fr.size() && failures <= 20; ++i)
            CHECK(prs[i].success && prs[i].message_type == fr[i][1] && prs[i].message_id == fr[i][2] &&
                  prs[i].payload == fr[i][3] && prs[i].headers == fr[i][4] && prs[i].timestamp == fm[i].timestamp);
    }
    // ---- session frames (src/session_manager.cpp:936-967, :1050-1144) ----
    {
        SessionFrameEncoder sf;
        sf.update_session_header(0x0102030405060708LL, -2);
        auto fr = sf.create_combined_message("orders", "CREATE_ORDER", "msg_1", "{\"a\":1}", "{\"h\":2}");
        CHECK(fr.size() == 32 + 63);
        CHECK(hex(fr).rfind("180001006f000800" "0807060504030201" "feffffffffffffff" "0000000000000000" "1000010001000100", 0) == 0);
        uint64_t ns = 0;
        std::memcpy(&ns, fr.data() + 40, 8);
        CHECK(ns > 1700000000000000000ULL);  // high_resolution_clock nanoseconds (:1075-1076)
        auto pr = MessageParser::parse_message(fr.data(), fr.size());
        CHECK(pr.success && pr.message_id == "msg_1" && pr.payload == "{\"a\":1}" && pr.block_length == 16);
        try {
            sf.create_combined_message(std::string(65535, 'x'), "", "", "", "");
            CHECK(false);
        } catch (const std::runtime_error& ex) {
            CHECK(std::string(ex.what()) == "topicLength too long for length type [E109]");
        }
        std::vector<TopicMessageFields> msgs;
        for (size_t i = 0; i < recs.size(); ++i)
            msgs.push_back({recs[i][0], recs[i][1], recs[i][2], recs[i][3], recs[i][4], (int64_t)tss[i]});
        EncodedBatch b = sf.encode_batch(msgs, EncodeLength::Wire);
        std::vector<uint8_t> eo(arena.size() + 66 * recs.size() + 16);
        std::vector<uint64_t> eoff(recs.size() + 1);
        std::vector<uint8_t> est(recs.size());
        orc_encode_session_batch(reinterpret_cast<const uint8_t*>(arena.data()), nullptr, lens.data(), tss.data(),
                                 recs.size(), 0, 0, 0x0102030405060708LL, -2, eo.data(), eoff.data(), est.data(), 1);
        CHECK(b.offsets == eoff);
        CHECK(b.bytes.size() == eoff.back() && std::memcmp(b.bytes.data(), eo.data(), b.bytes.size()) == 0);
    }
    // ---- CommitOffsetLite (src/commit_manager.cpp:107-132) ----
    {
        CommitManager cm;
        CommitOffset o;
        o.topic = "orders";
        o.message_identifier = "orders:17";
        o.message_id = "msg_42";
        o.sequence_number = 0x1122334455667788ULL;
        auto m = cm.build_commit_offset_message("orders", "client", o);
        CHECK(m.size() == 24 + 6 + 9);
        CHECK(hex(m) == "0c002d0101000100" "03000000" "8877665544332211" "0600" + hex(std::vector<uint8_t>(o.message_id.begin(), o.message_id.end())) +
                            "0900" + hex(std::vector<uint8_t>(o.message_identifier.begin(), o.message_identifier.end())));
        auto lr = decode_lite(m.data(), m.size());
        CHECK(lr && lr->template_id == 301 && lr->topic_id == 3 && lr->sequence == o.sequence_number &&
              lr->fields.size() == 2 && lr->fields[0] == "msg_42" && lr->fields[1] == "orders:17");
        CHECK(!decode_lite(m.data(), m.size() - 1));  // E100
        o.topic = "nope";
        bool threw = false;
        try {
            cm.build_commit_offset_message("nope", "c", o);
        } catch (const std::runtime_error&) {
            threw = true;
        }
        CHECK(threw);
        o.topic = "order_request_topic";
        o.message_id = std::string(65535, 'q');
        try {
            cm.build_commit_offset_message("x", "c", o);
            CHECK(false);
        } catch (const std::runtime_error& ex) {
            CHECK(std::string(ex.what()) == "messageIdLength too long for length type [E109]");
        }
    }
    // ---- fragment reassembly (src/cluster_client.cpp:39-82), the accumulator across calls ----
    {
        FragmentReassembler fr;
        const std::vector<std::string> frags = {"AB", "cd", "ef", "X", "gh", "ij", "k"};
        const std::vector<uint8_t> fl = {0xC0, 0x80, 0x00, 0xC0, 0x40, 0x80, 0x00};
        std::string joined;
        std::vector<uint64_t> off{0};
        for (auto& f : frags) {
            joined += f;
            off.push_back(joined.size());
        }
        auto r1 = fr.on_fragments(reinterpret_cast<const uint8_t*>(joined.data()), off.data(), fl.data(), frags.size());
        CHECK(r1.offsets.size() == 4);
        CHECK(std::string(r1.record(0)) == "AB" && std::string(r1.record(1)) == "X" && std::string(r1.record(2)) == "cdefgh");
        CHECK(fr.pending_bytes() == 3);  // "ijk" waits for its END
        const std::string rest = "lm";
        const uint64_t off2[2] = {0, 2};
        const uint8_t fl2[1] = {0x40};
        auto r2 = fr.on_fragments(reinterpret_cast<const uint8_t*>(rest.data()), off2, fl2, 1);
        CHECK(r2.offsets.size() == 2 && std::string(r2.record(0)) == "ijklm" && fr.pending_bytes() == 0);
    }
    {  // Order::to_json / orders_to_json (src/order_types.cpp:122-181, src/cluster_client.cpp:308-323)
        Order o;
        o.client_order_uuid = "cli-uuid-1";
        o.identifier = "FIXID";
        o.base_token = "BTC";
        o.quote_token = "USDC";
        o.side = "BUY";
        o.id = "ord-7";
        o.customer_id = 42;
        o.timestamp = 1760000000123456789LL;
        o.quantity = 0.1;
        const std::string known =
            "{\"message\":{\"headers\":{\"auth_token\":\"Bearer xxx\",\"connection_uuid\":\"130032\",\"create_ts\":"
            "\"1760000000123\",\"customer_id\":\"42\",\"ip_address\":\"10.37.62.251\",\"origin\":\"fix\",\"origin_id\":"
            "\"FIXID\",\"origin_name\":\"FIX_GATEWAY\"},\"message\":{\"action\":\"CREATE\",\"order_details\":{"
            "\"client_order_id\":\"cli-uuid-1\",\"order_type\":\"market\",\"quantity\":{\"token\":\"BTC\",\"value\":"
            "0.10000000000000001},\"quantity_value_str\":\"0.100000\",\"side\":\"BUY\",\"token_pair\":{\"base_token\":"
            "\"BTC\",\"quote_token\":\"USDC\"}}}},\"msg_type\":\"D\",\"uuid\":\"cli-uuid-1\"}";
        CHECK(o.to_json() == known);
        std::mt19937_64 rng(5);
        std::vector<Order> orders(3000);
        std::vector<std::string> mids(orders.size());
        for (size_t i = 0; i < orders.size(); ++i) {
            Order& x = orders[i];
            x.client_order_uuid = "u" + std::to_string(rng() % 100000) + (i % 7 == 0 ? "\"\\\n\xc3\xa9" : "");
            x.identifier = i % 11 == 0 ? std::string("id\0tail", 7) : "ID" + std::to_string(i);
            x.base_token = "BTC";
            x.quote_token = i % 2 ? "USDC" : "USDT";
            x.side = i % 3 ? "BUY" : "SELL";
            x.id = "o" + std::to_string(i);
            x.status = i % 5 == 0 ? "UPDATED" : (i % 5 == 1 ? "CANCELLED" : "CREATED");
            x.customer_id = (int64_t)(rng() >> 20);
            x.timestamp = (int64_t)rng();
            uint64_t bits = rng();
            double d;
            std::memcpy(&d, &bits, 8);
            x.quantity = i % 2 ? d : (double)(rng() % 1000000) / 10000.0;
            mids[i] = "msg_" + std::to_string(i);
        }
        OrderJsonBatch b = orders_to_json(orders, mids);
        for (size_t i = 0; i < orders.size(); ++i) {
            const Order& x = orders[i];
            const std::string* fs[8] = {&x.client_order_uuid, &x.identifier, &x.base_token, &x.quote_token,
                                        &x.side, &x.id, &mids[i], &x.status};
            const uint8_t* sp[8];
            uint32_t sl[8];
            for (int k = 0; k < 8; ++k) {
                sp[k] = reinterpret_cast<const uint8_t*>(fs[k]->data());
                sl[k] = (uint32_t)fs[k]->size();
            }
            for (int w = 0; w < 2; ++w) {
                const EncodedBatch& e = w ? b.headers : b.payload;
                std::vector<uint8_t> exp(orc_order_json_one(sp, sl, x.customer_id, x.timestamp, x.quantity, w, nullptr));
                orc_order_json_one(sp, sl, x.customer_id, x.timestamp, x.quantity, w, exp.data());
                const std::vector<uint8_t> got(e.bytes.begin() + e.offsets[i], e.bytes.begin() + e.offsets[i + 1]);
                if (got != exp) {
                    CHECK(got == exp);
                    break;
                }
            }
        }
        CHECK(b.payload.status.size() == orders.size() && b.headers.offsets.size() == orders.size() + 1);
    }
    {  // a lone Order at the per-record worst case (empty strings, extreme numbers): ADVICE r1
        for (double q : {DBL_MAX, -DBL_MAX, DBL_MIN, -0.0}) {
            Order o;
            o.status = "";
            o.quantity = q;
            o.customer_id = INT64_MIN;
            o.timestamp = INT64_MIN;
            const std::string got = o.to_json();
            const std::string* fs[8] = {&o.client_order_uuid, &o.identifier, &o.base_token, &o.quote_token,
                                        &o.side, &o.id, &o.status, &o.status};
            const std::string empty;
            fs[6] = &empty;
            const uint8_t* sp[8];
            uint32_t sl[8];
            for (int k = 0; k < 8; ++k) {
                sp[k] = reinterpret_cast<const uint8_t*>(fs[k]->data());
                sl[k] = (uint32_t)fs[k]->size();
            }
            std::vector<uint8_t> exp(orc_order_json_one(sp, sl, o.customer_id, o.timestamp, o.quantity, 0, nullptr));
            orc_order_json_one(sp, sl, o.customer_id, o.timestamp, o.quantity, 0, exp.data());
            CHECK(got == std::string(exp.begin(), exp.end()));
        }
    }
    {  // MessageHandler::handleMessage prints the whole std::string (src/message_handler.cpp:10-16)
        MessageHandler mh;
        ParseResult pr;
        pr.success = true;
        pr.message_type = std::string("CREATE\0ORDER", 12);
        std::ostringstream cap;
        std::streambuf* old = std::cout.rdbuf(cap.rdbuf());
        mh.handleMessage(pr);
        pr.success = false;
        pr.error_message = std::string("bad\0tail", 8);
        mh.handleMessage(pr);
        std::cout.rdbuf(old);
        const std::string want = std::string("[MessageHandler] Handled message: ") + std::string("CREATE\0ORDER", 12) +
                                 "\n[MessageHandler] Failed to handle message: " + std::string("bad\0tail", 8) + "\n";
        CHECK(cap.str() == want);
    }
    {  // ClusterClient::publish_topic's encoder block (src/cluster_client.cpp:1809-1864)
        std::vector<std::vector<uint8_t>> sent;
        TopicPublisher pub([&](const uint8_t* d, size_t n) {
            sent.emplace_back(d, d + n);
            return true;
        });
        const std::string big(70000, 'P');
        const std::string uuid = pub.publish_topic("orders", "CREATE_ORDER", big, "");
        CHECK(uuid.rfind("pub_", 0) == 0 && uuid.size() > 20);
        CHECK(sent.size() == 1);
        // expected: the oracle with the uuid and timestamp the record carries
        const std::vector<uint8_t>& r = sent[0];
        uint64_t ts = 0;
        for (int i = 7; i >= 0; --i) ts = (ts << 8) | r[8 + i];
        const std::string hd = "{}";
        const std::string tp = "orders", ty = "CREATE_ORDER";
        const uint8_t* sp[5] = {(const uint8_t*)tp.data(), (const uint8_t*)ty.data(), (const uint8_t*)uuid.data(),
                                (const uint8_t*)big.data(), (const uint8_t*)hd.data()};
        const uint32_t sl[5] = {(uint32_t)tp.size(), (uint32_t)ty.size(), (uint32_t)uuid.size(), (uint32_t)big.size(),
                                (uint32_t)hd.size()};
        std::vector<uint8_t> exp(34 + 6 + 12 + uuid.size() + (70000 - 65536) + 2);
        uint8_t st = 9;
        const uint64_t m = orc_encode_one(sp, sl, ts, SBE_ENC_PUBLISH_TOPIC, exp.data(), &st);
        CHECK(st == 0 && m == exp.size() && r == exp);
        CHECK(ts > 1700000000000000000ULL);
        std::vector<TopicMessageFields> msgs(50);
        for (auto& x : msgs) x = TopicMessageFields{"orders", "UPDATE_ORDER", "ignored", "{\"a\":1}", "{\"h\":1}", 0};
        sent.clear();
        const auto ids = pub.publish_topic_batch(msgs);
        CHECK(ids.size() == 50 && sent.size() == 50 && sent[49].size() == 34 + 6 + 12 + ids[49].size() + 7 + 7);
    }
    surface_tests(f5, wire, sack, ack45);
    std::printf("host api test: %s (%d failures)\n", failures ? "FAILED" : "ok", failures);
    return failures ? 1 : 0;
}
