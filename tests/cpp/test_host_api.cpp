// GPU test of the C++ host mirror (aeron-cluster-client-cpp_amd/host): the reference-shaped API
// against SURVEY Appendix B probe observations and against the oracle (oracle/liboracle.so).
#include <cfloat>
#include <cstdio>
#include <cstring>
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
    std::printf("host api test: %s (%d failures)\n", failures ? "FAILED" : "ok", failures);
    return failures ? 1 : 0;
}
