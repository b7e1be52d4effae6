// CPU test of the host mirror's SBEDecoder / SBEEncoder::get_current_timestamp (no device needed:
// these are the reference's one-record struct readers, src/sbe_encoder.cpp:169-323) against
// hand-built probes and the oracle restatement (orc_sbedecoder_*, oracle/sbe_oracle.c), on
// random and mutated records.
#include <chrono>
#include <cstdio>
#include <cstring>
#include <random>
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

static void put_le(std::vector<uint8_t>& b, uint64_t v, int bytes) {
    for (int i = 0; i < bytes; ++i) b.push_back((uint8_t)(v >> (8 * i)));
}
static void put_str32(std::vector<uint8_t>& b, const std::string& s) {
    put_le(b, s.size(), 4);
    b.insert(b.end(), s.begin(), s.end());
}
static std::vector<uint8_t> hdr(uint16_t blk, uint16_t tmpl, uint16_t schema, uint16_t ver) {
    std::vector<uint8_t> b;
    put_le(b, blk, 2), put_le(b, tmpl, 2), put_le(b, schema, 2), put_le(b, ver, 2);
    return b;
}
static std::vector<uint8_t> session_event(const std::string* detail, int64_t corr = 0x1122334455667788LL) {
    std::vector<uint8_t> b = hdr(32, 2, 111, 8);
    put_le(b, (uint64_t)corr, 8), put_le(b, 5, 8), put_le(b, 6, 8), put_le(b, 1, 4), put_le(b, 2, 4);
    if (detail) put_str32(b, *detail);
    return b;
}
static std::vector<uint8_t> ack32(int64_t ts, const std::vector<std::string>& f) {
    std::vector<uint8_t> b = hdr(8, 2, 1, 1);
    put_le(b, (uint64_t)ts, 8);
    for (auto& s : f) put_str32(b, s);
    return b;
}

static const std::string kSentinel = "SENTINEL-unchanged";

// mirror vs oracle on one record
static void cmp_session(const std::vector<uint8_t>& r, size_t len) {
    SessionEvent ev{};
    std::string detail = kSentinel;
    const bool ok = SBEDecoder::decode_session_event(r.empty() ? nullptr : r.data(), len, ev, detail);
    uint32_t off = 0, dl = 0, got = 0;
    const int ook = orc_sbedecoder_session_event(r.empty() ? nullptr : r.data(), len, &off, &dl, &got);
    CHECK(ok == (ook == 1));
    if (!ok || ook != 1) {
        CHECK(detail == kSentinel);
        return;
    }
    CHECK(std::memcmp(&ev, r.data() + 8, 32) == 0);
    if (got)
        CHECK(detail == std::string(reinterpret_cast<const char*>(r.data()) + off, dl));
    else
        CHECK(detail == kSentinel);
}

static void cmp_ack(const std::vector<uint8_t>& r, size_t len) {
    std::string s[3] = {kSentinel, kSentinel, kSentinel};
    int64_t ts = -7;
    const bool ok = SBEDecoder::decode_acknowledgment(r.empty() ? nullptr : r.data(), len, s[0], s[1], s[2], ts);
    uint32_t off[3] = {0, 0, 0}, sl[3] = {0, 0, 0}, got = 0;
    int64_t ots = -7;
    const int ook = orc_sbedecoder_ack(r.empty() ? nullptr : r.data(), len, off, sl, &got, &ots);
    CHECK(ok == (ook == 1));
    CHECK(ts == ((got & 8) ? ots : -7));
    for (int k = 0; k < 3; ++k) {
        if (got & (1u << k))
            CHECK(s[k] == std::string(reinterpret_cast<const char*>(r.data()) + off[k], sl[k]));
        else
            CHECK(s[k] == kSentinel);
    }
}

int main() {
    // ---- SBEEncoder::get_current_timestamp (src/sbe_encoder.cpp:169-172): high_resolution_clock
    // ticks (nanoseconds since the epoch with libstdc++)
    {
        const int64_t a = SBEEncoder::get_current_timestamp();
        const int64_t sys = (int64_t)std::chrono::duration_cast<std::chrono::nanoseconds>(
                                std::chrono::system_clock::now().time_since_epoch())
                                .count();
        const int64_t b = SBEEncoder::get_current_timestamp();
        CHECK(a > 1700000000000000000LL && b >= a);
        CHECK(sys - a < 1000000000LL && a - sys < 1000000000LL);
    }
    // ---- decode_message_header (:174-181)
    {
        const std::vector<uint8_t> h = hdr(48, 1, 1, 1);
        MessageHeader m{};
        CHECK(SBEDecoder::decode_message_header(h.data(), 8, m) && m.block_length == 48 && m.template_id == 1 &&
              m.schema_id == 1 && m.version == 1);
        MessageHeader u{7, 7, 7, 7};
        CHECK(!SBEDecoder::decode_message_header(h.data(), 7, u) && u.block_length == 7);
        CHECK(!SBEDecoder::decode_message_header(nullptr, 8, u));
    }
    // ---- decode_session_event probes (:183-238, :285-318)
    {
        const std::string d = "10.0.0.2:9002";
        auto r = session_event(&d);
        SessionEvent ev{};
        std::string detail = "old";
        CHECK(SBEDecoder::decode_session_event(r.data(), r.size(), ev, detail));
        CHECK(ev.correlation_id == 0x1122334455667788LL && ev.cluster_session_id == 5 && ev.leadership_term_id == 6 &&
              ev.leader_member_id == 1 && ev.code == 2 && detail == d);
        const std::string empty;
        auto r0 = session_event(&empty);  // length 0: the detail is cleared
        detail = "old";
        CHECK(SBEDecoder::decode_session_event(r0.data(), r0.size(), ev, detail) && detail.empty());
        auto rn = session_event(nullptr);  // no bytes after the block: detail untouched
        detail = "old";
        CHECK(SBEDecoder::decode_session_event(rn.data(), rn.size(), ev, detail) && detail == "old");
        auto r2 = rn;
        r2.push_back(1), r2.push_back(2);  // 2 bytes: no room for the u32 prefix, untouched
        CHECK(SBEDecoder::decode_session_event(r2.data(), r2.size(), ev, detail) && detail == "old");
        auto rl = session_event(&d);  // the prefix says more than the record holds: untouched
        rl.resize(rl.size() - 1);
        CHECK(SBEDecoder::decode_session_event(rl.data(), rl.size(), ev, detail) && detail == "old");
        CHECK(!SBEDecoder::decode_session_event(r.data(), 39, ev, detail));  // below 40 bytes
        auto rt = r;
        rt[2] = 1;  // template 1
        CHECK(!SBEDecoder::decode_session_event(rt.data(), rt.size(), ev, detail));
        auto rs = r;
        rs[4] = 1;  // schema 1
        CHECK(!SBEDecoder::decode_session_event(rs.data(), rs.size(), ev, detail));
    }
    // ---- decode_acknowledgment probes (:240-282)
    {
        auto r = ack32(1700000000000LL, {"msg_1", "OK", "none"});
        std::string id, st, er = "old";
        int64_t ts = 0;
        CHECK(SBEDecoder::decode_acknowledgment(r.data(), r.size(), id, st, er, ts));
        CHECK(id == "msg_1" && st == "OK" && er == "none" && ts == 1700000000000LL);
        auto r2 = ack32(5, {"msg_2", "FAIL"});  // no error field: untouched
        er = "old";
        CHECK(SBEDecoder::decode_acknowledgment(r2.data(), r2.size(), id, st, er, ts) && id == "msg_2" && st == "FAIL" &&
              er == "old" && ts == 5);
        auto r1 = ack32(9, {"only"});  // status missing: false, messageId already assigned
        id = st = "old";
        CHECK(!SBEDecoder::decode_acknowledgment(r1.data(), r1.size(), id, st, er, ts) && id == "only" && st == "old" &&
              ts == 9);
        CHECK(!SBEDecoder::decode_acknowledgment(r.data(), 15, id, st, er, ts));
        // a status length that passes the reference's `remaining - 4` check but runs past the
        // record: refused, nothing read past the end
        {
            auto ro = ack32(11, {"msg_3", "OK"});
            const size_t status_prefix = 16 + 4 + 5;   // header 8 + block 8, messageId prefix + bytes
            const uint32_t bad = (uint32_t)(ro.size() - 16 - 4);  // <= remaining - 4, > remaining - offset
            std::memcpy(ro.data() + status_prefix, &bad, 4);
            id = st = "old";
            CHECK(!SBEDecoder::decode_acknowledgment(ro.data(), ro.size(), id, st, er, ts) && id == "msg_3" &&
                  st == "old");
            cmp_ack(ro, ro.size());
        }
        auto rt = r;
        rt[2] = 1;
        ts = 3;
        CHECK(!SBEDecoder::decode_acknowledgment(rt.data(), rt.size(), id, st, er, ts) && ts == 3);
        // the heuristic-layout Ack (u16 prefixes) parse_message decodes is not this layout
        std::vector<uint8_t> u16ack = hdr(8, 2, 1, 1);
        put_le(u16ack, 1, 8);
        for (std::string s : {"msg_1", "orders", "corr"}) {
            put_le(u16ack, s.size(), 2);
            u16ack.insert(u16ack.end(), s.begin(), s.end());
        }
        cmp_ack(u16ack, u16ack.size());
    }
    // ---- random and mutated records vs the oracle restatement
    std::mt19937_64 rng(20261017);
    auto rstr = [&](size_t maxlen) {
        std::string s(rng() % (maxlen + 1), ' ');
        for (auto& c : s) c = (char)(rng() % 256);
        return s;
    };
    for (int it = 0; it < 20000; ++it) {
        std::vector<uint8_t> r;
        const int kind = (int)(rng() % 4);
        if (kind == 0) {
            const std::string d = rstr(40);
            r = session_event(rng() % 4 ? &d : nullptr);
        } else if (kind == 1) {
            std::vector<std::string> f;
            const int nf = (int)(rng() % 4);
            for (int k = 0; k < nf; ++k) f.push_back(rstr(30));
            r = ack32((int64_t)rng(), f);
        } else {  // random bytes behind a plausible header
            r = hdr((uint16_t)(rng() % 64), (uint16_t)(rng() % 4), rng() % 2 ? 111 : 1, (uint16_t)(rng() % 9));
            const size_t extra = rng() % 96;
            for (size_t k = 0; k < extra; ++k) r.push_back((uint8_t)(rng() % 256));
        }
        // mutations: a length prefix byte, a header byte, the record's length
        if (!r.empty() && rng() % 3 == 0) r[rng() % r.size()] ^= (uint8_t)(1u << (rng() % 8));
        if (r.size() > 44 && rng() % 4 == 0) r[40 + rng() % 4] = (uint8_t)(rng() % 256);
        size_t len = r.size();
        if (len && rng() % 3 == 0) len = rng() % (len + 1);
        cmp_session(r, len);
        cmp_ack(r, len);
        if (failures > 20) break;
    }
    cmp_session({}, 0);
    cmp_ack({}, 0);
    // BatchingParser without a device (this binary runs on the CPU): refused at construction with
    // the mirror's exception, as every entry point of the mirror is
    if (!gpu_codec_available()) {
        bool threw = false;
        try {
            BatchingParser bp([](const ParseResult&) {});
        } catch (const std::runtime_error& e) {
            threw = std::strstr(e.what(), "gfx950") != nullptr;
        }
        CHECK(threw);
    }
    std::printf("sbedecoder test: %s (%d failures)\n", failures ? "FAILED" : "ok", failures);
    return failures ? 1 : 0;
}
