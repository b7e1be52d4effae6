// GPU test of the host mirror's batch pipeline (aeron-cluster-client-cpp_amd/host): batches of
// distinct variable-length records past one pipeline chunk (65536 records), through every batch
// entry point, from pageable and from page-locked (host_register) memory, against the oracle
// restatement record by record.  Run it with AERON_AMD_CHUNK_BYTES small (many chunks cycling the
// 3-slot ring) and with the defaults (a few chunks; one-chunk batches on the zero-copy path):
// tests/test_gpu_host_api.py does both.  ADVICE r3: per-chunk offset rebasing, descriptor
// indexing, cross-stream event order and the on_chunk overlap.
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>
#include <stdexcept>
#include <string>
#include <vector>

#include "aeron_cluster_amd.hpp"
#include "../../oracle/sbe_oracle.h"

using namespace aeron_cluster;

static int failures = 0;
#define CHECK(c)                                                                   \
    do {                                                                           \
        if (!(c)) {                                                                \
            if (failures < 30) std::fprintf(stderr, "FAIL %s:%d: %s\n", __FILE__, __LINE__, #c); \
            ++failures;                                                            \
        }                                                                          \
    } while (0)

struct Recs {
    std::vector<std::vector<std::string>> f;  // [n][5]
    std::vector<uint64_t> ts;
    std::vector<uint8_t> arena;  // packed, for the oracle
    std::vector<uint32_t> len;
};

static Recs make(size_t n, uint64_t seed) {
    Recs r;
    std::mt19937_64 rng(seed);
    r.f.resize(n);
    for (size_t i = 0; i < n; ++i) {
        for (int k = 0; k < 5; ++k) {
            const size_t L = rng() % (k == 3 ? 300 : 40);
            std::string s(L, ' ');
            for (auto& c : s) c = (char)(32 + rng() % 95);
            if (k == 3 && i % 97 == 0 && L > 40) s.replace(5, 21, "\"_sequence_number\":" + std::to_string(i % 10) + ",");
            r.arena.insert(r.arena.end(), s.begin(), s.end());
            r.len.push_back((uint32_t)s.size());
            r.f[i].push_back(std::move(s));
        }
        r.ts.push_back(rng() | 1);
    }
    return r;
}

static std::vector<TopicMessageFields> fields(const Recs& r) {
    std::vector<TopicMessageFields> m;
    for (size_t i = 0; i < r.f.size(); ++i)
        m.push_back({r.f[i][0], r.f[i][1], r.f[i][2], r.f[i][3], r.f[i][4], (int64_t)r.ts[i]});
    return m;
}

// the oracle's parse_message descriptor of every record, and sequence numbers
struct Want {
    std::vector<uint8_t> st, fl;
    std::vector<uint16_t> hdr;
    std::vector<uint64_t> ts, seq;
    std::vector<uint32_t> vo, vl;
};
static Want oracle_parse(const uint8_t* data, const uint64_t* off, size_t n) {
    Want w;
    w.st.resize(n), w.fl.resize(n), w.hdr.resize(4 * n), w.ts.resize(n), w.seq.assign(n, 0), w.vo.resize(5 * n),
        w.vl.resize(5 * n);
    orc_decode_batch(data, off, n, SBE_DEC_PARSE_MESSAGE, w.st.data(), w.fl.data(), w.hdr.data(), w.ts.data(), w.vo.data(),
                     w.vl.data(), 8);
    orc_seq_batch(data, off, n, w.st.data(), w.fl.data(), w.vo.data(), w.vl.data(), w.seq.data(), 8);
    return w;
}

// ParseResult of record i against the oracle descriptor (TopicMessage / Ack / error records)
static bool matches(const ParseResult& r, const uint8_t* rec, const Want& w, size_t i) {
    const uint8_t st = w.st[i];
    auto v = [&](int k) { return std::string(reinterpret_cast<const char*>(rec) + w.vo[5 * i + k], w.vl[5 * i + k]); };
    if (st == SBE_ST_TM)
        return r.success && r.message_type == v(1) && r.message_id == v(2) && r.payload == v(3) && r.headers == v(4) &&
               (uint64_t)r.timestamp == w.ts[i] && r.sequence_number == w.seq[i] && r.template_id == w.hdr[4 * i + 1];
    if (st == SBE_ST_ACK) {
        const std::string id = (w.fl[i] & SBE_FL_ID_DEFAULT) ? "ack_" + std::to_string(w.ts[i]) : v(0);
        const std::string pay = (w.fl[i] & SBE_FL_PAYLOAD_DEFAULT) ? std::string("SUCCESS") : v(1);
        return r.success && r.message_type == "Acknowledgment" && r.message_id == id && r.payload == pay &&
               r.headers == v(2) && (uint64_t)r.timestamp == w.ts[i];
    }
    return !r.success && !r.error_message.empty();
}

static void check_parse(const char* what, const uint8_t* data, const uint64_t* off, size_t n, const Want& w,
                        const uint8_t* rec_base) {
    const int f0 = failures;
    // fresh vector, reused vector (twice: the second call rewrites in place), views, for_each
    const auto fresh = MessageParser::parse_batch(data, off, n);
    std::vector<ParseResult> reuse(7);
    MessageParser::parse_batch(data, off, n, reuse);
    MessageParser::parse_batch(data, off, n, reuse);
    const ParsedBatch pb = MessageParser::decode_batch(data, off, n);
    CHECK(fresh.size() == n && reuse.size() == n && pb.size() == n);
    for (size_t i = 0; i < n && failures - f0 < 10; ++i) {
        const uint8_t* rec = rec_base + off[i];
        CHECK(matches(fresh[i], rec, w, i));
        CHECK(matches(reuse[i], rec, w, i));
        CHECK(pb.status(i) == w.st[i]);
        if (w.st[i] == SBE_ST_TM) {
            CHECK(pb.view(i, 3) == std::string_view(reinterpret_cast<const char*>(rec) + w.vo[5 * i + 3], w.vl[5 * i + 3]));
            CHECK(pb.sequence_number(i) == w.seq[i]);
        }
        if (i % 4099 == 0) CHECK(matches(pb.result(i), rec, w, i));
    }
    size_t seen = 0;
    pb.for_each([&](size_t i, const ParseResult& r) {
        if (i != seen || (i % 1013 == 0 && !matches(r, rec_base + off[i], w, i))) ++failures;
        ++seen;
    });
    CHECK(seen == n);
    std::printf("  %-44s n=%zu %s\n", what, n, failures == f0 ? "ok" : "FAIL");
}

int main() {
    if (!gpu_codec_available()) {
        std::fprintf(stderr, "no gfx950 device\n");
        return 2;
    }
    const char* cb = std::getenv("AERON_AMD_CHUNK_BYTES");
    std::printf("host pipeline test, AERON_AMD_CHUNK_BYTES=%s AERON_AMD_ZC_BYTES=%s\n", cb ? cb : "(default)",
                std::getenv("AERON_AMD_ZC_BYTES") ? std::getenv("AERON_AMD_ZC_BYTES") : "(default)");
    for (size_t n : {1, 300, 5000, 70000, 150001}) {
        const Recs R = make(n, 0x9e37 + n);
        const auto msgs = fields(R);
        for (auto len : {EncodeLength::Wire, EncodeLength::Reference}) {
            const int f0 = failures;
            const uint32_t flags = len == EncodeLength::Reference ? SBE_ENC_REF_TRUNCATE8 : 0u;
            std::vector<uint8_t> eo(R.arena.size() + 34 * n + 16);
            std::vector<uint64_t> eoff(n + 1);
            std::vector<uint8_t> est(n);
            orc_encode_batch(R.arena.data(), nullptr, R.len.data(), R.ts.data(), n, 0, flags, eo.data(), eoff.data(),
                             est.data(), 8);
            const EncodedBatch b = SBEEncoder::encode_topic_batch(msgs, len);
            CHECK(b.offsets == eoff);
            CHECK(b.status == est);
            CHECK(b.bytes.size() == eoff[n] && std::memcmp(b.bytes.data(), eo.data(), eoff[n]) == 0);
            std::printf("  encode %-37s n=%zu %s\n", len == EncodeLength::Wire ? "wire" : "reference", n,
                        failures == f0 ? "ok" : "FAIL");
            if (len != EncodeLength::Wire) continue;
            // parse: from the encoder's page-locked result (direct), from a pageable copy (staged)
            const Want w = oracle_parse(eo.data(), eoff.data(), n);
            check_parse("parse, page-locked input (EncodedBatch)", b.bytes.data(), b.offsets.data(), n, w, b.bytes.data());
            std::vector<uint8_t> pageable(eo.begin(), eo.begin() + eoff[n]);
            check_parse("parse, pageable input", pageable.data(), eoff.data(), n, w, pageable.data());
            // a sub-range starting mid-buffer in host_register'd memory (rec_off[0] > 0)
            if (n >= 300) {
                const size_t a = n / 3, m = n - a;
                std::vector<uint8_t> reg(pageable);
                reg.resize(reg.size() + 4096);
                host_register(reg.data(), reg.size());
                Want ws;
                ws.st.assign(w.st.begin() + a, w.st.end());
                ws.fl.assign(w.fl.begin() + a, w.fl.end());
                ws.hdr.assign(w.hdr.begin() + 4 * a, w.hdr.end());
                ws.ts.assign(w.ts.begin() + a, w.ts.end());
                ws.seq.assign(w.seq.begin() + a, w.seq.end());
                ws.vo.assign(w.vo.begin() + 5 * a, w.vo.end());
                ws.vl.assign(w.vl.begin() + 5 * a, w.vl.end());
                check_parse("parse, registered input, records [n/3, n)", reg.data(), eoff.data() + a, m, ws, reg.data());
                host_unregister(reg.data());
            }
            // on_egress_batch: every record is a wire TopicMessage with 8 bytes of slack after it
            // (MessageHandler's E100 rule wants them, message_handler.hpp:47-50)
            std::vector<uint8_t> eg;
            std::vector<uint64_t> egoff{0};
            for (size_t i = 0; i < n; ++i) {
                eg.insert(eg.end(), eo.begin() + eoff[i], eo.begin() + eoff[i + 1]);
                eg.resize(eg.size() + 8, 0);
                egoff.push_back(eg.size());
            }
            // the callbacks on_egress makes, from the oracle's on_egress descriptors (EG_TM records,
            // in order, up to the first record where the reference throws)
            std::vector<uint8_t> est2(n), efl(n);
            std::vector<uint16_t> eh(4 * n);
            std::vector<uint64_t> ets(n);
            std::vector<uint32_t> evo(5 * n), evl(5 * n);
            orc_decode_batch(eg.data(), egoff.data(), n, SBE_DEC_ON_EGRESS, est2.data(), efl.data(), eh.data(), ets.data(),
                             evo.data(), evl.data(), 8);
            std::vector<size_t> cb_rec;
            bool want_throw = false;
            for (size_t i = 0; i < n && !want_throw; ++i) {
                if (est2[i] == SBE_ST_EG_TM) cb_rec.push_back(i);
                want_throw = est2[i] == SBE_ST_EG_THROW_E100;
            }
            MessageHandler h;
            size_t j = 0;
            int bad = 0;
            h.set_topic_message_callback([&](std::string_view t, std::string_view y, std::string_view u, std::string_view p,
                                             std::string_view hd) {
                if (j < cb_rec.size()) {
                    const size_t i = cb_rec[j];
                    const char* rec = reinterpret_cast<const char*>(eg.data()) + egoff[i];
                    const std::string_view got[5] = {t, y, u, p, hd};
                    for (int q = 0; q < 5; ++q)
                        if (got[q] != std::string_view(rec + evo[5 * i + q], evl[5 * i + q])) ++bad;
                }
                ++j;
            });
            bool threw = false;
            try {
                h.on_egress_batch(eg.data(), egoff.data(), n);
            } catch (const std::runtime_error& e) {
                threw = std::string(e.what()) == "buffer too short [E100]";
            }
            const size_t expect_cb = cb_rec.size();
            CHECK(threw == want_throw);
            CHECK(j == expect_cb && bad == 0);
            std::printf("  %-44s n=%zu %s\n", "on_egress_batch", n, (j == expect_cb && bad == 0) ? "ok" : "FAIL");
        }
        std::fflush(stdout);
        if (failures > 50) break;
    }
    std::printf("host pipeline test: %s (%d failures)\n", failures ? "FAILED" : "ok", failures);
    return failures ? 1 : 0;
}
