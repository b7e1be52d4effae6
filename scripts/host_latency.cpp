// host_latency.cpp — per-call latency of the drop-in C++ mirror (host memory in, host memory out)
// against the CPU restatement, for the reference's per-fragment call site
// (MessageParser::parse_message at src/cluster_client.cpp:1185, one call per Aeron fragment) and
// for batches.  Prints one JSON line per (operation, batch size): mirror µs per call, µs per record,
// the oracle's µs per record on one host thread, and whether the GPU path is ahead.
// Build + run (GPU box): make -C scripts host_latency && scripts/host_latency
#include <chrono>
#include <cstdint>
#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include <hip/hip_runtime.h>

#include "aeron_cluster_amd.hpp"
#include "sbecodec.h"
#include "../oracle/sbe_oracle.h"

using namespace aeron_cluster;
using clk = std::chrono::steady_clock;

static double us_since(clk::time_point t0) {
    return std::chrono::duration<double, std::micro>(clk::now() - t0).count();
}

int main(int argc, char** argv) {
    // optional: one batch size only (profiling runs), skipping the single-call section
    const size_t only = argc > 1 ? (size_t)std::strtoull(argv[1], nullptr, 10) : 0;
    if (!gpu_codec_available()) {
        std::fprintf(stderr, "no gfx950 device\n");
        return 2;
    }
    const std::string topic = "orders", type = "CREATE_ORDER", uuid = "msg_1760000000000000000_00042";
    const std::string payload(143, 'p'), headers(32, 'h');
    // warm up the device context
    for (int i = 0; i < 20; ++i) (void)SBEEncoder::encode_topic_message(topic, type, uuid, payload, headers, 1);
    const std::vector<uint8_t> rec = SBEEncoder::encode_topic_batch(
        {TopicMessageFields{topic, type, uuid, payload, headers, 1760000000000000000LL}}, EncodeLength::Wire).bytes.to_vector();

    // single-record calls: the reference's per-call surface
    if (!only) {
        const int iters = 2000;
        auto t0 = clk::now();
        for (int i = 0; i < iters; ++i) (void)SBEEncoder::encode_topic_message(topic, type, uuid, payload, headers, 1);
        const double enc = us_since(t0) / iters;
        t0 = clk::now();
        for (int i = 0; i < iters; ++i) (void)MessageParser::parse_message(rec.data(), rec.size());
        const double par = us_since(t0) / iters;
        t0 = clk::now();
        for (int i = 0; i < iters; ++i) (void)decode_ack(rec.data(), rec.size());
        const double ack = us_since(t0) / iters;
        std::printf("{\"op\": \"single_call\", \"encode_topic_message_us\": %.2f, \"parse_message_us\": %.2f, "
                    "\"decode_ack_us\": %.2f}\n", enc, par, ack);
    }
    // the serve kernel through the C ABI alone (no mirror): an empty request (a round trip and one
    // store), one record decoded from host memory, one record encoded from host memory; outputs in
    // page-locked memory through their device addresses
    if (!only) {
        sbe_server* srv = nullptr;
        if (sbe_server_create(&srv, 0) == SBE_OK) {
            void* pin = nullptr;
            (void)hipHostMalloc(&pin, 1 << 16, hipHostMallocDefault);
            void* dpin = nullptr;
            (void)hipHostGetDevicePointer(&dpin, pin, 0);
            uint8_t* d = static_cast<uint8_t*>(dpin);
            const uint64_t ro[2] = {0, rec.size()};
            sbe_decoded out{d, d + 64, reinterpret_cast<uint16_t*>(d + 128), reinterpret_cast<uint64_t*>(d + 192),
                            reinterpret_cast<uint32_t*>(d + 256), reinterpret_cast<uint32_t*>(d + 320),
                            reinterpret_cast<uint64_t*>(d + 384)};
            std::vector<uint8_t> arena;
            for (const std::string* f : {&topic, &type, &uuid, &payload, &headers}) arena.insert(arena.end(), f->begin(), f->end());
            const uint32_t lens[5] = {(uint32_t)topic.size(), (uint32_t)type.size(), (uint32_t)uuid.size(),
                                      (uint32_t)payload.size(), (uint32_t)headers.size()};
            const uint64_t ts1 = 1;
            sbe_tm_batch tb{arena.data(), nullptr, lens, &ts1};
            sbe_tm_batch t0{nullptr, nullptr, nullptr, nullptr};
            const int iters = 4000;
            auto bench = [&](auto&& f) {
                for (int i = 0; i < 200; ++i) f();
                const auto t0c = clk::now();
                for (int i = 0; i < iters; ++i) f();
                return us_since(t0c) / iters;
            };
            const double ping = bench([&] {
                (void)sbe_serve_encode_topic(srv, &t0, 0, 0, 0, d + 4096, 0, reinterpret_cast<uint64_t*>(d + 8192), nullptr);
            });
            const double dec1 = bench([&] { (void)sbe_serve_decode_host(srv, rec.data(), ro, 1, SBE_DEC_PARSE_MESSAGE, &out); });
            const double enc1 = bench([&] {
                (void)sbe_serve_encode_topic_host(srv, &tb, 1, 0, 0, d + 4096, 4096, reinterpret_cast<uint64_t*>(d + 8192),
                                                  d + 8256);
            });
            std::printf("{\"op\": \"serve_abi\", \"empty_request_us\": %.2f, \"decode_1_host_us\": %.2f, "
                        "\"encode_1_host_us\": %.2f}\n", ping, dec1, enc1);
            (void)sbe_server_destroy(srv);
            (void)hipHostFree(pin);
        }
    }
    // batches: mirror (stage + H2D + kernels + D2H, pipelined over two streams) vs the oracle on
    // one thread.  decode = MessageParser::decode_batch (device descriptors + views, ParseResults on
    // demand); parse = MessageParser::parse_batch (every ParseResult built, and destroyed by the
    // next iteration, inside the timing)
    for (size_t n : {1, 4, 16, 64, 256, 1024, 4096, 16384, 65536, 262144, 1048576}) {
        if (only && n != only) continue;
        std::vector<TopicMessageFields> msgs(n, TopicMessageFields{topic, type, uuid, payload, headers, 1760000000000000000LL});
        const int reps = n <= 1024 ? 200 : (n <= 16384 ? 40 : (n <= 262144 ? 10 : 4));
        // warm-up: the page-locked pool allocates each block size once (hipHostMalloc costs
        // milliseconds); a caller that keeps one result while making the next needs two sets
        EncodedBatch b = SBEEncoder::encode_topic_batch(msgs, EncodeLength::Wire);
        for (int w = 0; w < 2; ++w) b = SBEEncoder::encode_topic_batch(msgs, EncodeLength::Wire);
        auto t0 = clk::now();
        double enc_drop = 0, enc_call = 0;  // of which: the call itself, releasing the previous batch
        for (int r = 0; r < reps; ++r) {
            const auto tc = clk::now();
            EncodedBatch nb = SBEEncoder::encode_topic_batch(msgs, EncodeLength::Wire);
            enc_call += us_since(tc);
            const auto td = clk::now();
            b = std::move(nb);
            enc_drop += us_since(td);
        }
        const double enc = us_since(t0) / reps;
        enc_drop /= reps;
        enc_call /= reps;
        ParsedBatch pb = MessageParser::decode_batch(b.bytes.data(), b.offsets.data(), n);
        for (int w = 0; w < 2; ++w) pb = MessageParser::decode_batch(b.bytes.data(), b.offsets.data(), n);
        t0 = clk::now();
        for (int r = 0; r < reps; ++r) pb = MessageParser::decode_batch(b.bytes.data(), b.offsets.data(), n);
        const double dec = us_since(t0) / reps;
        std::vector<ParseResult> prs = MessageParser::parse_batch(b.bytes.data(), b.offsets.data(), n);
        prs = MessageParser::parse_batch(b.bytes.data(), b.offsets.data(), n);
        t0 = clk::now();
        for (int r = 0; r < reps; ++r) prs = MessageParser::parse_batch(b.bytes.data(), b.offsets.data(), n);
        const double par = us_since(t0) / reps;
        // parse into one reused vector (the ParseResults keep their string buffers across calls)
        std::vector<ParseResult> reuse;
        MessageParser::parse_batch(b.bytes.data(), b.offsets.data(), n, reuse);
        MessageParser::parse_batch(b.bytes.data(), b.offsets.data(), n, reuse);
        t0 = clk::now();
        for (int r = 0; r < reps; ++r) MessageParser::parse_batch(b.bytes.data(), b.offsets.data(), n, reuse);
        const double par_reuse = us_since(t0) / reps;
        bool ok = reuse.size() == n && reuse[n - 1].payload == payload && reuse[0].message_id == uuid &&
                  prs.size() == n && pb.size() == n && prs[n - 1].success && prs[n - 1].payload == payload &&
                  pb.view(n - 1, 2) == uuid && b.offsets[n] == 256 * n;
        // oracle (CPU restatement, 1 thread) on the same records
        std::vector<uint8_t> arena;
        std::vector<uint32_t> lens;
        std::vector<uint64_t> ts(n, 1760000000000000000ULL);
        for (size_t i = 0; i < n; ++i)
            for (const std::string* f : {&topic, &type, &uuid, &payload, &headers}) {
                arena.insert(arena.end(), f->begin(), f->end());
                lens.push_back((uint32_t)f->size());
            }
        std::vector<uint8_t> out(b.bytes.size() + 64), st(n), dst(n), dfl(n);
        std::vector<uint64_t> off(n + 1), dts(n);
        std::vector<uint16_t> dh(4 * n);
        std::vector<uint32_t> vo(5 * n), vl(5 * n);
        const int creps = std::max(1, reps / 2);
        t0 = clk::now();
        for (int r = 0; r < creps; ++r)
            orc_encode_batch(arena.data(), nullptr, lens.data(), ts.data(), n, 0, 0, out.data(), off.data(), st.data(), 1);
        const double cenc = us_since(t0) / creps;
        t0 = clk::now();
        for (int r = 0; r < creps; ++r)
            orc_decode_batch(out.data(), off.data(), n, SBE_DEC_PARSE_MESSAGE, dst.data(), dfl.data(), dh.data(),
                             dts.data(), vo.data(), vl.data(), 1);
        const double cdec = us_since(t0) / creps;
        ok = ok && std::memcmp(out.data(), b.bytes.data(), b.bytes.size()) == 0;
        std::printf("{\"op\": \"batch\", \"records\": %zu, \"mirror_encode_us\": %.1f, \"mirror_decode_us\": %.1f, "
                    "\"mirror_parse_us\": %.1f, \"oracle_encode_us\": %.1f, \"oracle_parse_us\": %.1f, "
                    "\"mirror_enc_dec_rec_per_s\": %.4g, \"mirror_enc_parse_rec_per_s\": %.4g, \"oracle_rec_per_s\": %.4g, "
                    "\"gpu_ahead\": %s, \"bytes_ok\": %s, \"encode_release_us\": %.1f, \"encode_call_us\": %.1f, "
                    "\"mirror_parse_reuse_us\": %.1f, \"mirror_enc_parse_reuse_rec_per_s\": %.4g, \"host_threads\": %u}\n",
                    n, enc, dec, par, cenc, cdec, n / ((enc + dec) * 1e-6), n / ((enc + par) * 1e-6),
                    n / ((cenc + cdec) * 1e-6), (enc + dec) < (cenc + cdec) ? "true" : "false", ok ? "true" : "false", enc_drop, enc_call,
                    par_reuse, n / ((enc + par_reuse) * 1e-6), host_threads());
        std::fflush(stdout);
    }
    return 0;
}
