// batching_parser_bench.cpp — the reference's call granularity through the mirror: fragments
// arrive one at a time in polls of up to 100 (include/aeron_cluster/performance_config.hpp:17;
// handle_incoming_message parses each, src/cluster_client.cpp:1185).  Compares, on the same 1 M
// fixed-256 TopicMessages:
//   per_fragment      MessageParser::parse_message once per fragment (the drop-in as the reference
//                     calls it: one serve-kernel round trip per call)
//   batching_parser   BatchingParser (host/aeron_cluster_amd.hpp): fragments copied into a
//                     page-locked batch, decoded by its decode thread while the next batch fills,
//                     handlers run on the polling thread at poll()
//   oracle_1thread    the CPU restatement's decode of the same records on one thread (what one
//                     host thread of the reference-equivalent C path sustains)
// For the batching parser it prints the sustained rate and the added latency per record (from
// on_fragment to its handler; every 613th record sampled): p50 / p99 / max.
// Build + run (GPU box): make -C scripts batching_parser_bench && scripts/batching_parser_bench
#include <algorithm>
#include <chrono>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <string>
#include <vector>

#include "aeron_cluster_amd.hpp"
#include "sbecodec.h"
#include "../oracle/sbe_oracle.h"

using namespace aeron_cluster;
using clk = std::chrono::steady_clock;

static double us_between(clk::time_point a, clk::time_point b) {
    return std::chrono::duration<double, std::micro>(b - a).count();
}

int main(int argc, char** argv) {
    // optional: one max_records setting only (diagnosis runs, e.g. with AERON_AMD_TRACE=1)
    const size_t only = argc > 1 ? (size_t)std::strtoull(argv[1], nullptr, 10) : 0;
    if (!gpu_codec_available()) {
        std::fprintf(stderr, "no gfx950 device\n");
        return 2;
    }
    const size_t N = 1 << 20;
    const std::string topic = "orders", type = "CREATE_ORDER", payload(143, 'p'), headers(32, 'h');
    std::vector<std::string> uuids(N);  // TopicMessageFields holds views
    std::vector<TopicMessageFields> msgs;
    msgs.reserve(N);
    for (size_t i = 0; i < N; ++i) {
        char uuid[32];
        std::snprintf(uuid, sizeof uuid, "msg_%019llu_%05zu", 1760000000000000000ULL + i, i % 100000);
        uuids[i] = uuid;
        msgs.push_back(TopicMessageFields{topic, type, uuids[i], payload, headers, (int64_t)(1760000000000000000LL + i)});
    }
    const EncodedBatch enc = SBEEncoder::encode_topic_batch(msgs, EncodeLength::Wire);
    const std::vector<uint8_t> data = enc.bytes.to_vector();
    std::vector<uint64_t> off(enc.offsets.data(), enc.offsets.data() + N + 1);

    // the drop-in called once per fragment (10 K fragments: a few tens of milliseconds)
    {
        const size_t M = 10000;
        for (size_t i = 0; i < 100; ++i) (void)MessageParser::parse_message(data.data() + off[i], off[i + 1] - off[i]);
        const auto t0 = clk::now();
        size_t ok = 0;
        for (size_t i = 0; i < M; ++i) ok += MessageParser::parse_message(data.data() + off[i], off[i + 1] - off[i]).success;
        const double us = us_between(t0, clk::now());
        std::printf("{\"op\": \"per_fragment\", \"records\": %zu, \"us_per_record\": %.2f, \"rec_per_s\": %.4g, \"ok\": %s}\n",
                    M, us / M, M / (us * 1e-6), ok == M ? "true" : "false");
    }
    // the CPU restatement on one thread, same records
    double oracle_rate = 0;
    {
        std::vector<uint8_t> st(N), fl(N);
        std::vector<uint16_t> h(4 * N);
        std::vector<uint64_t> ts(N);
        std::vector<uint32_t> vo(5 * N), vl(5 * N);
        const auto t0 = clk::now();
        orc_decode_batch(data.data(), off.data(), N, SBE_DEC_PARSE_MESSAGE, st.data(), fl.data(), h.data(), ts.data(),
                         vo.data(), vl.data(), 1);
        const double us = us_between(t0, clk::now());
        oracle_rate = N / (us * 1e-6);
        std::printf("{\"op\": \"oracle_1thread\", \"records\": %zu, \"rec_per_s\": %.4g}\n", N, oracle_rate);
    }
    struct Setting {
        size_t max_records;
        int max_delay_us;
        size_t batches;
        int spin_us;
    };
    for (const Setting s : {Setting{1024, 100, 2, 0}, Setting{1024, 100, 4, 200}, Setting{1024, 100, 8, 200},
                            Setting{512, 50, 8, 200}, Setting{2048, 100, 4, 200}, Setting{4096, 200, 4, 200},
                            Setting{8192, 200, 4, 200}, Setting{16384, 500, 4, 200}, Setting{65536, 2000, 4, 200}}) {
        if (only && s.max_records != only) continue;
        // one parser per setting, as an application keeps one: a warm-up pass (the decode thread's
        // device context and serve kernel, the page-locked pool), then the timed pass
        std::vector<clk::time_point> t_in((N + 612) / 613);
        std::vector<double> lat;
        lat.reserve(t_in.size());
        size_t got = 0, bad = 0, base = 0;
        bool timing = false;
        BatchingParser::Options o;
        o.max_records = s.max_records;
        o.max_delay = std::chrono::microseconds(s.max_delay_us);
        o.batches = s.batches;
        o.spin = std::chrono::microseconds(s.spin_us);
        BatchingParser bp(
            [&](const ParseResult& r) {
                const size_t k = got - base;
                if (timing && k % 613 == 0) lat.push_back(us_between(t_in[k / 613], clk::now()));
                bad += !(r.success && r.payload.size() == 143);
                ++got;
            },
            o);
        double in_us = 0;  // of the timed pass: time inside on_fragment
        auto pass = [&](size_t count) {
            size_t i = 0;
            while (i < count) {
                const size_t end = std::min(count, i + 100);  // one poll: up to 100 fragments
                const auto ta = clk::now();
                for (; i < end; ++i) {
                    if (timing && i % 613 == 0) t_in[i / 613] = clk::now();
                    bp.on_fragment(data.data() + off[i], off[i + 1] - off[i]);
                }
                if (timing) in_us += us_between(ta, clk::now());
                (void)bp.poll();
            }
            (void)bp.flush();
        };
        pass(N / 8);
        base = got;
        timing = true;
        const auto t0 = clk::now();
        pass(N);
        const double us = us_between(t0, clk::now());
        std::sort(lat.begin(), lat.end());
        const auto pct = [&](double q) { return lat.empty() ? 0.0 : lat[std::min(lat.size() - 1, (size_t)(q * lat.size()))]; };
        std::printf("{\"op\": \"batching_parser\", \"records\": %zu, \"poll_fragments\": 100, \"max_records\": %zu, "
                    "\"max_delay_us\": %d, \"batches\": %zu, \"spin_us\": %d, \"rec_per_s\": %.4g, \"vs_oracle_1thread\": %.2f, \"latency_us_p50\": %.1f, "
                    "\"latency_us_p99\": %.1f, \"latency_us_max\": %.1f, \"on_fragment_share\": %.2f, \"ok\": %s}\n",
                    N, s.max_records, s.max_delay_us, s.batches, s.spin_us, N / (us * 1e-6), N / (us * 1e-6) / oracle_rate, pct(0.5), pct(0.99),
                    lat.empty() ? 0.0 : lat.back(), in_us / us, (got - base == N && bad == 0) ? "true" : "false");
        std::fflush(stdout);
    }
    return 0;
}
