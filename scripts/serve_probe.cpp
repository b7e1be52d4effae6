// serve_probe.cpp — where a served request's time goes: the serve kernel's C ABI (loaded with
// dlopen from the library given, a -DSBE_SERVE_PROF build for the phase split) driven with empty
// requests, one-record decodes and one-record encodes from host memory; prints the host round trip
// and the kernel's own phase times per request.  Measurement tooling, not product code.
// Build: g++ -O2 -std=c++17 -I../include -I/opt/rocm/include -D__HIP_PLATFORM_AMD__ -o serve_probe
//        serve_probe.cpp -L/opt/rocm/lib -lamdhip64 -ldl
#include <dlfcn.h>
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <string>
#include <vector>

#include "sbecodec.h"

using clk = std::chrono::steady_clock;

int main(int argc, char** argv) {
    const char* path = argc > 1 ? argv[1] : "libsbecodec.so";
    void* h = dlopen(path, RTLD_NOW | RTLD_LOCAL);
    if (!h) {
        std::printf("dlopen %s: %s\n", path, dlerror());
        return 2;
    }
#define SYM(name) auto name = reinterpret_cast<decltype(&::name)>(dlsym(h, #name))
    SYM(sbe_server_create);
    SYM(sbe_server_destroy);
    SYM(sbe_serve_encode_topic);
    SYM(sbe_serve_encode_topic_host);
    SYM(sbe_serve_decode_host);
    auto prof = reinterpret_cast<int (*)(uint64_t*)>(dlsym(h, "sbe_debug_serve_prof"));
    sbe_server* srv = nullptr;
    if (!sbe_server_create || sbe_server_create(&srv, 0) != SBE_OK) return 3;
    void* pin = nullptr;
    if (hipHostMalloc(&pin, 1 << 16, hipHostMallocDefault) != hipSuccess) return 4;
    void* dpin = nullptr;
    (void)hipHostGetDevicePointer(&dpin, pin, 0);
    uint8_t* d = static_cast<uint8_t*>(dpin);
    // one 256-B TopicMessage (fields of the fixed-256 Order record)
    const std::string f[5] = {"orders", "CREATE_ORDER", "msg_1760000000000000000_00042", std::string(143, 'p'),
                              std::string(32, 'h')};
    std::vector<uint8_t> arena;
    uint32_t lens[5];
    for (int k = 0; k < 5; ++k) {
        arena.insert(arena.end(), f[k].begin(), f[k].end());
        lens[k] = (uint32_t)f[k].size();
    }
    const uint64_t ts1 = 1760000000000000000ull;
    sbe_tm_batch tb{arena.data(), nullptr, lens, &ts1};
    sbe_tm_batch t0{nullptr, nullptr, nullptr, nullptr};
    uint8_t* out = d + 4096;
    uint64_t* off = reinterpret_cast<uint64_t*>(d + 8192);
    if (sbe_serve_encode_topic_host(srv, &tb, 1, 0, 0, out, 4096, off, d + 8256) != SBE_OK) return 5;
    std::vector<uint8_t> rec(static_cast<uint8_t*>(pin) + 4096, static_cast<uint8_t*>(pin) + 4096 + 256);
    const uint64_t ro[2] = {0, 256};
    sbe_decoded dd{d, d + 64, reinterpret_cast<uint16_t*>(d + 128), reinterpret_cast<uint64_t*>(d + 192),
                   reinterpret_cast<uint32_t*>(d + 256), reinterpret_cast<uint32_t*>(d + 320),
                   reinterpret_cast<uint64_t*>(d + 384)};
    auto run = [&](const char* name, auto&& fn) {
        for (int i = 0; i < 300; ++i) fn();
        uint64_t p[16] = {};
        if (prof) prof(p);
        const int n = 4000;
        const auto a = clk::now();
        for (int i = 0; i < n; ++i) fn();
        const double us = std::chrono::duration<double, std::micro>(clk::now() - a).count() / n;
        if (prof) prof(p);
        const double c = p[4] ? (double)p[4] : 1.0;
        std::printf("{\"probe\": \"%s\", \"host_us\": %.2f, \"kernel_seen_to_request_us\": %.2f, "
                    "\"inline_copy_us\": %.2f, \"body_us\": %.2f, \"release_us\": %.2f, \"requests\": %llu, "
                    "\"tile_offsets_us\": %.2f, \"tile_window_us\": %.2f, \"tile_parsed_us\": %.2f, "
                    "\"tile_stores_issued_us\": %.2f}\n",
                    name, us, p[0] / c / 100.0, p[1] / c / 100.0, p[2] / c / 100.0, p[3] / c / 100.0,
                    (unsigned long long)p[4], p[5] / c / 100.0, p[6] / c / 100.0, p[7] / c / 100.0, p[8] / c / 100.0);
    };
    run("empty", [&] { (void)sbe_serve_encode_topic(srv, &t0, 0, 0, 0, out, 0, off, nullptr); });
    run("decode_1_host", [&] { (void)sbe_serve_decode_host(srv, rec.data(), ro, 1, SBE_DEC_PARSE_MESSAGE, &dd); });
    run("encode_1_host", [&] { (void)sbe_serve_encode_topic_host(srv, &tb, 1, 0, 0, out, 4096, off, d + 8256); });
    // a -DSBE_PACK_PHASES build: the pack loop's phase clocks (s_memtime) of the last served encode
    if (auto ph = reinterpret_cast<int (*)(uint64_t*, int)>(dlsym(h, "sbe_debug_phases"))) {
        uint64_t v[8] = {};
        (void)sbe_serve_encode_topic_host(srv, &tb, 1, 0, 0, out, 4096, off, d + 8256);
        if (ph(v, 1) == 0)
            std::printf("{\"probe\": \"encode_1_phases_clk\", \"prologue_and_issue\": %llu, \"chunks\": %llu, "
                        "\"zone_fixup\": %llu, \"literals\": %llu, \"store\": %llu, \"stage_write\": %llu, "
                        "\"slow_path\": %llu, \"prepare_next\": %llu}\n",
                        (unsigned long long)v[0], (unsigned long long)v[1], (unsigned long long)v[2],
                        (unsigned long long)v[3], (unsigned long long)v[4], (unsigned long long)v[5],
                        (unsigned long long)v[6], (unsigned long long)v[7]);
    }
    sbe_server_destroy(srv);
    return 0;
}
