// sbe_codec.hip — MI355X (gfx950) batch SBE codec: HIP kernels + the C ABI of include/sbecodec.h.
//
// Byte packing, not a contraction: no MFMA.  Both kernels are HBM-stream kernels built around
// one record per lane, one 64-record tile per single-wave workgroup, and an LDS window that turns
// the per-record byte scatter/gather into coalesced 16-byte HBM accesses.
//
//  encode  (SBEEncoder::encode_topic_message, src/sbe_encoder.cpp:131-167)
//    1. lane loads its record's 5 lengths + timestamp, wave-scans output (and, packed, input) sizes
//    2. tile base offsets by single-pass decoupled look-back over per-tile 8-byte status words
//       (flag | value in one word → no payload hand-off; tile ids from an atomic ticket, so every
//       tile waited on is already running: no dispatch-order assumption)
//    3. each lane composes its wire record (header, ts, seq=0, u16 len + bytes ×5) as aligned
//       dwords into an XOR-swizzled LDS window; record edges use byte writes
//    4. the wave stores the window with global_store_dwordx4 (edge chunks byte-wise)
//  decode  (MessageParser::parse_message :513-551 / MessageHandler::on_egress
//           include/aeron_cluster/message_handler.hpp:35-68 + decode_ack src/ack_decoder.cpp:29-105)
//    1. the wave stages its tile's contiguous bytes into the same swizzled LDS window with
//       global_load_dwordx4
//    2. each lane parses its record from LDS (template-ID dispatch per lane) and writes the
//       descriptor SoA; bytes outside the window are read from global memory.
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstring>

#include "../../include/sbecodec.h"

namespace {

constexpr int kWave = 64;
constexpr int kTile = 64;                 // records per workgroup (one per lane)
constexpr uint32_t kWin = 16384;          // LDS window bytes (encode output / decode input)
constexpr uint32_t kWinDw = kWin / 4;
constexpr uint64_t kFlagAgg = 1ull << 62; // look-back status word: [63:62] flag, [61:0] value
constexpr uint64_t kFlagInc = 2ull << 62;
constexpr uint64_t kValMask = (1ull << 62) - 1;

// ------------------------------------------------------------------------------------------
// LDS window.  Dword i of the window lives at i ^ ((i >> 6) & 31): lanes that write dword j of
// records 256 B apart then hit 32 distinct banks, and a 16-byte chunk stays inside one aligned
// 4-dword slot (permuted by the low 2 bits of the XOR), so chunk copies use ds_*_b128.
// ------------------------------------------------------------------------------------------
__device__ __forceinline__ uint32_t swz(uint32_t i) { return i ^ ((i >> 6) & 31u); }

__device__ __forceinline__ uint4 permute4(uint4 v, uint32_t y) {
    // out[k] = v[k ^ y]
    if (y & 1u) {
        uint32_t t = v.x; v.x = v.y; v.y = t;
        t = v.z; v.z = v.w; v.w = t;
    }
    if (y & 2u) {
        uint32_t t = v.x; v.x = v.z; v.z = t;
        t = v.y; v.y = v.w; v.w = t;
    }
    return v;
}

// chunk c (16 B) of the window in natural byte order
__device__ __forceinline__ uint4 lds_read_chunk(const uint32_t* win, uint32_t c) {
    const uint32_t x = (c >> 4) & 31u;
    const uint4 v = *reinterpret_cast<const uint4*>(win + ((4u * c) ^ (x & 28u)));
    return permute4(v, x & 3u);
}

__device__ __forceinline__ void lds_write_chunk(uint32_t* win, uint32_t c, uint4 v) {
    const uint32_t x = (c >> 4) & 31u;
    *reinterpret_cast<uint4*>(win + ((4u * c) ^ (x & 28u))) = permute4(v, x & 3u);
}

__device__ __forceinline__ uint32_t lds_dw(const uint32_t* win, uint32_t i) { return win[swz(i)]; }

// ------------------------------------------------------------------------------------------
// wave helpers
// ------------------------------------------------------------------------------------------
__device__ __forceinline__ uint32_t wave_incl_scan(uint32_t v, int lane) {
#pragma unroll
    for (int d = 1; d < kWave; d <<= 1) {
        uint32_t t = __shfl_up(v, d, kWave);
        if (lane >= d) v += t;
    }
    return v;
}

__device__ __forceinline__ uint64_t wave_sum64(uint64_t v) {
#pragma unroll
    for (int d = 32; d >= 1; d >>= 1) v += __shfl_xor(v, d, kWave);
    return v;
}

__device__ __forceinline__ uint64_t uniform64(uint64_t v) {
    uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)v);
    uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)(v >> 32));
    return ((uint64_t)hi << 32) | lo;
}

__device__ __forceinline__ uint32_t byte_mask_bits(uint32_t nbytes) {
    return nbytes >= 4 ? 0xffffffffu : ((1u << (8u * nbytes)) - 1u);
}

// ------------------------------------------------------------------------------------------
// Encode
// ------------------------------------------------------------------------------------------
// Encode workspace: a 64-byte header, then two parities of per-tile look-back status words.
// Zeroed once by sbe_encode_workspace_init; each call zeroes the parity the previous call used
// and the last tile through the look-back flips `parity`, so calls need no reset in between.
struct EncWorkspace {
    uint32_t ticket;   // tile tickets drawn in the running call
    uint32_t done;     // tiles past their look-back
    uint32_t parity;   // status array used by the next call
    uint32_t err;      // bit 0: a look-back spin gave up (never expected)
    uint64_t used[2];  // tiles written in each status array by its last call
    uint64_t pad[4];
};
static_assert(sizeof(EncWorkspace) == 64, "workspace header is 64 bytes");
constexpr uint32_t kMaxSpins = 1u << 22;

template <typename T>
__device__ __forceinline__ T atomic_read(T* p) {
    return __hip_atomic_fetch_or(p, (T)0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void publish(uint64_t* p, uint64_t v) {
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

struct EncArgs {
    const uint8_t* arena;
    const uint32_t* str_off;
    const uint32_t* str_len;
    const uint64_t* timestamp;
    uint64_t n;
    uint64_t ts_default;
    uint8_t* out;
    uint64_t cap;
    uint64_t* out_off;
    uint8_t* status;
    EncWorkspace* ws;
    uint64_t* st;        // 2 parities x {out, in} x cap_tiles status words
    uint64_t cap_tiles;
};

// Per-lane dword composer.  Bytes are appended in stream order; whole dwords are flushed to the
// LDS window when they fall inside [wb, we) and are masked to the record's own bytes [rs, re).
struct Composer {
    uint64_t q;     // absolute position of the first pending byte's dword (4-aligned)
    uint64_t acc;   // pending bytes, little-endian
    uint32_t nacc;  // pending byte count incl. (rs & 3) leading don't-care bytes for the 1st dword
    uint64_t rs, re, wb, we;
    uint32_t* win;

    __device__ __forceinline__ void flush(uint32_t v) {
        if (q >= wb && q < we) {
            const uint32_t i = (uint32_t)((q - wb) >> 2);
            if (q >= rs && q + 4 <= re) {
                win[swz(i)] = v;
            } else {
                uint8_t* b = reinterpret_cast<uint8_t*>(win + swz(i));
#pragma unroll
                for (uint32_t k = 0; k < 4; ++k)
                    if (q + k >= rs && q + k < re) b[k] = (uint8_t)(v >> (8 * k));
            }
        }
        q += 4;
    }
    // append nb (1..4) bytes held in the low bytes of v (bytes above nb must be zero)
    __device__ __forceinline__ void append(uint32_t v, uint32_t nb) {
        acc |= (uint64_t)v << (8u * nacc);
        nacc += nb;
        if (nacc >= 4) {
            flush((uint32_t)acc);
            acc >>= 32;
            nacc -= 4;
        }
    }
    __device__ __forceinline__ void finish() {
        if (nacc) flush((uint32_t)acc);
    }
    // position of the next byte to be appended
    __device__ __forceinline__ uint64_t pos() const { return q + nacc; }
    // jump to absolute position p (> current), discarding pending bytes: valid only when every
    // dword holding the skipped bytes lies before the window (p + 4 <= wb)
    __device__ __forceinline__ void skip_to(uint64_t p) {
        q = p & ~3ull;
        nacc = (uint32_t)(p & 3u);
        acc = 0;
    }
    // append L bytes of global memory starting at src
    __device__ __forceinline__ void append_bytes(const uint8_t* src, uint32_t L) {
        if (L == 0) return;
        const uint64_t p0 = pos();
        if (p0 + L + 4 <= wb) { skip_to(p0 + L); return; }
        const uintptr_t a = reinterpret_cast<uintptr_t>(src);
        const uint32_t sh = (uint32_t)(a & 3u);
        const uint32_t* w = reinterpret_cast<const uint32_t*>(a - sh);
        uint32_t nb = 4u - sh;
        if (nb > L) nb = L;
        append((w[0] >> (8u * sh)) & byte_mask_bits(nb), nb);
        uint32_t rem = L - nb;
        ++w;
        while (rem >= 4) {
            if (q >= we) return;  // past the window: nothing more to write for this record
            append(w[0], 4);
            ++w;
            rem -= 4;
        }
        if (rem) append(w[0] & byte_mask_bits(rem), rem);
    }
};

template <bool kPacked, bool kTrunc>
__global__ __launch_bounds__(kWave) void sbe_encode_kernel(EncArgs a) {
    __shared__ uint32_t win[kWinDw];
    const int lane = threadIdx.x;

    // ---- tile ticket (dynamic tile order = start order: look-back never waits on an unstarted tile)
    uint32_t tile = 0, par = 0;
    uint64_t used_other = 0;
    if (lane == 0) {
        tile = atomicAdd(&a.ws->ticket, 1u);
        par = atomic_read(&a.ws->parity) & 1u;
        used_other = atomic_read(&a.ws->used[par ^ 1u]);
    }
    tile = __builtin_amdgcn_readfirstlane(__shfl(tile, 0, kWave));
    par = __builtin_amdgcn_readfirstlane(__shfl(par, 0, kWave));
    used_other = uniform64(__shfl(used_other, 0, kWave));
    const uint64_t r = (uint64_t)tile * kTile + lane;
    const bool valid = r < a.n;
    const uint64_t ntiles = (a.n + kTile - 1) / kTile;
    uint64_t* const st_out = a.st + (uint64_t)par * 2 * a.cap_tiles;
    uint64_t* const st_in = st_out + a.cap_tiles;
    uint64_t* const other_out = a.st + (uint64_t)(par ^ 1u) * 2 * a.cap_tiles;
    uint64_t* const other_in = other_out + a.cap_tiles;
    // zero the other parity's words used by the previous call (that call has completed)
    for (uint64_t t = tile + (uint64_t)lane * ntiles; t < used_other; t += (uint64_t)kWave * ntiles) {
        other_out[t] = 0;
        other_in[t] = 0;
    }

    // ---- record sizes
    uint32_t L[5] = {0, 0, 0, 0, 0};
    uint32_t sum = 0;
    uint8_t st = SBE_ENC_OK;
    uint64_t ts = 0;
    if (valid) {
#pragma unroll
        for (int f = 0; f < 5; ++f) {
            L[f] = a.str_len[5 * r + f];
            sum += L[f];
        }
#pragma unroll
        for (int f = 4; f >= 0; --f)
            if (L[f] > SBE_VAR_MAX_LEN) st = (uint8_t)(SBE_ENC_E109_TOPIC + f);
        ts = a.timestamp[r];
        if (ts == 0) ts = a.ts_default;
    }
    const uint32_t ovh = kTrunc ? SBE_TM_REF_OVERHEAD : SBE_TM_WIRE_OVERHEAD;
    const uint32_t rec_out = (valid && st == SBE_ENC_OK) ? ovh + sum : 0u;
    const uint32_t rec_in = (kPacked && valid) ? sum : 0u;  // E109 records keep their arena bytes
    const uint32_t inc_out = wave_incl_scan(rec_out, lane);
    const uint32_t inc_in = kPacked ? wave_incl_scan(rec_in, lane) : 0u;
    const uint64_t agg_out = __shfl(inc_out, kWave - 1, kWave);
    const uint64_t agg_in = kPacked ? (uint64_t)__shfl(inc_in, kWave - 1, kWave) : 0ull;

    // ---- decoupled look-back.  Each status word is a self-contained 8-B granule (flag | value),
    // published with an agent-scope store and polled with agent-scope atomic RMW reads, which are
    // performed at the device coherence point (per-XCD L2s are not coherent with each other).
    // This call's words live in array `par`; the other array was zeroed above for the next call.
    uint64_t base_out = 0, base_in = 0;
    if (tile == 0) {
        if (lane == 0) {
            publish(st_out, kFlagInc | agg_out);
            publish(st_in, kFlagInc | agg_in);
        }
    } else {
        if (lane == 0) {
            publish(st_out + tile, kFlagAgg | agg_out);
            publish(st_in + tile, kFlagAgg | agg_in);
        }
        int64_t pred = (int64_t)tile - 1;
        uint32_t spins = 0;
        for (;;) {
            const int64_t idx = pred - lane;
            uint64_t so = kFlagInc, si = kFlagInc;  // before tile 0: inclusive zero
            if (idx >= 0) {
                so = atomic_read(st_out + idx);
                si = atomic_read(st_in + idx);
            }
            const uint64_t fo = so >> 62, fi = si >> 62;
            const bool ready = fo != 0 && fo == fi;
            const uint64_t incm = __ballot(ready && fo == 2);
            const uint64_t notready = __ballot(!ready);
            const int k = incm ? __builtin_ctzll(incm) : 64;  // nearest inclusive predecessor
            const uint64_t need = k >= 63 ? ~0ull : ((2ull << k) - 1ull);
            if ((notready & need) && ++spins < kMaxSpins) {
                __builtin_amdgcn_s_sleep(2);
                continue;
            }
            if (notready & need) {  // bounded spin: record the failure instead of hanging
                if (lane == 0) atomicOr(&a.ws->err, 1u);
            }
            const bool take = lane <= k;
            base_out += wave_sum64(take ? (so & kValMask) : 0ull);
            base_in += wave_sum64(take ? (si & kValMask) : 0ull);
            if (k < 64 || (notready & need)) break;
            pred -= kWave;
        }
        base_out = uniform64(base_out);
        base_in = uniform64(base_in);
        if (lane == 0) {
            publish(st_out + tile, kFlagInc | (base_out + agg_out));
            publish(st_in + tile, kFlagInc | (base_in + agg_in));
        }
    }
    // the last tile through the look-back hands the workspace to the next call
    if (lane == 0) {
        const uint32_t done = atomicAdd(&a.ws->done, 1u);
        if (done == ntiles - 1) {
            __hip_atomic_store(&a.ws->used[par], ntiles, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            __hip_atomic_store(&a.ws->used[par ^ 1u], 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            __hip_atomic_store(&a.ws->parity, par ^ 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            __hip_atomic_store(&a.ws->ticket, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            __hip_atomic_store(&a.ws->done, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
    }

    // ---- per-record offsets / status
    const uint64_t rs = base_out + inc_out - rec_out;
    const uint64_t re = rs + rec_out;
    if (valid) {
        if (st == SBE_ENC_OK && re > a.cap) st = SBE_ENC_OVERFLOW;
        a.out_off[r] = rs;
        if (r == a.n - 1) a.out_off[a.n] = re;
        if (a.status) a.status[r] = st;
    }

    // ---- source addresses of the five strings
    const uint8_t* src[5];
    if (kPacked) {
        uint64_t o = base_in + inc_in - rec_in;
#pragma unroll
        for (int f = 0; f < 5; ++f) {
            src[f] = a.arena + o;
            o += L[f];
        }
    } else {
#pragma unroll
        for (int f = 0; f < 5; ++f) src[f] = valid ? a.arena + a.str_off[5 * r + f] : a.arena;
    }

    // ---- compose windows and store them
    const uint64_t T0 = base_out;
    const uint64_t T1 = (base_out + agg_out) < a.cap ? (base_out + agg_out) : a.cap;
    const uint64_t hi_rec = re < a.cap ? re : a.cap;
    for (uint64_t wb = T0 & ~15ull; wb < T1; wb += kWin) {
        const uint64_t we = wb + kWin;
        if (rec_out && rs < we && hi_rec > wb && rs < hi_rec) {
            Composer c;
            c.q = rs & ~3ull;
            c.acc = 0;
            c.nacc = (uint32_t)(rs & 3u);
            c.rs = rs;
            c.re = hi_rec;
            c.wb = wb;
            c.we = we;
            c.win = win;
            // header {blockLength 16, templateId 1, schemaId 1, version 1}, ts, sequenceNumber 0
            c.append(SBE_TM_BLOCK_LEN | (SBE_TM_TEMPLATE_ID << 16), 4);
            c.append(SBE_TOPIC_SCHEMA_ID | (1u << 16), 4);
            c.append((uint32_t)ts, 4);
            c.append((uint32_t)(ts >> 32), 4);
            c.append(0u, 4);
            c.append(0u, 4);
#pragma unroll
            for (int f = 0; f < 5; ++f) {
                if (c.q >= we) break;
                c.append(L[f] & 0xffffu, 2);
                c.append_bytes(src[f], L[f]);
            }
            if (c.q < we) c.finish();
        }
        __syncthreads();
        // store [max(wb,T0), min(we,T1)) : 16-B chunks, partial edge chunks byte-wise
        const uint64_t lo = wb > T0 ? wb : T0;
        const uint64_t hi = we < T1 ? we : T1;
        const uint32_t nch = (uint32_t)((hi - wb + 15) >> 4);
        for (uint32_t ch = lane; ch < nch; ch += kWave) {
            const uint64_t g = wb + 16ull * ch;
            const uint4 v = lds_read_chunk(win, ch);
            if (g >= lo && g + 16 <= hi) {
                *reinterpret_cast<uint4*>(a.out + g) = v;
            } else {
                const uint32_t w4[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
                for (uint32_t k = 0; k < 16; ++k)
                    if (g + k >= lo && g + k < hi) a.out[g + k] = (uint8_t)(w4[k >> 2] >> (8 * (k & 3)));
            }
        }
        __syncthreads();
    }
}

// ------------------------------------------------------------------------------------------
// Decode
// ------------------------------------------------------------------------------------------
struct DecArgs {
    const uint8_t* in;
    const uint64_t* rec_off;
    uint64_t n;
    uint8_t* status;
    uint8_t* flags;
    uint16_t* hdr;
    uint64_t* ts;
    uint32_t* view_off;
    uint32_t* view_len;
};

// Reads of one record: LDS window [wb, we) where staged, global memory elsewhere.
struct RecReader {
    const uint8_t* in;
    const uint32_t* win;
    uint64_t wb, we;  // staged window (absolute stream positions)
    uint64_t s;       // record start (absolute)

    // dword of the stream at aligned absolute position qa
    __device__ __forceinline__ uint32_t dw(uint64_t qa) const {
        if (qa >= wb && qa < we) return lds_dw(win, (uint32_t)((qa - wb) >> 2));
        return *reinterpret_cast<const uint32_t*>(in + qa);
    }
    // up to 4 bytes at record offset p (the caller guarantees p+nb <= record length)
    __device__ __forceinline__ uint32_t bytes(uint64_t p, uint32_t nb) const {
        const uint64_t ap = s + p;
        const uint64_t qa = ap & ~3ull;
        const uint32_t sh = (uint32_t)(ap & 3u);
        uint32_t lo = dw(qa);
        uint32_t v = lo >> (8 * sh);
        if (sh + nb > 4) v = __builtin_amdgcn_alignbyte(dw(qa + 4), lo, sh);
        return v & byte_mask_bits(nb);
    }
    __device__ __forceinline__ uint16_t u16(uint64_t p) const { return (uint16_t)bytes(p, 2); }
    __device__ __forceinline__ uint32_t u32(uint64_t p) const { return bytes(p, 4); }
    __device__ __forceinline__ uint64_t u64(uint64_t p) const {
        return (uint64_t)bytes(p, 4) | ((uint64_t)bytes(p + 4, 4) << 32);
    }
};

struct Desc {
    uint32_t status, flags;
    uint16_t hdr[4];
    uint64_t ts;
    uint32_t off[5], len[5];
    __device__ __forceinline__ void clear() {
        status = flags = 0;
        hdr[0] = hdr[1] = hdr[2] = hdr[3] = 0;
        ts = 0;
#pragma unroll
        for (int k = 0; k < 5; ++k) off[k] = len[k] = 0;
    }
    __device__ __forceinline__ void fail(uint32_t st, uint32_t param) {
        clear();
        status = st;
        off[0] = param;
    }
    __device__ __forceinline__ void set_hdr(const RecReader& R, uint64_t p) {
        const uint32_t a = R.u32(p), b = R.u32(p + 4);
        hdr[0] = (uint16_t)a;
        hdr[1] = (uint16_t)(a >> 16);
        hdr[2] = (uint16_t)b;
        hdr[3] = (uint16_t)(b >> 16);
    }
};

__device__ __forceinline__ uint32_t has_byte(uint32_t w, uint32_t byte) {
    const uint32_t x = w ^ (byte * 0x01010101u);
    return (x - 0x01010101u) & ~x & 0x80808080u;
}

// "_sequence_number" anywhere in [p, p+n) of the record (flag only; src/sbe_encoder.cpp:1031-1125)
__device__ bool has_seq_key(const RecReader& R, uint64_t p, uint32_t n) {
    constexpr uint32_t K = 16;  // strlen("_sequence_number")
    if (n < K) return false;
    const uint32_t k0 = 0x7165735fu, k1 = 0x636e6575u, k2 = 0x756e5f65u, k3 = 0x7265626du;
    for (uint32_t i = 0; i + K <= n; i += 4) {
        const uint32_t w = R.u32(p + i);
        uint32_t m = has_byte(w, '_');
        while (m) {
            const uint32_t b = (uint32_t)__builtin_ctz(m) >> 3;
            m &= m - 1;
            const uint64_t q = p + i + b;
            if (i + b + K <= n && R.u32(q) == k0 && R.u32(q + 4) == k1 && R.u32(q + 8) == k2 &&
                R.u32(q + 12) == k3)
                return true;
        }
    }
    return false;
}

// decode_topic_message_with_sbe (src/sbe_encoder.cpp:957-1143); record bytes [b, b+len)
__device__ void dec_tm_parse(const RecReader& R, uint64_t b, uint64_t len, Desc& d) {
    const uint32_t h0 = R.u32(b), h1 = R.u32(b + 4);
    const uint32_t blk = h0 & 0xffffu, ver = h1 >> 16;
    uint64_t pos = 8u + blk;
    if (pos > len) { d.fail(SBE_ST_ERR_TM_E100, 0); return; }
    d.clear();
#pragma unroll
    for (int f = 0; f < 4; ++f) {
        if (pos + 2 > len) { d.fail(SBE_ST_ERR_TM_E100, 0); return; }
        const uint64_t L = R.u16(b + pos);
        if (pos + 2 + L > len) { d.fail(SBE_ST_ERR_TM_E100, 0); return; }
        d.off[f] = (uint32_t)(b + pos + 2);
        d.len[f] = (uint32_t)L;
        pos += 2 + L;
    }
    d.status = SBE_ST_TM;
    d.hdr[0] = (uint16_t)blk;
    d.hdr[1] = 1;
    d.hdr[2] = 1;
    d.hdr[3] = (uint16_t)ver;
    d.ts = R.u64(b + 8);
    if (b) d.flags |= SBE_FL_WRAPPED;
    if (has_seq_key(R, d.off[3], d.len[3])) d.flags |= SBE_FL_SEQ_KEY;
    if (pos + 2 > len || pos + 2 + (uint64_t)R.u16(b + pos) > len) {
        d.flags |= SBE_FL_HEADERS_E100;
    } else {
        d.off[4] = (uint32_t)(b + pos + 2);
        d.len[4] = R.u16(b + pos);
    }
}

// decode_acknowledgment_with_sbe (src/sbe_encoder.cpp:833-954)
__device__ void dec_ack_heuristic(const RecReader& R, uint64_t b, uint64_t len, Desc& d) {
    if (len < 16) { d.fail(SBE_ST_ERR_ACK_SHORT, (uint32_t)len); return; }
    d.clear();
    d.set_hdr(R, b);
    d.status = SBE_ST_ACK;
    d.ts = R.u64(b + 8);
    if (b) d.flags |= SBE_FL_WRAPPED;
    uint32_t nruns = 0;
    uint64_t run_start = 0, run_len = 0;
    for (uint64_t i = 16; i < len && nruns < 3; i += 4) {
        const uint32_t nb = (len - i) < 4 ? (uint32_t)(len - i) : 4u;
        const uint32_t w = R.bytes(b + i, nb);
        for (uint32_t k = 0; k < nb; ++k) {
            const uint32_t c = (w >> (8 * k)) & 0xffu;
            if (c >= 32 && c <= 126) {
                if (run_len == 0) run_start = i + k;
                ++run_len;
            } else {
                if (run_len >= 3 && nruns < 3) {
                    d.off[nruns] = (uint32_t)(b + run_start);
                    d.len[nruns] = (uint32_t)run_len;
                    ++nruns;
                }
                run_len = 0;
            }
        }
    }
    if (nruns < 3 && run_len >= 3) {
        d.off[nruns] = (uint32_t)(b + run_start);
        d.len[nruns] = (uint32_t)run_len;
        ++nruns;
    }
    if (nruns < 1) d.flags |= SBE_FL_ID_DEFAULT;
    if (nruns < 2) d.flags |= SBE_FL_PAYLOAD_DEFAULT;
}

// parse_session_event / decode_session_event (src/sbe_encoder.cpp:618-647, :183-238, :285-318)
__device__ void dec_session_event(const RecReader& R, uint64_t len, Desc& d) {
    if (len < 40) { d.fail(SBE_ST_ERR_SESSION_EVENT, 0); return; }
    d.clear();
    d.status = SBE_ST_SESSION_EVENT;
    d.set_hdr(R, 0);
    const uint64_t rem = len - 40;
    if (rem >= 4) {
        const uint64_t L = R.u32(40);
        if (!(L > rem - 4 || L > 10u * 1024u * 1024u) && L > 0) {
            d.off[3] = 44;
            d.len[3] = (uint32_t)L;
        }
    }
}

// parse_message + parse_topic_message (src/sbe_encoder.cpp:513-551, :724-831)
__device__ void dec_parse_message(const RecReader& R, uint64_t len, Desc& d) {
    if (len == 0) { d.fail(SBE_ST_ERR_NULL_EMPTY, 0); return; }
    if (len < 8) { d.fail(SBE_ST_ERR_HEADER, 0); return; }
    const uint32_t h0 = R.u32(0), h1 = R.u32(4);
    const uint32_t blk = h0 & 0xffffu, tmpl = h0 >> 16, schema = h1 & 0xffffu;
    if (tmpl == 2 && schema == SBE_CLUSTER_SCHEMA_ID) { dec_session_event(R, len, d); return; }
    const bool is_topic = (tmpl == 1 && schema == 1) || (schema == SBE_CLUSTER_SCHEMA_ID && tmpl == 1) ||
                          (schema == 1 && tmpl == 2);
    if (!is_topic) {
        d.fail(SBE_ST_ERR_UNKNOWN_TYPE, 0);
        d.set_hdr(R, 0);
        return;
    }
    if (schema == SBE_CLUSTER_SCHEMA_ID) {
        const uint64_t shs = 8u + blk;
        if (len <= shs) { d.fail(SBE_ST_ERR_SESSION_SHORT, 0); return; }
        const uint64_t elen = len - shs;
        if (elen < 8) { d.fail(SBE_ST_ERR_EMBEDDED_SHORT, 0); return; }
        const uint32_t e0 = R.u32(shs), e1 = R.u32(shs + 4);
        const uint32_t etmpl = e0 >> 16, eschema = e1 & 0xffffu;
        if (eschema == 1) {
            if (etmpl == 1) { dec_tm_parse(R, shs, elen, d); return; }
            if (etmpl == 2) { dec_ack_heuristic(R, shs, elen, d); return; }
            d.fail(SBE_ST_ERR_EMBEDDED_TEMPLATE, etmpl);
            return;
        }
        d.fail(SBE_ST_ERR_EMBEDDED_SCHEMA, eschema);
        return;
    }
    if (tmpl == 1) { dec_tm_parse(R, 0, len, d); return; }
    if (tmpl == 2) { dec_ack_heuristic(R, 0, len, d); return; }
    d.fail(SBE_ST_ERR_DIRECT_TEMPLATE, tmpl);
}

__device__ __forceinline__ uint64_t to_nanos_auto(uint64_t ts) {
    return ts < 100000000000000ull ? ts * 1000000ull : ts;
}

// decode_ack (src/ack_decoder.cpp:29-105) then MessageHandler::on_egress
// (include/aeron_cluster/message_handler.hpp:35-68)
__device__ void dec_on_egress(const RecReader& R, uint64_t len, Desc& d) {
    d.clear();
    if (len < 8) { d.status = SBE_ST_EG_NONE; return; }
    const uint32_t h0 = R.u32(0), h1 = R.u32(4);
    const uint32_t blk = h0 & 0xffffu, tmpl = h0 >> 16, schema = h1 & 0xffffu;
    d.set_hdr(R, 0);
    if (schema == 1 && tmpl == 2) {
        if (len == 16 && blk == 8) {
            d.status = SBE_ST_EG_ACK_SIMPLE;
            d.ts = to_nanos_auto(R.u64(8));
            return;
        }
        const uint64_t lim = len - 8;
        uint64_t pos = 8u + blk;
        bool ok = pos <= lim;
        for (int f = 0; f < 3 && ok; ++f) {
            const uint64_t L = R.u16(pos);
            if (L > 0) {
                if (pos + 2 + L > lim) { ok = false; break; }
                d.off[f] = (uint32_t)(pos + 2);
                d.len[f] = (uint32_t)L;
                pos += 2 + L;
            }
        }
        if (ok) {
            d.status = SBE_ST_EG_ACK;
            d.ts = to_nanos_auto(R.u64(8));
            return;
        }
#pragma unroll
        for (int k = 0; k < 5; ++k) d.off[k] = d.len[k] = 0;
    }
    if (!(tmpl == 1 && schema == 1)) { d.status = SBE_ST_EG_NONE; return; }
    const uint64_t lim = len - 8;
    uint64_t pos = 8u + blk;
    if (pos > lim) { d.status = SBE_ST_EG_THROW_E100; return; }
#pragma unroll
    for (int f = 0; f < 5; ++f) {
        const uint64_t L = R.u16(pos);
        if (L > 0) {
            if (pos + 2 + L > lim) {
#pragma unroll
                for (int k = 0; k < 5; ++k) d.off[k] = d.len[k] = 0;
                d.status = SBE_ST_EG_THROW_E100;
                return;
            }
            d.off[f] = (uint32_t)(pos + 2);
            d.len[f] = (uint32_t)L;
            pos += 2 + L;
        }
    }
    if (d.len[0] == 0) {
#pragma unroll
        for (int k = 0; k < 5; ++k) d.off[k] = d.len[k] = 0;
        d.status = SBE_ST_EG_NONE;
        return;
    }
    d.status = SBE_ST_EG_TM;
}

template <uint32_t kMode>
__global__ __launch_bounds__(kWave) void sbe_decode_kernel(DecArgs a) {
    __shared__ uint32_t win[kWinDw];
    const int lane = threadIdx.x;
    const uint64_t t0 = (uint64_t)blockIdx.x * kTile;
    const uint64_t r = t0 + lane;
    const bool valid = r < a.n;
    const uint64_t last = (t0 + kTile < a.n ? t0 + kTile : a.n);
    const uint64_t T0 = uniform64(a.rec_off[t0]);
    const uint64_t T1 = uniform64(a.rec_off[last]);
    const uint64_t rs = valid ? a.rec_off[r] : 0;
    const uint64_t rl = valid ? a.rec_off[r + 1] - rs : 0;

    // ---- stage [wb, min(wb+kWin, align16(T1))) into LDS with 16-byte loads
    const uint64_t wb = T0 & ~15ull;
    const uint64_t end = (T1 + 15) & ~15ull;
    const uint64_t we = (wb + kWin) < end ? wb + kWin : end;
    const uint32_t nch = (uint32_t)((we - wb) >> 4);
    for (uint32_t ch = lane; ch < nch; ch += kWave)
        lds_write_chunk(win, ch, *reinterpret_cast<const uint4*>(a.in + wb + 16ull * ch));
    __syncthreads();

    if (!valid) return;
    RecReader R{a.in, win, wb, we, rs};
    Desc d;
    if (kMode == SBE_DEC_ON_EGRESS)
        dec_on_egress(R, rl, d);
    else
        dec_parse_message(R, rl, d);

    a.status[r] = (uint8_t)d.status;
    a.flags[r] = (uint8_t)d.flags;
    *reinterpret_cast<uint2*>(a.hdr + 4 * r) =
        make_uint2((uint32_t)d.hdr[0] | ((uint32_t)d.hdr[1] << 16), (uint32_t)d.hdr[2] | ((uint32_t)d.hdr[3] << 16));
    a.ts[r] = d.ts;
#pragma unroll
    for (int k = 0; k < 5; ++k) {
        a.view_off[5 * r + k] = d.off[k];
        a.view_len[5 * r + k] = d.len[k];
    }
}

thread_local char g_last_error[256] = "";

int record_hip(hipError_t e) {
    if (e == hipSuccess) return SBE_OK;
    std::strncpy(g_last_error, hipGetErrorString(e), sizeof(g_last_error) - 1);
    return SBE_EHIP;
}

constexpr uint64_t kMaxTiles = 0xffffffffull;

}  // namespace

// ============================================================================================
// C ABI
// ============================================================================================
extern "C" {

int sbe_abi_version(void) { return SBECODEC_ABI_VERSION; }

const char* sbe_last_error(void) { return g_last_error; }

int sbe_device_ready(void) {
    int count = 0;
    hipError_t e = hipGetDeviceCount(&count);
    if (e != hipSuccess) return e == hipErrorNoDevice ? 0 : record_hip(e);
    for (int i = 0; i < count; ++i) {
        hipDeviceProp_t p;
        if (hipGetDeviceProperties(&p, i) == hipSuccess && std::strncmp(p.gcnArchName, "gfx950", 6) == 0)
            return 1;
    }
    return 0;
}

size_t sbe_encode_workspace_size(uint64_t n) {
    const uint64_t tiles = (n + kTile - 1) / kTile;
    return (size_t)(sizeof(EncWorkspace) + 32 * (tiles ? tiles : 1));
}

uint64_t sbe_encode_output_bound(uint64_t n, uint64_t string_bytes, uint32_t flags) {
    (void)flags;
    return string_bytes + (uint64_t)SBE_TM_WIRE_OVERHEAD * n;
}

int sbe_encode_workspace_init(void* workspace, size_t workspace_bytes, void* stream) {
    if (!workspace) return SBE_EINVAL;
    return record_hip(hipMemsetAsync(workspace, 0, workspace_bytes, reinterpret_cast<hipStream_t>(stream)));
}

int sbe_encode_topic_batch(const sbe_tm_batch* in, uint64_t n, uint64_t ts_default, uint32_t flags,
                           uint8_t* out, uint64_t out_capacity, uint64_t* out_off, uint8_t* status,
                           void* workspace, size_t workspace_bytes, void* stream) {
    if (!in || !out_off) return SBE_EINVAL;
    if (flags & ~SBE_ENC_REF_TRUNCATE8) return SBE_EINVAL;
    hipStream_t s = reinterpret_cast<hipStream_t>(stream);
    if (n == 0) return record_hip(hipMemsetAsync(out_off, 0, sizeof(uint64_t), s));
    if (!in->str_len || !in->timestamp || !in->arena || !out) return SBE_EINVAL;
    if ((reinterpret_cast<uintptr_t>(out) & 15u) || (reinterpret_cast<uintptr_t>(out_off) & 7u)) return SBE_EINVAL;
    const uint64_t tiles = (n + kTile - 1) / kTile;
    if (tiles > kMaxTiles) return SBE_EINVAL;
    if (!workspace || workspace_bytes < sbe_encode_workspace_size(n)) return SBE_ENOSPC;
    if (reinterpret_cast<uintptr_t>(workspace) & 63u) return SBE_EINVAL;
    uint8_t* ws = static_cast<uint8_t*>(workspace);
    const uint64_t cap_tiles = (workspace_bytes - sizeof(EncWorkspace)) / 32;
    EncArgs a{in->arena, in->str_off, in->str_len, in->timestamp, n, ts_default, out, out_capacity, out_off,
              status, reinterpret_cast<EncWorkspace*>(ws), reinterpret_cast<uint64_t*>(ws + sizeof(EncWorkspace)),
              cap_tiles};
    const dim3 grid((uint32_t)tiles), block(kWave);
    const bool packed = in->str_off == nullptr;
    const bool trunc = (flags & SBE_ENC_REF_TRUNCATE8) != 0;
    if (packed && !trunc) hipLaunchKernelGGL((sbe_encode_kernel<true, false>), grid, block, 0, s, a);
    else if (packed && trunc) hipLaunchKernelGGL((sbe_encode_kernel<true, true>), grid, block, 0, s, a);
    else if (!packed && !trunc) hipLaunchKernelGGL((sbe_encode_kernel<false, false>), grid, block, 0, s, a);
    else hipLaunchKernelGGL((sbe_encode_kernel<false, true>), grid, block, 0, s, a);
    return record_hip(hipGetLastError());
}

int sbe_decode_batch(const uint8_t* in, const uint64_t* rec_off, uint64_t n, uint32_t mode,
                     const sbe_decoded* out, void* stream) {
    if (mode != SBE_DEC_PARSE_MESSAGE && mode != SBE_DEC_ON_EGRESS) return SBE_EINVAL;
    if (n == 0) return SBE_OK;
    if (!in || !rec_off || !out || !out->status || !out->flags || !out->hdr || !out->ts || !out->view_off ||
        !out->view_len)
        return SBE_EINVAL;
    if ((reinterpret_cast<uintptr_t>(in) & 15u) || (reinterpret_cast<uintptr_t>(rec_off) & 7u) ||
        (reinterpret_cast<uintptr_t>(out->hdr) & 7u) || (reinterpret_cast<uintptr_t>(out->ts) & 7u) ||
        (reinterpret_cast<uintptr_t>(out->view_off) & 3u) || (reinterpret_cast<uintptr_t>(out->view_len) & 3u))
        return SBE_EINVAL;
    const uint64_t tiles = (n + kTile - 1) / kTile;
    if (tiles > kMaxTiles) return SBE_EINVAL;
    DecArgs a{in, rec_off, n, out->status, out->flags, out->hdr, out->ts, out->view_off, out->view_len};
    hipStream_t s = reinterpret_cast<hipStream_t>(stream);
    const dim3 grid((uint32_t)tiles), block(kWave);
    if (mode == SBE_DEC_ON_EGRESS)
        hipLaunchKernelGGL((sbe_decode_kernel<SBE_DEC_ON_EGRESS>), grid, block, 0, s, a);
    else
        hipLaunchKernelGGL((sbe_decode_kernel<SBE_DEC_PARSE_MESSAGE>), grid, block, 0, s, a);
    return record_hip(hipGetLastError());
}

}  // extern "C"
