// sbe_codec.hip — MI355X (gfx950) batch SBE codec: HIP kernels + the C ABI of include/sbecodec.h.
//
// Byte packing, not a contraction: no MFMA.  Both kernels are HBM-stream kernels whose LDS windows
// turn the per-record byte scatter / gather into coalesced 16-byte HBM accesses.
//
//  encode  (SBEEncoder::encode_topic_message, src/sbe_encoder.cpp:131-167, and the session / Lite
//           layouts), two launches:
//    sbe_enc_sums  one 1024-thread workgroup per superblock of 128 tiles: each tile's output /
//                  packed-input byte prefix inside its superblock, the superblock totals
//    sbe_enc_pack  persistent, one wave per workgroup, tiles of 32 records (two lanes per record;
//                  the session and Lite layouts 64, a lane per record; Lay::kRpt), windows whose
//                  chunks would leave some lane more than 8 rebalanced over the lanes:
//                  record offsets by a DPP wave scan; output windows of <= 8 KiB holding whole
//                  records; the next window's input strings loaded into registers while the current
//                  one is composed (b128 chunk composition from the staged input: five LDS dword
//                  reads + four v_alignbyte per 16-byte chunk, a zone fix-up pass for string starts
//                  inside a chunk, literal headers / lengths as byte stores); the window stored with
//                  16-byte buffer stores (nt)
//  decode  (MessageParser::parse_message :513-551 / MessageHandler::on_egress
//           include/aeron_cluster/message_handler.hpp:35-68 + decode_ack src/ack_decoder.cpp:29-105 /
//           the Lite flyweights), one launch, one wave per 64-record tile:
//    1. the tile's bytes are staged window by window (16 KiB windows; 20 KiB for batches of records
//       of 257-320 B on average, 13 KiB above, 15 KiB up to 204 B, 8 KiB up to 112 B:
//       sbe_decode_batch_sized) into
//       an XOR-swizzled LDS window with 16-byte loads; the second
//       window's loads are issued before the first one is parsed
//    2. each lane parses its record from LDS (template-ID dispatch per lane) and writes the
//       descriptor SoA; records no window can hold are parsed from HBM.
#include <hip/hip_ext.h>
#include <hip/hip_runtime.h>
#include <dlfcn.h>
#include <rccl/rccl.h>  // types only: the library is dlopen-ed (rccl_api)

#include <chrono>
#include <mutex>
#include <new>
#include <thread>
#include <type_traits>

#include <cstdint>
#include <cstdio>
#include <cstring>

#include "../../include/sbecodec.h"

namespace {

constexpr int kWave = 64;
constexpr int kTile = 64;                 // records per workgroup (one per lane)
// LDS window bytes of the decode kernel: kWin for records up to 256 B on average (a 64-record
// tile in one window), kWinWide for 257-320 B (a 64-record tile of 280-B session frames, 17.9 KB,
// whole in one 20 KiB window: 8 workgroups per CU, where 12 KiB windows allowed 13 but took two
// windows a tile; session-frame decode 71.8-73.7 -> 64.2-65.1 us, 300-B records 1890 -> 1846 us,
// 320-B 1844 -> 1791 us at 4 M; 18 KiB read 64.1 us on the frames but 2300 / 2396 us on the 300 /
// 320-B records, which it cannot hold whole; profiles/r06_ab_decsess{,2}.log, r06_ab_declarge.log).
// sbe_decode_batch_sized picks by the batch's average record size.
#ifndef SBE_DEC_WIN
#define SBE_DEC_WIN 16384
#endif
#ifndef SBE_DEC_WIN_WIDE
#define SBE_DEC_WIN_WIDE 20480
#endif
constexpr uint32_t kWin = SBE_DEC_WIN;
constexpr uint32_t kWinWide = SBE_DEC_WIN_WIDE;
constexpr uint64_t kWideAvg = 256;  // average record bytes above which the kWinWide kernel runs
// Tiles of shorter records leave most of a 16 KiB window empty, and the window's LDS is what caps
// the workgroups (and so the bytes in flight) per CU: batches of records up to kMidAvg / kSmallAvg
// bytes on average take a 14 / 8 KiB window (64 records of 204 B average fill 12.8 KiB; a tile past
// the window takes a second one, as any tile does).
#ifndef SBE_DEC_SMALL_AVG  // A/B builds only
#define SBE_DEC_SMALL_AVG 112
#endif
#ifndef SBE_DEC_MID_AVG
#define SBE_DEC_MID_AVG 204
#endif
// 15 KiB: config 3 (1 M mixed TM / Ack records, 200 B on average) decodes in 56.6 us against 60.0
// at 14 KiB, 60.5 at 16 KiB and 64.1 at 13 KiB (A/B in one process, profiles/r05_ab_decmid.log,
// profiles/r04_ab_decmid.log): a CU then holds 10 workgroups instead of 11, but the tiles a 14 KiB
// window cannot hold whole no longer pay a second window.
#ifndef SBE_DEC_WIN_MID  // A/B builds only
#define SBE_DEC_WIN_MID 15360
#endif
constexpr uint32_t kWinMid = SBE_DEC_WIN_MID, kWinSmall = 8192;
// Batches of records over kLargeAvg bytes on average (config 4: 387 B) take a 13 KiB window: a
// 64-record tile of ~24.8 KB then fits two windows (12 KiB windows hold ~24.2 KB in two, so most
// tiles paid a third).  Config 4 decode 422.4 -> 405.8 us at 4 M records (profiles/r05_ab_decwide.log).
// Windows holding most config-4 tiles whole (25 / 27 KiB, 6 workgroups per CU) read 685.7 / 632.5
// against 405.3 us (profiles/r06_ab_declarge.log).
#ifndef SBE_DEC_WIN_LARGE  // A/B builds only
#define SBE_DEC_WIN_LARGE 13312
#endif
#ifndef SBE_DEC_LARGE_AVG
#define SBE_DEC_LARGE_AVG 320
#endif
constexpr uint32_t kWinLarge = SBE_DEC_WIN_LARGE;
constexpr uint64_t kLargeAvg = SBE_DEC_LARGE_AVG;
constexpr uint64_t kMidAvg = SBE_DEC_MID_AVG, kSmallAvg = SBE_DEC_SMALL_AVG;

// ------------------------------------------------------------------------------------------
// LDS window.  Dword i of the window lives at i ^ ((i >> 6) & 28): within each 256-B row (64
// dwords) the 16-byte chunk slots are XOR-permuted by the row index, so lanes reading dword j of
// records 256 B apart spread over 8 chunk slots, while a chunk stays whole and in order in one
// aligned slot (chunk copies are plain ds_*_b128).  A 2-bit in-chunk dword permutation on top of it
// (i ^ ((i >> 6) & 31)) spread them over more banks but cost ~8 selects per staged chunk: decode
// 2.7 % (fixed-256) and 3 % (config 4) slower.
// ------------------------------------------------------------------------------------------
__device__ __forceinline__ uint32_t swz(uint32_t i) { return i ^ ((i >> 6) & 28u); }

// chunk c (16 B) of the window
__device__ __forceinline__ uint4 lds_read_chunk(const uint32_t* win, uint32_t c) {
    const uint32_t x = (c >> 4) & 31u;
    return *reinterpret_cast<const uint4*>(win + ((4u * c) ^ (x & 28u)));
}

__device__ __forceinline__ void lds_write_chunk(uint32_t* win, uint32_t c, uint4 v) {
    const uint32_t x = (c >> 4) & 31u;
    *reinterpret_cast<uint4*>(win + ((4u * c) ^ (x & 28u))) = v;
}

__device__ __forceinline__ uint32_t lds_dw(const uint32_t* win, uint32_t i) { return win[swz(i)]; }
// the four dwords of logical chunk c (the same as lds_read_chunk)
__device__ __forceinline__ uint4 lds_read_chunk_raw(const uint32_t* win, uint32_t c) {
    return *reinterpret_cast<const uint4*>(win + ((4u * c) ^ (((c >> 4) & 31u) & 28u)));
}

// ------------------------------------------------------------------------------------------
// wave helpers
// ------------------------------------------------------------------------------------------
// Cross-lane steps on DPP (VALU data movement, no LDS round trip):
//   row_shr:n (0x110 + n) within rows of 16 lanes; row_bcast:15 (0x142) / row_bcast:31 (0x143)
//   carry lane 15 / lane 31 into the following rows; quad_perm (0x00-0xff) within quads.
// update_dpp(old, src, ...) yields `old` (0 here) where the source lane is out of range or the
// row is masked off, so the adds below are Hillis-Steele steps.
template <int kCtrl, int kRowMask = 0xf>
__device__ __forceinline__ uint32_t dpp0(uint32_t v) {
    return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, kCtrl, kRowMask, 0xf, false);
}

// inclusive prefix sum over the 64 lanes
__device__ __forceinline__ uint32_t wave_incl_scan(uint32_t v, int lane) {
    (void)lane;
    v += dpp0<0x111>(v);
    v += dpp0<0x112>(v);
    v += dpp0<0x114>(v);
    v += dpp0<0x118>(v);
    v += dpp0<0x142, 0xa>(v);
    v += dpp0<0x143, 0xc>(v);
    return v;
}

// ceil(a / b) for a, b < 2^20, b > 0: a float reciprocal estimate corrected by one step either
// way (exact), instead of the compiler's ~20-instruction u32 division
__device__ __forceinline__ uint32_t ceil_div_small(uint32_t a, uint32_t b) {
    const uint32_t x = a + b - 1;
    uint32_t q = (uint32_t)((float)x * __builtin_amdgcn_rcpf((float)b));
    q += (q + 1) * b <= x;
    q -= q * b > x;
    return q;
}

// inclusive max over the 64 lanes of values >= 0 (0 is the identity DPP fills in)
__device__ __forceinline__ uint32_t wave_incl_max(uint32_t v) {
    v = max(v, dpp0<0x111>(v));
    v = max(v, dpp0<0x112>(v));
    v = max(v, dpp0<0x114>(v));
    v = max(v, dpp0<0x118>(v));
    v = max(v, dpp0<0x142, 0xa>(v));
    v = max(v, dpp0<0x143, 0xc>(v));
    return v;
}

// the same on 64-bit values (lo / hi halves with the carries of the lo adds)
template <int kCtrl, int kRowMask = 0xf>
__device__ __forceinline__ uint64_t dpp_add64(uint64_t v) {
    const uint32_t lo = (uint32_t)v, hi = (uint32_t)(v >> 32);
    const uint32_t tlo = dpp0<kCtrl, kRowMask>(lo), thi = dpp0<kCtrl, kRowMask>(hi);
    const uint32_t nlo = lo + tlo;
    return ((uint64_t)(hi + thi + (nlo < lo ? 1u : 0u)) << 32) | nlo;
}
__device__ __forceinline__ uint64_t wave_incl_scan64(uint64_t v, int lane) {
    (void)lane;
    v = dpp_add64<0x111>(v);
    v = dpp_add64<0x112>(v);
    v = dpp_add64<0x114>(v);
    v = dpp_add64<0x118>(v);
    v = dpp_add64<0x142, 0xa>(v);
    v = dpp_add64<0x143, 0xc>(v);
    return v;
}

// lane-uniform value of lane `l` (l uniform)
__device__ __forceinline__ uint32_t lane_u32(uint32_t v, int l) { return __builtin_amdgcn_readlane(v, l); }
// (the builtin returns int: each half goes through uint32_t, or the low word would sign-extend
// into the high one whenever its bit 31 is set)
__device__ __forceinline__ uint64_t lane_u64(uint64_t v, int l) {
    const uint32_t hi = (uint32_t)__builtin_amdgcn_readlane((uint32_t)(v >> 32), l);
    const uint32_t lo = (uint32_t)__builtin_amdgcn_readlane((uint32_t)v, l);
    return ((uint64_t)hi << 32) | lo;
}

// sum over the 64 lanes, uniform
__device__ __forceinline__ uint64_t wave_sum64(uint64_t v) { return lane_u64(wave_incl_scan64(v, 0), kWave - 1); }

__device__ __forceinline__ uint64_t uniform64(uint64_t v) {
    uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)v);
    uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)(v >> 32));
    return ((uint64_t)hi << 32) | lo;
}

__device__ __forceinline__ uint32_t byte_mask_bits(uint32_t nbytes) {
    return nbytes >= 4 ? 0xffffffffu : ((1u << (8u * nbytes)) - 1u);
}

// Global-memory accesses through address_space(1) pointers: integer address arithmetic would
// otherwise degrade them to flat_* instructions, which also count on lgkmcnt and make every LDS
// read wait for outstanding memory loads.
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(1))) const uint32_t g_u32;
typedef __attribute__((address_space(1))) const u32x4 g_u32x4;
__device__ __forceinline__ uint32_t gload32(uintptr_t addr) { return *reinterpret_cast<g_u32*>(addr); }
__device__ __forceinline__ uint4 gload128(uintptr_t addr) {
    const u32x4 v = *reinterpret_cast<g_u32x4*>(addr);
    return make_uint4(v.x, v.y, v.z, v.w);
}
// streamed-once loads / stores with the non-temporal cache policy (nt)
__device__ __forceinline__ uint4 gload128_nt(uintptr_t addr) {
    const u32x4 v = __builtin_nontemporal_load(reinterpret_cast<g_u32x4*>(addr));
    return make_uint4(v.x, v.y, v.z, v.w);
}
// decode descriptor stores: written once, read by the host or the next kernel
template <typename T>
__device__ __forceinline__ void dst_store(T* p, T v) {
    __builtin_nontemporal_store(v, p);
}

// ------------------------------------------------------------------------------------------
// Encode: two launches, no inter-workgroup hand-off inside either.
//   K1 sbe_enc_sums   one workgroup per 4096-record superblock: every 32-record tile's output /
//                     packed-input byte prefix inside its superblock, and the superblock totals
//   K3 sbe_enc_pack   persistent, one wave per tile: the superblock totals before the tile (a
//                     running sum per workgroup: its tiles come in increasing order), record
//                     offsets, LDS-staged input, per-lane record composition into an LDS output
//                     window, coalesced 16-byte stores
// ------------------------------------------------------------------------------------------
constexpr int kSbThreads = 1024;
constexpr int kTilesPerSb = 2 * kWave;  // tiles per superblock (one K1 workgroup)
constexpr int kSbRecMin = kTilesPerSb * 32;  // records per superblock of the smallest tile shape

// Record layouts (compile-time): kPre bytes of session header, the 8-byte SBE header, a kBlk-byte
// fixed block, then kNF u16-length-prefixed strings.
//   LayTM   TopicMessage                     TopicMessage.h:98-1435
//   LayTMS  SessionMessageHeader + TopicMessage  src/session_manager.cpp:936-967, :1118-1144
//   LayL2   CommitOffsetLite (301)           include/model/CommitOffsetLite.h:114-118
//   LayL3   OrderRequestLite / OrderNotificationLite (201 / 202)  OrderRequestLite.h:114-118
// kRpt: records per K3 tile (one wave), kLpr = 64 / kRpt lanes per record.  32-record tiles (two
// lanes a record) for the TopicMessage layout, whose 256-B Order records fill one 8 KiB window
// per tile; 64-record tiles (a lane a record, chunks rebalanced over the lanes) for the session
// frames and Lite records, whose 32-record tiles (8.8 / 2.5 / 10.4 KiB) leave windows part full:
// measured session pack 156 -> 144 us, CommitOffsetLite 61 -> 43, OrderRequestLite 167 -> 150
// (fixed-256 TopicMessage 90 -> 93, variable-length unchanged).
template <int kPre_, int kBlk_, int kNF_, bool kTM_, int kRpt_>
struct Lay {
    static constexpr int kRpt = kRpt_;
    static constexpr int kLpr = kWave / kRpt;
    static constexpr int kSbRec = kTilesPerSb * kRpt;  // records per superblock
    static_assert((kRpt == 32 || kRpt == 64) && kSbRec % kSbThreads == 0 && kSbThreads % kRpt == 0, "tile shape");
    static constexpr int32_t kPre = kPre_;
    static constexpr int32_t kBlk = kBlk_;
    static constexpr int kNF = kNF_;
    static constexpr bool kTM = kTM_;                 // TopicMessage block (timestamp default, truncation)
    // staged-input loads nontemporal: the input is read once.  On inputs that rotate over three
    // buffer sets (no step finds its input in the 256 MB MALL, as streaming data would not) they
    // read fixed-256 96.0 -> 94.2 us, config 4 723.3 -> 716.6, OrderRequestLite 146.3 -> 143.8,
    // session frames 137.7 -> 137.2 (profiles/r06_ab_ntl_rot.log); only a batch re-read every step
    // (rounds 1-5's bench) prefers the default policy, whose lines the MALL keeps (86.6 vs 93.9 us)
#ifndef SBE_PACK_NTL  // A/B builds: 0 = never, 1 = TopicMessage / OrderRequestLite, 2 = always
#define SBE_PACK_NTL 2
#endif
    static constexpr bool kNtIn = SBE_PACK_NTL == 2 || (SBE_PACK_NTL == 1 && (kTM_ ? kPre_ == 0 : kNF_ == 3));
    static constexpr int32_t kLit = kPre + 8 + kBlk;  // literal prefix bytes (multiple of 4)
    static constexpr int32_t kS0 = kLit + 2;          // first string byte
    static constexpr int32_t kOvh = kLit + 2 * kNF;   // wire overhead
    static constexpr int32_t ovh(bool trunc) { return kOvh - (trunc ? 8 : 0); }
    // window store rows issued unconditionally (store_window): CommitOffsetLite's 32-record tiles
    // (~77-B records) are ~2.5 KiB, three of the eight 1-KiB rows
    static constexpr int kStoreRows0 = kNF == 2 ? (kRpt == 64 ? 5 : 3) : 8;
};
#ifndef SBE_TM_RPT
#define SBE_TM_RPT 32  // A/B builds only (scripts/abv.py)
#endif
// Session frames take 32-record tiles (two lanes a record) since the pack loop is chosen per launch:
// their virtual tiles fill one 8 KiB window with ~29 frames, which two lanes a record compose in
// one pass (session pack 131.8 -> 126.1 us on rotated inputs, profiles/r06_ab_rpt.log; with the
// tile loop alone 64-record tiles had won, 156 -> 144 us, round 3).  OrderRequestLite keeps 64
// (144.4 -> 155.3 us with 32).
#ifndef SBE_TMS_RPT
#define SBE_TMS_RPT 32
#endif
#ifndef SBE_L3_RPT
#define SBE_L3_RPT 64  // A/B builds only
#endif
using LayTM = Lay<0, 16, 5, true, SBE_TM_RPT>;
using LayTMS = Lay<32, 16, 5, true, SBE_TMS_RPT>;
using LayL2 = Lay<0, 12, 2, false, 64>;
using LayL3 = Lay<0, 12, 3, false, SBE_L3_RPT>;
static_assert(LayTM::kOvh == SBE_TM_WIRE_OVERHEAD && LayTM::ovh(true) == SBE_TM_REF_OVERHEAD, "TM layout");
static_assert(LayL2::kOvh == SBE_LITE_OVERHEAD(2) && LayTMS::kPre == SBE_SESSION_HDR_LEN, "layouts");
// the layout's tile shape as local constants (functions templated on the layout)
#define SBE_TILE_SHAPE(LY)                                                  \
    [[maybe_unused]] constexpr int kRpt = LY::kRpt, kLpr = LY::kLpr; \
    [[maybe_unused]] constexpr int kSbRec = LY::kSbRec

struct EncArgs {
    const uint8_t* arena;
    const uint32_t* str_off;
    const uint32_t* str_len;   // [n][kNF]
    const uint64_t* timestamp; // TopicMessage timestamp / Lite sequence
    const uint32_t* topic_id;  // Lite topicId
    uint32_t tmpl;             // Lite template id
    int64_t term_id, sess_id;  // session header
    uint64_t n;
    uint64_t ts_default;
    uint8_t* out;
    uint64_t cap;
    uint64_t* out_off;
    uint8_t* status;
    uint64_t* tsum;  // [tiles][2]        output / input bytes before the tile within its superblock
    uint64_t* bsum;  // [superblocks][2]  output / input bytes of the superblock
    uint8_t* sink;   // kSinkBytes of workspace: target of the pack kernel's don't-care stores
};
constexpr int kSinkBytes = 16 * 64;

// Cache policy of the pack kernel's output stores (buffer stores; 2 = nt: the stream is written
// once and read by the next kernel or the host, not from this kernel's caches)
constexpr int kOutAux = 2;

// Record length modes of the TopicMessage encoders:
//   kLenWire  the wire record, 34+Σlen (computeLength's E109 above 65534 B)
//   kLenRef   SBEEncoder::encode_topic_message's 26+Σlen prefix (src/sbe_encoder.cpp:163-164)
//   kLenPub   ClusterClient::publish_topic (src/cluster_client.cpp:1850-1857): wire length, each
//             length taken mod 65536 by put*(const char*, std::uint16_t) (TopicMessage.h:515-529),
//             no E109; the packed input still advances by the full lengths
enum : int { kLenWire = 0, kLenRef = 1, kLenPub = 2 };

// Sizes of record r: output bytes (0 on E109) and packed-input bytes (its strings, always).
template <class LY, int kLen>
__device__ __forceinline__ void rec_sizes(const EncArgs& a, uint64_t r, uint32_t& out_b, uint64_t& in_b,
                                          uint8_t& st) {
    uint32_t sum = 0;
    uint64_t sum_in = 0;
    st = SBE_ENC_OK;
    if (r < a.n) {
#pragma unroll
        for (int f = LY::kNF - 1; f >= 0; --f) {  // first failing field in wire order (TopicMessage.h:1396-1428)
            const uint32_t L = a.str_len[LY::kNF * r + f];
            sum += kLen == kLenPub ? (L & 0xffffu) : L;
            sum_in += L;
            if (kLen != kLenPub && L > SBE_VAR_MAX_LEN) st = (uint8_t)(SBE_ENC_E109_TOPIC + f);
        }
    }
    const uint32_t ovh = (uint32_t)LY::ovh(kLen == kLenRef);
    out_b = (r < a.n && st == SBE_ENC_OK) ? ovh + sum : 0u;
    in_b = r < a.n ? sum_in : 0u;
}


// K1: superblock sb = records [4096 sb, 4096 (sb+1)).  Thread t takes records t, t+1024, t+2048,
// t+3072 of it (each load instruction of a wave then covers 1280 contiguous bytes of lengths); the
// 32 records of a tile are 32 consecutive threads.  Tile sums go through LDS to one wave, which
// writes the 128 tile prefixes and the superblock's totals.
template <class LY, bool kPacked, int kLen>
__global__ __launch_bounds__(kSbThreads) void sbe_enc_sums(EncArgs a) {
    SBE_TILE_SHAPE(LY);
    __shared__ uint64_t tl[2][kTilesPerSb];
    const int tid = threadIdx.x;
    const uint64_t sb = blockIdx.x;
#pragma unroll
    for (int j = 0; j < kSbRec / kSbThreads; ++j) {
        const uint64_t r = sb * kSbRec + (uint64_t)j * kSbThreads + tid;
        uint32_t ob;
        uint64_t ib;
        uint8_t st;
        rec_sizes<LY, kLen>(a, r, ob, ib, st);
        // per tile (kRpt consecutive lanes: two 32-record tiles or one 64-record tile per wave):
        // one DPP scan over the wave, the tiles' sums read at lanes 31 and 63 (input side in 64
        // bits: E109 records may carry up to 5 x 4 GiB of strings)
        const int lane = tid & (kWave - 1);
        const uint32_t so = wave_incl_scan(ob, lane);
        const uint32_t o31 = lane_u32(so, 31), o63 = lane_u32(so, kWave - 1);
        uint64_t i31 = 0, i63 = 0;
        if (kPacked) {
            const uint64_t si = wave_incl_scan64(ib, lane);
            i31 = lane_u64(si, 31);
            i63 = lane_u64(si, kWave - 1);
        }
        if (lane == 0) {
            const int tile = j * (kSbThreads / kRpt) + (kWave / kRpt) * (tid / kWave);
            if (kRpt == 32) {
                tl[0][tile] = o31;
                tl[1][tile] = i31;
                tl[0][tile + 1] = o63 - o31;
                tl[1][tile + 1] = i63 - i31;
            } else {
                tl[0][tile] = o63;
                tl[1][tile] = i63;
            }
        }
    }
    __syncthreads();
    if (tid < kWave) {  // exclusive scan of the superblock's tile sums, kTilesPerSb / 64 per lane
        const int lane = tid;
        constexpr int kPer = kTilesPerSb / kWave;
        const uint64_t o0 = tl[0][kPer * lane], o1 = kPer == 2 ? tl[0][kPer * lane + 1] : 0ull;
        const uint64_t i0 = tl[1][kPer * lane], i1 = kPer == 2 ? tl[1][kPer * lane + 1] : 0ull;
        const uint64_t io = wave_incl_scan64(o0 + o1, lane), ii = wave_incl_scan64(i0 + i1, lane);
        const uint64_t eo = io - o0 - o1, ei = ii - i0 - i1;
        const uint64_t t0 = sb * kTilesPerSb + kPer * lane;
        *reinterpret_cast<ulonglong2*>(a.tsum + 2 * t0) = make_ulonglong2(eo, ei);
        if (kPer == 2) *reinterpret_cast<ulonglong2*>(a.tsum + 2 * t0 + 2) = make_ulonglong2(eo + o0, ei + i0);
        if (lane == kWave - 1) *reinterpret_cast<ulonglong2*>(a.bsum + 2 * sb) = make_ulonglong2(io, ii);
    }
}

#ifndef SBE_PACK_MIN_WAVES  // minimum waves per SIMD the pack kernel's registers must allow
#define SBE_PACK_MIN_WAVES 1
#endif
#ifndef SBE_ENC_WIN
#define SBE_ENC_WIN 8192
#endif
constexpr int32_t kEW = SBE_ENC_WIN;            // output window bytes per pass
constexpr int32_t kEWIn = SBE_ENC_WIN + 256;    // staged input bytes per pass

// ---- K3 LDS layout -------------------------------------------------------------------------
// Input window: linear bytes (window byte 0 sits kInSlack bytes into the array, so the reads a
// lane makes up to 4 bytes before / 8 bytes after a string stay inside it); per-lane string
// reads are ds_read_b32 at immediate offsets from one base.  Output window: 256-byte rows
// padded by 8 bytes, so the two lanes of each of 32 records (256 B apart) write banks
// 2r + 32q + k: at most 2-way, which ds_write_b32 absorbs.
constexpr int32_t kInSlack = 64;
constexpr int32_t kRowPad = 16;
constexpr int32_t kWoutBytes = kEW + (kEW / 256) * kRowPad;
constexpr int32_t kWinBytes = kEWIn + 2 * kInSlack;

// LDS pointers keep their address space through structs and non-inlined calls (a generic
// pointer there would turn every window access into a flat_* instruction).
typedef __attribute__((address_space(3))) uint8_t lds_u8;
typedef __attribute__((address_space(3))) const uint8_t lds_cu8;
typedef __attribute__((address_space(3))) uint32_t lds_u32;
typedef __attribute__((address_space(3))) const uint32_t lds_cu32;
typedef unsigned int u32x2 __attribute__((ext_vector_type(2)));
typedef __attribute__((address_space(3))) u32x4 lds_u32x4;
typedef __attribute__((address_space(3))) const u32x2 lds_cu32x2;
typedef __attribute__((address_space(3))) u32x2 lds_u32x2;
__device__ __forceinline__ void lds_store16(lds_u8* p, uint4 v) {
    u32x4 x;
    x.x = v.x; x.y = v.y; x.z = v.z; x.w = v.w;
    *reinterpret_cast<lds_u32x4*>(p) = x;
}

__device__ __forceinline__ uint32_t wout_addr(int32_t d) { return (uint32_t)d + (((uint32_t)d >> 8) * kRowPad); }

// Sources of string dwords: dw(i) = the aligned dword i of the source (byte 4i..4i+3).
struct LdsLin {
    lds_cu8* b;  // window byte 0
    __device__ __forceinline__ uint32_t dw(int32_t i) const { return reinterpret_cast<lds_cu32*>(b)[i]; }
};
struct GlbClamp {  // global memory; reads outside [imin, imax] fetch a neighbour (only don't-care bytes)
    uintptr_t base4;
    int32_t imax;
    __device__ __forceinline__ uint32_t dw(int32_t i) const {
        i = i < 0 ? 0 : (i > imax ? imax : i);
        return gload32(base4 + 4u * (uint32_t)i);
    }
};

__device__ __forceinline__ uint64_t low_bytes64(uint64_t v, int32_t n) { return n >= 8 ? v : v & ((1ull << (8 * n)) - 1); }

// Streams one lane's part of a record into the output window as whole-dword writes: `carry`
// holds the bytes [pos & ~3, pos) not yet written (zero above them; bytes below `lo` belong to the
// previous record and are never written).  Only the part's first and last dwords, which a
// record boundary may share with a neighbour, are written byte by byte.
struct Writer {
    lds_u8* w;
    int32_t lo, pos;
    uint32_t carry;

    __device__ __forceinline__ void put_dw(int32_t d, uint32_t v) const {
        *reinterpret_cast<lds_u32*>(w + wout_addr(d)) = v;
    }
    __device__ __forceinline__ void put_bytes(int32_t d, uint32_t v, int32_t b0, int32_t b1) const {
        lds_u8* p = w + wout_addr(d);
#pragma unroll
        for (int k = 0; k < 4; ++k)
            if (k >= b0 && k < b1) p[k] = (uint8_t)(v >> (8 * k));
    }
    __device__ __forceinline__ void put_first(int32_t d, uint32_t v) const {
        if (d >= lo) put_dw(d, v); else put_bytes(d, v, lo - d, 4);
    }
    // n (1..8) literal bytes, v zero above them
    __device__ __forceinline__ void lit(uint64_t v, int32_t n) {
        const int32_t t = pos & 3, d = pos & ~3, total = t + n;
        const uint64_t lo64 = (v << (8 * t)) | carry;
        const uint32_t x0 = (uint32_t)lo64, x1 = (uint32_t)(lo64 >> 32);
        const uint32_t x2 = t ? (uint32_t)(v >> (64 - 8 * t)) : 0u;
        if (total >= 4) put_first(d, x0);
        if (total >= 8) put_dw(d + 4, x1);
        carry = total >= 8 ? x2 : (total >= 4 ? x1 : x0);
        pos += n;
    }
    // m >= 1 bytes from source bytes [s, s+m): output dword d+4k takes source bytes
    // [u+4k, u+4k+4), u = s - (pos & 3) — one v_alignbyte of two source dwords.
    template <typename Src>
    __device__ __forceinline__ void str(const Src& S, int32_t s, int32_t m) {
        const int32_t t = pos & 3, d = pos & ~3, total = t + m;
        const int32_t u = s - t;
        const uint32_t sh = (uint32_t)u & 3u;
        const int32_t i0 = u >> 2;
        const int32_t nd = total >> 2, rem = total & 3;
        uint32_t prev = S.dw(i0);
        const uint32_t nx = S.dw(i0 + 1);
        const uint32_t w0 = (__builtin_amdgcn_alignbyte(nx, prev, sh) & ~byte_mask_bits((uint32_t)t)) | carry;
        pos += m;
        if (nd == 0) {
            carry = w0 & byte_mask_bits((uint32_t)total);
            return;
        }
        put_first(d, w0);
        prev = nx;
        int32_t k = 1;
        // single dwords up to a 16-byte output boundary, then whole 16-byte groups (never
        // across a padded row: one address, one ds_write2_b64), then the tail
        const int32_t kg = 4 - ((d >> 2) & 3);
        for (; k < kg && k < nd; ++k) {
            const uint32_t n0 = S.dw(i0 + k + 1);
            put_dw(d + 4 * k, __builtin_amdgcn_alignbyte(n0, prev, sh));
            prev = n0;
        }
        for (; k + 4 <= nd; k += 4) {
            const uint32_t n0 = S.dw(i0 + k + 1), n1 = S.dw(i0 + k + 2), n2 = S.dw(i0 + k + 3), n3 = S.dw(i0 + k + 4);
            u32x2 lo2, hi2;
            lo2.x = __builtin_amdgcn_alignbyte(n0, prev, sh);
            lo2.y = __builtin_amdgcn_alignbyte(n1, n0, sh);
            hi2.x = __builtin_amdgcn_alignbyte(n2, n1, sh);
            hi2.y = __builtin_amdgcn_alignbyte(n3, n2, sh);
            lds_u8* g = w + wout_addr(d + 4 * k);
            reinterpret_cast<lds_u32x2*>(g)[0] = lo2;
            reinterpret_cast<lds_u32x2*>(g)[1] = hi2;
            prev = n3;
        }
        for (; k < nd; ++k) {
            const uint32_t n0 = S.dw(i0 + k + 1);
            put_dw(d + 4 * k, __builtin_amdgcn_alignbyte(n0, prev, sh));
            prev = n0;
        }
        carry = rem ? (__builtin_amdgcn_alignbyte(S.dw(i0 + nd + 1), prev, sh) & byte_mask_bits((uint32_t)rem)) : 0u;
    }
    __device__ __forceinline__ void flush() const {
        const int32_t t = pos & 3;
        if (t) {
            const int32_t d = pos & ~3;
            put_bytes(d, carry, lo > d ? lo - d : 0, t);
        }
    }
};

// string bytes from global memory (gather mode, or outside the staged window)
__device__ __noinline__ Writer str_global(Writer W, uintptr_t sa, int32_t m) {
    const uintptr_t b4 = sa & ~(uintptr_t)3;
    const int32_t sl = (int32_t)(sa - b4);
    W.str(GlbClamp{b4, (sl + m - 1) >> 2}, sl, m);
    return W;
}

// K3 workgroups are one wave, whose LDS accesses execute in issue order: a phase change needs only
// a compiler barrier.  (__syncthreads() would also wait on vmcnt(0), draining the next tile's
// prefetch loads and this tile's stores at every phase.)
__device__ __forceinline__ void wsync() { __builtin_amdgcn_wave_barrier(); }

// ---- K3: persistent, software-pipelined pack kernel ---------------------------------------
// One wave per workgroup loops over tiles t = blockIdx.x, += gridDim.x.  While it composes tile
// t it already holds tile t+G's staged-input loads in flight (registers) and tile t+2G's lengths,
// so the two dependent HBM round trips of a tile hide behind the previous tile's work.  Each
// record is composed by kLpr lanes (one contiguous part each) into an XOR-swizzled LDS output
// window, which the wave then stores with global_store_dwordx4 (1 KiB per instruction).
constexpr int kStageRegs = (kEWIn / 16 + kWave - 1) / kWave;  // uint4 staging registers per lane

// Diagnosis build only (-DSBE_PACK_PHASES, scripts/abv.py): per-wave core-clock time of the pack
// loop's phases, read back by sbe_debug_phases.  The product build compiles the laps away.
#ifdef SBE_PACK_PHASES
__device__ uint64_t g_pack_phase[16384 * 8];
struct Ph {
    uint64_t t, acc[8];
    __device__ void start() {
        t = __builtin_amdgcn_s_memtime();
        for (int k = 0; k < 8; ++k) acc[k] = 0;
    }
    __device__ void lap(int k) {
        const uint64_t n = __builtin_amdgcn_s_memtime();
        acc[k] += n - t;
        t = n;
    }
    __device__ void put(int lane) {  // lane k writes phase k: a vector store
        uint64_t v = 0;
        for (int k = 0; k < 8; ++k) v = lane == k ? acc[k] : v;
        if (lane < 8 && blockIdx.x < 16384) g_pack_phase[8 * blockIdx.x + lane] = v;
    }
};
#else
struct Ph {
    __device__ void start() {}
    __device__ void lap(int) {}
    __device__ void put(int) {}
};
#endif

struct TileIn {  // raw per-lane loads of one tile
    uint32_t L[5];
    uint64_t ts;      // timestamp (TopicMessage) / sequence (Lite)
    uint32_t tid;     // Lite topicId
    // tile start = (superblock totals before the tile) + tile prefix inside its superblock, for
    // output / packed input.  The superblock totals the workgroup has not yet summed come as
    // per-lane partials (po, pi); tile_prepare reduces them: an add here would wait on these
    // loads, and vmcnt retires in order, so on the prefetch too.
    uint64_t to, ti, po, pi;
    uint32_t pcount;  // uniform: lanes [0, pcount) of po / pi are superblock totals to add
};

struct TileSt {  // prepared per-lane state of one tile; offsets are bytes from T0 / in_tile
    uint32_t rs, rec_out, ps, pe;  // this lane's record and its part [ps, pe) of it
    uint32_t pe_rec;               // end of the record's composed bytes (clipped to the capacity)
    uint64_t in0;                  // packed: the record's first string byte
    uint32_t L[5];
    uint64_t ts;                   // timestamp (default applied) / Lite sequence
    uint32_t tid;                  // Lite topicId
    uint64_t T0;                   // tile output start (uniform)
    uint32_t len;                  // tile output bytes, clipped to the capacity (uniform)
    uint32_t agg_in;               // packed: staged-input limit, bytes from in_tile (uniform)
    uintptr_t in_tile;             // packed: absolute address of the tile's first input byte (uniform)
    uintptr_t gsrc[5];             // gather mode (and kLenPub packed): absolute string addresses
    bool wrapped;                  // kLenPub packed: some record's input strings are longer than its
                                   // output ones (a length >= 65536): compose from gsrc (uniform)
    uint32_t agg_out;              // output bytes of the tile's records (uniform)
    uint64_t tot_in;               // packed: input bytes of the tile's records, 64-bit (uniform)
};

// sb_next: the first superblock whose total this workgroup has not loaded yet (tiles come in
// increasing order; a clamped repeat of the last tile loads nothing new)
template <class LY, bool kPacked>
__device__ __forceinline__ TileIn tile_load(const EncArgs& a, uint64_t tile, int lane, uint64_t& sb_next) {
    SBE_TILE_SHAPE(LY);
    TileIn x;
    // unconditional loads at a clamped index: a select on the loaded value here would make the
    // compiler wait for it (tile_prepare applies r < n)
    uint64_t r = tile * kRpt + lane / kLpr;
    r = r < a.n ? r : a.n - 1;
#pragma unroll
    for (int f = 0; f < 5; ++f) x.L[f] = f < LY::kNF ? a.str_len[LY::kNF * r + f] : 0u;
    x.ts = a.timestamp[r];
    x.tid = LY::kTM ? 0u : a.topic_id[r];
    x.to = a.tsum[2 * tile];  // uniform: scalar loads
    x.ti = kPacked ? a.tsum[2 * tile + 1] : 0ull;
    // totals of superblocks [sb_next, tile's superblock): lane l loads superblock sb_next + l at a
    // clamped index, unconditionally (tile_prepare masks lanes >= count); at most G/128 + 1 of
    // them, so one per lane while the persistent grid stays under 63 x 128 workgroups
    const uint64_t sbt = tile / kTilesPerSb;
    const uint64_t last_sb = (a.n - 1) / kSbRec;
    uint64_t s = sb_next + (uint64_t)lane;
    s = s < last_sb ? s : last_sb;
    x.po = a.bsum[2 * s];
    x.pi = kPacked ? a.bsum[2 * s + 1] : 0ull;
    x.pcount = sbt > sb_next ? (uint32_t)(sbt - sb_next) : 0u;
    sb_next = sbt > sb_next ? sbt : sb_next;
    return x;
}

// The tile of kRpt records from record r_first (records at or past rend are not part of it), its
// output starting at base_out and its packed input at arena + base_in.
template <class LY, bool kPacked, int kLen>
__device__ __forceinline__ TileSt tile_prepare_at(const EncArgs& a, const TileIn& x, uint64_t r_first, uint64_t rend,
                                                  int lane, uint64_t base_out, uint64_t base_in);

// sp_out / sp_in: running totals of the superblocks before this workgroup's current tile
template <class LY, bool kPacked, int kLen>
__device__ __forceinline__ TileSt tile_prepare(const EncArgs& a, const TileIn& x, uint64_t tile, int lane,
                                               uint64_t& sp_out, uint64_t& sp_in) {
    SBE_TILE_SHAPE(LY);
    sp_out += wave_sum64((uint32_t)lane < x.pcount ? x.po : 0ull);
    if (kPacked) sp_in += wave_sum64((uint32_t)lane < x.pcount ? x.pi : 0ull);
    const uint64_t base_out = uniform64(sp_out + x.to);
    const uint64_t base_in = kPacked ? uniform64(sp_in + x.ti) : 0ull;
    return tile_prepare_at<LY, kPacked, kLen>(a, x, tile * kRpt, a.n, lane, base_out, base_in);
}

template <class LY, bool kPacked, int kLen>
__device__ __forceinline__ TileSt tile_prepare_at(const EncArgs& a, const TileIn& x, uint64_t r_first, uint64_t rend,
                                                  int lane, uint64_t base_out, uint64_t base_in) {
    SBE_TILE_SHAPE(LY);
    TileSt S;
    const int q = lane % kLpr;
    const uint64_t r = r_first + lane / kLpr;
    const bool valid = r < rend;
    uint64_t sum = 0, sum_in = 0;
    uint8_t st = SBE_ENC_OK;
#pragma unroll
    for (int f = 0; f < 5; ++f) {
        const uint32_t Lx = valid ? x.L[f] : 0u;
        S.L[f] = kLen == kLenPub ? (Lx & 0xffffu) : Lx;
        sum += S.L[f];
        sum_in += Lx;
    }
    if (kLen != kLenPub) {
#pragma unroll
        for (int f = LY::kNF - 1; f >= 0; --f)  // first failing field in wire order (TopicMessage.h:1396-1428)
            if (S.L[f] > SBE_VAR_MAX_LEN) st = (uint8_t)(SBE_ENC_E109_TOPIC + f);
    }
    const uint32_t ovh = (uint32_t)LY::ovh(kLen == kLenRef);
    const uint32_t rec_out = (valid && st == SBE_ENC_OK) ? ovh + (uint32_t)sum : 0u;
    const uint64_t rec_in = (kPacked && valid) ? sum_in : 0ull;
    S.wrapped = kLen == kLenPub && kPacked && __ballot(sum_in != sum) != 0;
    const uint32_t lo_out = q == 0 ? rec_out : 0u;
    const uint32_t inc_out = wave_incl_scan(lo_out, lane);
    const uint32_t agg_out = lane_u32(inc_out, kWave - 1);
    // the record's lead lane's value (kLpr = 2: quad_perm [0,0,2,2])
    S.rs = kLpr == 2 ? dpp0<0xa0>(inc_out - lo_out) : inc_out - lo_out;
    S.rec_out = rec_out;
    S.agg_out = agg_out;
    S.tot_in = 0;
    if (kPacked) {
        // every record of the tile encodable: input offsets follow the output ones (34 B apart
        // per record); otherwise (E109 / past the end) a 64-bit scan of the input sizes
        if (__ballot(!(valid && st == SBE_ENC_OK)) == 0 && !S.wrapped) {
            const uint32_t ovh0 = ovh;
            S.in0 = S.rs - ovh0 * (uint32_t)(lane / kLpr);
            const uint64_t agg_in = agg_out - (uint64_t)ovh0 * kRpt;
            S.agg_in = (uint32_t)agg_in;
            S.tot_in = agg_in;
        } else {
            const uint64_t lo_in = q == 0 ? rec_in : 0ull;
            const uint64_t inc_in = wave_incl_scan64(lo_in, lane);
            const uint64_t agg_in = lane_u64(inc_in, kWave - 1);
            S.agg_in = agg_in < 0x7fffffffull ? (uint32_t)agg_in : 0x7fffffffu;
            S.tot_in = agg_in;
            const uint64_t ex = inc_in - lo_in;
            S.in0 = kLpr == 2 ? ((uint64_t)dpp0<0xa0>((uint32_t)(ex >> 32)) << 32) | dpp0<0xa0>((uint32_t)ex) : ex;
        }
    } else {
        S.agg_in = 0;
        S.in0 = 0;
    }
    S.ts = LY::kTM ? ((valid && x.ts) ? x.ts : a.ts_default) : x.ts;
    S.tid = x.tid;
    const uint32_t re = S.rs + rec_out;
    const uint64_t cap_rel64 = a.cap > base_out ? a.cap - base_out : 0ull;
    const uint32_t cap_rel = cap_rel64 < (uint64_t)agg_out ? (uint32_t)cap_rel64 : agg_out;
    if (valid && q == 0) {
        if (st == SBE_ENC_OK && (uint64_t)re > cap_rel64) st = SBE_ENC_OVERFLOW;
        a.out_off[r] = base_out + S.rs;
        if (r == a.n - 1) a.out_off[a.n] = base_out + re;
        if (a.status) a.status[r] = st;
    }
    const uint32_t ps = q == 0 ? S.rs : ((S.rs + (uint32_t)q * rec_out / kLpr + 3) & ~3u);
    const uint32_t pe = q == kLpr - 1 ? re : ((S.rs + (uint32_t)(q + 1) * rec_out / kLpr + 3) & ~3u);
    const uint32_t hi_rec = re < cap_rel ? re : cap_rel;
    S.ps = ps < re ? ps : re;
    S.pe = pe < hi_rec ? pe : hi_rec;
    S.pe_rec = hi_rec;
    S.T0 = base_out;
    S.len = cap_rel;
    S.in_tile = reinterpret_cast<uintptr_t>(a.arena) + base_in;
    if (kPacked && kLen == kLenPub) {  // string f of the record at its full-length input offset
        uintptr_t g = S.in_tile + S.in0;
#pragma unroll
        for (int f = 0; f < 5; ++f) {
            S.gsrc[f] = g;
            g += (valid && f < LY::kNF) ? x.L[f] : 0u;
        }
    }
    if (!kPacked) {
#pragma unroll
        for (int f = 0; f < 5; ++f)
            S.gsrc[f] = reinterpret_cast<uintptr_t>(a.arena) +
                        ((valid && f < LY::kNF) ? a.str_off[LY::kNF * r + f] : 0u);
    }
    return S;
}


// Staged input range for the output window starting wrel bytes from T0: from the first string
// byte at/after max(wrel, 0) (input offset >= p - kOvh within the record holding it) for kEWIn
// bytes, clipped to the tile's input.
template <class LY>
__device__ __forceinline__ void stage_range(const TileSt& S, int32_t wrel, int lane, uintptr_t& swb,
                                            int32_t& nbytes) {
    SBE_TILE_SHAPE(LY);
    const uint32_t g = wrel > 0 ? (uint32_t)wrel : 0u;
    const int q = lane % kLpr;
    const uint64_t mine = __ballot(q == 0 && S.rec_out && S.rs <= g && g < S.rs + S.rec_out);
    const int ra = mine ? __builtin_ctzll(mine) : 0;
    const uint32_t ra_rs = lane_u32(S.rs, ra);
    const uint64_t ra_in = lane_u64(S.in0, ra);
    const uint32_t p = g - ra_rs;
    const uintptr_t first = S.in_tile + ra_in + (p > (uint32_t)LY::kOvh ? p - (uint32_t)LY::kOvh : 0);
    swb = first & ~(uintptr_t)15;
    const uintptr_t lim = (S.in_tile + S.agg_in + 15) & ~(uintptr_t)15;
    const uintptr_t swe = swb + kEWIn < lim ? swb + kEWIn : (lim > swb ? lim : swb);
    nbytes = (int32_t)(swe - swb);
}

// Always kStageRegs loads (all lanes, offsets clamped into [swb, swb + nbytes); swb must be
// readable for 16 bytes when nbytes == 0): the loop body's vector-memory operations are then
// straight-line, so the compiler's vmcnt waits count them exactly instead of draining all.
// kNt: nontemporal loads (Lay::kNtIn: the input is read once and not from this kernel's caches again)
template <bool kNt>
__device__ __forceinline__ void stage_issue(uintptr_t swb, int32_t nbytes, int lane, uint4 (&I)[kStageRegs]) {
    g_u32x4* const base = reinterpret_cast<g_u32x4*>(swb);  // uniform base + 32-bit lane offsets
    const uint32_t last = nbytes >= 16 ? (uint32_t)(nbytes - 16) >> 4 : 0u;
#pragma unroll
    for (int k = 0; k < kStageRegs; ++k) {
        const uint32_t ch = lane + kWave * k;
        u32x4 v;
        if constexpr (kNt) v = __builtin_nontemporal_load(base + (ch < last ? ch : last));
        else v = base[ch < last ? ch : last];
        I[k] = make_uint4(v.x, v.y, v.z, v.w);
    }
}

// The staged chunks into LDS, unconditionally like stage_issue (lanes past the end rewrite the
// last chunk with its own bytes), so every path consumes the staging registers.
__device__ __forceinline__ void stage_write(lds_u8* inb, int32_t nbytes, int lane, const uint4 (&I)[kStageRegs]) {
    const uint32_t last = nbytes >= 16 ? (uint32_t)(nbytes - 16) >> 4 : 0u;
#pragma unroll
    for (int k = 0; k < kStageRegs; ++k) {
        const uint32_t ch = lane + kWave * k;
        lds_store16(inb + 16 * (ch < last ? ch : last), I[k]);
    }
}

// Dword j (compile-time after unrolling) of a record's literal prefix:
//  session header {24, 1, 111, 8}, leadershipTermId, clusterSessionId, timestamp 0
//    (src/session_manager.cpp:936-967, :1018-1046);
//  SBE header {blockLength, templateId, schemaId 1, version 1} (TopicMessage.h:221-238);
//  block: TopicMessage timestamp, sequenceNumber 0 (:362-437) / Lite u32 topicId, u64 sequence
//    (CommitOffsetLite.h:337-420).
template <class LY>
__device__ __forceinline__ uint32_t lit_word(const EncArgs& a, const TileSt& S, int j) {
    if (j < LY::kPre / 4) {
        switch (j) {
            case 0: return SBE_SESSION_BLOCK_LEN | (SBE_SESSION_TEMPLATE_ID << 16);
            case 1: return SBE_CLUSTER_SCHEMA_ID | (SBE_CLUSTER_SCHEMA_VERSION << 16);
            case 2: return (uint32_t)(uint64_t)a.term_id;
            case 3: return (uint32_t)((uint64_t)a.term_id >> 32);
            case 4: return (uint32_t)(uint64_t)a.sess_id;
            case 5: return (uint32_t)((uint64_t)a.sess_id >> 32);
            default: return 0u;
        }
    }
    j -= LY::kPre / 4;
    if (j == 0) return (uint32_t)LY::kBlk | ((LY::kTM ? SBE_TM_TEMPLATE_ID : a.tmpl) << 16);
    if (j == 1) return SBE_TOPIC_SCHEMA_ID | (1u << 16);
    if (LY::kTM) return j == 2 ? (uint32_t)S.ts : (j == 3 ? (uint32_t)(S.ts >> 32) : 0u);
    return j == 2 ? S.tid : (j == 3 ? (uint32_t)S.ts : (uint32_t)(S.ts >> 32));
}

// compose this lane's part [ps, pe) of its record, clipped to output window [wb, we); record
// layout TopicMessage.h:221-238 (header), :362-437 (timestamp, sequenceNumber 0), :515-1231
// (u16 length + bytes per string)
template <class LY, bool kPacked>
__device__ __forceinline__ void compose(const EncArgs& a, lds_u8* wout, lds_cu8* inb, const TileSt& S, int32_t wrel,
                                        int32_t we_rel, uintptr_t swb, int32_t win_bytes) {
    if (!(S.rec_out && S.ps < S.pe && (int32_t)S.ps < we_rel && (int32_t)S.pe > wrel)) return;
    const int32_t R0 = (int32_t)S.rs - wrel;
    const int32_t pl = (int32_t)S.ps - wrel;
    const int32_t lo = pl > 0 ? pl : 0;
    const int32_t hi = ((int32_t)S.pe < we_rel ? (int32_t)S.pe : we_rel) - wrel;
    Writer W{wout, lo, lo, 0u};
    int32_t x = lo - R0;  // record-relative position of W.pos
    const int32_t end = hi - R0;
#pragma unroll
    for (int j = 0; j < LY::kLit / 4; ++j) {
        if (x < 4 * j + 4 && x < end) {
            const int32_t e = end < 4 * j + 4 ? end : 4 * j + 4;
            W.lit(low_bytes64((uint64_t)lit_word<LY>(a, S, j) >> (8 * (x - 4 * j)), e - x), e - x);
            x = e;
        }
    }
    int32_t o = LY::kLit;
    const int64_t src0 = kPacked ? (int64_t)(S.in_tile + S.in0) - (int64_t)swb : 0;
    int64_t src = src0;
#pragma nounroll
    for (int f = 0; f < LY::kNF; ++f) {
        if (x >= end) break;
        const uint32_t Lu = f == 0 ? S.L[0] : f == 1 ? S.L[1] : f == 2 ? S.L[2] : f == 3 ? S.L[3] : S.L[4];
        const int32_t Lf = (int32_t)Lu;
        if (x < o + 2) {
            const int32_t e = end < o + 2 ? end : o + 2;
            W.lit((uint64_t)((Lu & 0xffffu) >> (8 * (x - o))) & ((1u << (8 * (e - x))) - 1u), e - x);
            x = e;
            if (x >= end) break;
        }
        const int32_t so = o + 2;
        if (x < so + Lf) {
            const int32_t e = end < so + Lf ? end : so + Lf;
            const int32_t m = e - x, off = x - so;
            if (kPacked && src + off >= 0 && src + off + m <= (int64_t)win_bytes) {
                W.str(LdsLin{inb}, (int32_t)(src + off), m);
            } else {
                uintptr_t sa;
                if (kPacked) {
                    sa = swb + (uintptr_t)(src + off);
                } else {
                    sa = (f == 0 ? S.gsrc[0] : f == 1 ? S.gsrc[1] : f == 2 ? S.gsrc[2] : f == 3 ? S.gsrc[3] : S.gsrc[4]) +
                         (uintptr_t)off;
                }
                W = str_global(W, sa, m);
            }
            x = e;
        }
        o = so + Lf;
        src += Lf;
    }
    W.flush();
}

// window chunks → HBM: 16-byte stores; the (at most two) chunks holding lo / we partially go
// through store_edges.
// Rows of 64 chunks [0, kRows0) are stored unconditionally; the rows after them only when the
// window reaches them (a uniform branch).  kRows0 = all rows for layouts whose windows are usually
// full; layouts of small records whose 32-record tiles are a few KiB (CommitOffsetLite) skip the
// empty rows: the join after the branch makes the compiler wait for the longer path's extra stores
// before the next window's staging, but the short path, the one those tiles take, waits exactly.
template <int kRows0>
__device__ __forceinline__ void store_rows(uint8_t* out, lds_cu8* wout, uint64_t wb, uint64_t lo, uint64_t we,
                                           uint32_t nch, uint32_t c_lo, uint32_t c_hi,
                                           const __amdgpu_buffer_rsrc_t& rs, int lane, int k0) {
    uint4 v[kRows0];
#pragma unroll
    for (int k = 0; k < kRows0; ++k) {
        const uint32_t ch = lane + kWave * (k0 + k);
        const u32x4 a0 = *reinterpret_cast<const __attribute__((address_space(3))) u32x4*>(wout + 16 * ch + (ch >> 4) * kRowPad);
        v[k] = make_uint4(a0.x, a0.y, a0.z, a0.w);
    }
    // unconditional 16-byte buffer stores; chunks not wholly inside [lo, we) take an offset past
    // the descriptor's range, which the hardware drops (cache policy kOutAux)
#pragma unroll
    for (int k = 0; k < kRows0; ++k) {
        const uint32_t ch = lane + kWave * (k0 + k);
        const bool full = ch >= c_lo && ch < c_hi;
        u32x4 x;
        x.x = v[k].x; x.y = v[k].y; x.z = v[k].z; x.w = v[k].w;
        __builtin_amdgcn_raw_buffer_store_b128(x, rs, full ? (int)(16u * ch) : 0x7ffffff0, 0, kOutAux);
    }
}

typedef __attribute__((address_space(1))) uint8_t g_w8;
typedef __attribute__((address_space(1))) uint16_t g_w16;
typedef __attribute__((address_space(1))) uint32_t g_w32;

// The window's partial chunks: lane 0 the one holding lo (bytes before lo belong to the previous
// window or tile), lane 1 the one holding we.  Bytes [s, e) of a 16-B aligned chunk as at most
// eight stores (byte, short, four dwords, short, byte), one instruction stream for both lanes.
__device__ __forceinline__ void store_edges(uint8_t* out, lds_cu8* wout, uint64_t wb, uint64_t lo, uint64_t we,
                                            uint32_t c_lo, uint32_t c_hi, int lane) {
    const int32_t nb = (int32_t)(we - wb), lb = (int32_t)(lo - wb);
    // head chunk c_lo - 1 (when lo is not chunk aligned), tail chunk c_hi (when we is not, and it
    // is not the head chunk too: the head then ends at we)
    const bool head = lane == 0 && c_lo > 0 && lb < nb;
    const bool tail = lane == 1 && (nb & 15) != 0 && c_hi >= c_lo;
    if (!(head || tail)) return;
    const int32_t c = head ? (int32_t)c_lo - 1 : (int32_t)c_hi;
    const int32_t s0 = head ? lb - 16 * c : 0;
    const int32_t e = min(16, nb - 16 * c);
    const u32x4 v = *reinterpret_cast<const __attribute__((address_space(3))) u32x4*>(wout + 16 * c + (c >> 4) * kRowPad);
    auto byte_at = [&](int32_t p) { return (uint8_t)(v[p >> 2] >> (8 * (p & 3))); };
    auto half_at = [&](int32_t p) { return (uint16_t)(v[p >> 2] >> (8 * (p & 3))); };  // p even: same dword
    g_w8* const g = reinterpret_cast<g_w8*>(reinterpret_cast<uintptr_t>(out) + wb + 16 * (uint32_t)c);
    int32_t p = s0;
    if ((p & 1) && p < e) {
        g[p] = byte_at(p);
        ++p;
    }
    if ((p & 2) && p + 2 <= e) {
        *reinterpret_cast<g_w16*>(g + p) = half_at(p);
        p += 2;
    }
#pragma unroll
    for (int j = 0; j < 4; ++j)
        if (4 * j >= p && 4 * j + 4 <= e) reinterpret_cast<g_w32*>(g)[j] = v[j];
    int32_t p2 = max(p, e & ~3);
    if (p2 + 2 <= e) {
        *reinterpret_cast<g_w16*>(g + p2) = half_at(p2);
        p2 += 2;
    }
    if (p2 < e) g[p2] = byte_at(p2);
}

constexpr int kStoreRows = kEW / 16 / kWave;  // rows of 64 chunks in a window
template <int kRows0 = kStoreRows>
__device__ __forceinline__ void store_window(uint8_t* out, lds_cu8* wout, uint64_t T0, uint64_t wb, uint64_t we,
                                             int lane) {
    static_assert(kRows0 >= 1 && kRows0 <= kStoreRows, "store rows");
    const uint64_t lo = wb > T0 ? wb : T0;
    const uint32_t nch = (uint32_t)((we - wb + 15) >> 4);
    const uint32_t c_lo = (uint32_t)((lo - wb + 15) >> 4);  // chunks [c_lo, c_hi) lie inside [lo, we)
    const uint32_t c_hi = (uint32_t)((we - wb) >> 4);
    const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(out + wb, 0, (int)(16u * c_hi), 0x00020000);
    store_rows<kRows0>(out, wout, wb, lo, we, nch, c_lo, c_hi, rs, lane, 0);
    if constexpr (kRows0 < kStoreRows) {
        if (nch > (uint32_t)(kWave * kRows0))
            store_rows<kStoreRows - kRows0>(out, wout, wb, lo, we, nch, c_lo, c_hi, rs, lane, kRows0);
    }
    store_edges(out, wout, wb, lo, we, c_lo, c_hi, lane);
}

// ---- packed mode: chunk / fixup / literal passes ---------------------------------------------
// Lane l owns the kCpl 16-byte chunks [l*kCpl, (l+1)*kCpl) of the window (128 contiguous bytes).
// A chunk's string bytes all belong to the record holding its first byte (string bytes start 26 B
// into a record, past any 16-byte chunk that begins before it), and within a record string f sits
// at output = staged input + sh0 + 2f.  So one pass computes every chunk from the "zone" (string
// index) of its first byte with five LDS dword reads and four v_alignbyte; a second pass rewrites
// the bytes after a string start that falls inside a chunk (<= 15 per string), and a third
// writes the header and the u16 lengths.  Non-string bytes are don't-care until the third pass.
constexpr int32_t kChunks = kEW / 16;
constexpr int32_t kCpl = kChunks / kWave;        // chunks per lane
constexpr int32_t kLaneBytes = 16 * kCpl;
static_assert(kChunks % kWave == 0 && 256 % kLaneBytes == 0, "window shape");
constexpr int32_t kRecEnt = 8;                   // dwords per record-table entry

typedef __attribute__((address_space(3))) int32_t lds_i32;
typedef int i32x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) i32x4 lds_i32x4;

struct RecEnt {     // window-relative (bytes from the window start)
    int32_t rw;     // record start
    int32_t rend;   // end of its composed bytes (record end clipped to the capacity)
    int32_t sh0;    // string 0: output position - staged-input position (staged records)
    int32_t z1, z2, z3, z4;  // record-relative starts of strings 1..4
    int32_t z5;              // end of string 4 (| kNotStaged); scalars, so selects never become a
                             // dynamically indexed (scratch) array
};
constexpr int32_t kNotStaged = 0x40000000;  // z[4] flag: strings not all in the staged window

// z_{j+1} for a compile-time j (unrolled loops)
__device__ __forceinline__ int32_t zat(const RecEnt& E, int j) {
    switch (j) {
        case 0: return E.z1;
        case 1: return E.z2;
        case 2: return E.z3;
        case 3: return E.z4;
        default: return E.z5;
    }
}

__device__ __forceinline__ RecEnt rec_load(lds_i32* rt, int32_t r) {
    const i32x4 a = reinterpret_cast<lds_i32x4*>(rt + kRecEnt * r)[0];
    const i32x4 b = reinterpret_cast<lds_i32x4*>(rt + kRecEnt * r)[1];
    RecEnt E;
    E.rw = a.x; E.rend = a.y; E.sh0 = a.z; E.z1 = a.w;
    E.z2 = b.x; E.z3 = b.y; E.z4 = b.z; E.z5 = b.w;
    return E;
}

// The five dwords i .. i+4 of the staged input (a 16-byte chunk at any byte alignment inside them).
// SBE_CHUNK_B64: as three ds_read_b64 at the 8-byte aligned dword i & ~1 and one select per dword
// (banks (a/4) mod 64 for ds_read_b64, against (a/4) mod 32 for ds_read_b32: lanes whose chunks lie
// 128 B apart, the two lanes of a 256-B record, or a rebalanced window's runs of 16 T bytes, stop
// sharing banks); else five ds_read_b32.  i <= imax - 1 (the b64 form reads one dword further).
#ifndef SBE_CHUNK_B64
#define SBE_CHUNK_B64 0
#endif
__device__ __forceinline__ void lds_dw5(lds_cu8* inb, int32_t i, uint32_t (&d)[5]) {
    if (SBE_CHUNK_B64) {
        const lds_cu32x2* q = reinterpret_cast<lds_cu32x2*>(reinterpret_cast<lds_cu32*>(inb) + (i & ~1));
        const u32x2 a = q[0], b = q[1], c = q[2];
        const bool odd = (i & 1) != 0;
        d[0] = odd ? a.y : a.x;
        d[1] = odd ? b.x : a.y;
        d[2] = odd ? b.y : b.x;
        d[3] = odd ? c.x : b.y;
        d[4] = odd ? c.y : c.x;
    } else {
        lds_cu32* q = reinterpret_cast<lds_cu32*>(inb) + i;
#pragma unroll
        for (int j = 0; j < 5; ++j) d[j] = q[j];
    }
}

// SBE_CHUNK_UA (A/B builds): a chunk at any staged byte position as ONE unaligned ds_read_b128
// (the LDS replays the misaligned access) instead of five dword reads and four v_alignbyte.
// Fewer instructions, but the replays cost more: fixed-256 pack 94.7 -> 99.0 us, config 4 706.3
// -> 709.3, session 125.6 -> 128.6, OrderRequestLite 144.6 -> 150.2 (profiles/r06_ab_ua.log).
#ifndef SBE_CHUNK_UA
#define SBE_CHUNK_UA 0
#endif
typedef uint32_t u32x4_ua1 __attribute__((ext_vector_type(4), aligned(1)));
typedef __attribute__((address_space(3))) const u32x4_ua1 lds_cu32x4_ua;
// the 16 bytes at staged byte u, u clamped to [-kInSlack, 4 * imax] (a clamped read only ever feeds
// don't-care bytes; 4 * imax + 16 <= the dword form's last byte read)
__device__ __forceinline__ u32x4 lds_chunk_ua(lds_cu8* inb, int32_t u, int32_t imax) {
    const int32_t lo = -kInSlack, hi = 4 * imax;
    u = u < lo ? lo : (u > hi ? hi : u);
    const u32x4_ua1 x = *reinterpret_cast<lds_cu32x4_ua*>(inb + u);
    u32x4 v;
    v.x = x.x; v.y = x.y; v.z = x.z; v.w = x.w;
    return v;
}
// the 16 bytes at staged-input position u (any alignment); the base is clamped into the array
// (a clamped read only ever feeds don't-care bytes)
__device__ __forceinline__ u32x4 chunk_lds(lds_cu8* inb, int32_t u, int32_t imax) {
    if (SBE_CHUNK_UA) return lds_chunk_ua(inb, u, imax);
    int32_t i = u >> 2;
    i = i < -kInSlack / 4 ? -kInSlack / 4 : (i > imax ? imax : i);
    const uint32_t sh = (uint32_t)u & 3u;
    lds_cu32* q = reinterpret_cast<lds_cu32*>(inb) + i;
    const uint32_t d0 = q[0], d1 = q[1], d2 = q[2], d3 = q[3], d4 = q[4];
    u32x4 v;
    v.x = __builtin_amdgcn_alignbyte(d1, d0, sh);
    v.y = __builtin_amdgcn_alignbyte(d2, d1, sh);
    v.z = __builtin_amdgcn_alignbyte(d3, d2, sh);
    v.w = __builtin_amdgcn_alignbyte(d4, d3, sh);
    return v;
}
// the 16 bytes at absolute address a, dword reads clamped to [lo4, hi4] (the record's strings)
__device__ __forceinline__ u32x4 chunk_glb(uint64_t a, uint64_t lo4, uint64_t hi4) {
    const uint32_t sh = (uint32_t)(a & 3);
    uint32_t d[5];
#pragma unroll
    for (int k = 0; k < 5; ++k) {
        uint64_t q = (a & ~3ull) + 4ull * k;
        q = q < lo4 ? lo4 : (q > hi4 ? hi4 : q);
        d[k] = gload32((uintptr_t)q);
    }
    u32x4 v;
    v.x = __builtin_amdgcn_alignbyte(d[1], d[0], sh);
    v.y = __builtin_amdgcn_alignbyte(d[2], d[1], sh);
    v.z = __builtin_amdgcn_alignbyte(d[3], d[2], sh);
    v.w = __builtin_amdgcn_alignbyte(d[4], d[3], sh);
    return v;
}

// bytes [lo, hi) of the dword at window position d (4-aligned)
__device__ __forceinline__ void put_clip(lds_u8* wout, int32_t d, uint32_t v, int32_t lo, int32_t hi) {
    if (d >= lo && d + 4 <= hi) {
        *reinterpret_cast<lds_u32*>(wout + wout_addr(d)) = v;
    } else if (d + 4 > lo && d < hi) {
        lds_u8* q = wout + wout_addr(d);
#pragma unroll
        for (int k = 0; k < 4; ++k)
            if (d + k >= lo && d + k < hi) q[k] = (uint8_t)(v >> (8 * k));
    }
}

// Record table, bucket table and per-record absolute string bases for one window; returns true
// (wave-uniform) when some record of the window has strings outside the staged input.
template <class LY>
__device__ __forceinline__ bool build_tables(lds_i32* rt, lds_i32* bk, uint64_t* sbase, const TileSt& S,
                                             int32_t wrel, int32_t wlen, uintptr_t swb, int32_t nb, int ra, int rb,
                                             int lg, int lane) {
    SBE_TILE_SHAPE(LY);
    const int q = lane % kLpr, r = lane / kLpr;
    bk[lane] = ra;
    bool outside = false;
    if (q == 0) {
        // records outside [ra, rb) compose nothing in this window
        const bool live = S.rec_out && r >= ra && r < rb;
        const int32_t rw = (int32_t)S.rs - wrel;
        const int32_t rend = (live ? (int32_t)S.pe_rec : (int32_t)S.rs) - wrel;
        const uint64_t s0 = S.in_tile + S.in0;                 // absolute address of string 0
        const int64_t src0 = (int64_t)s0 - (int64_t)swb;       // its staged position
        uint32_t nstr = 0;
#pragma unroll
        for (int f = 0; f < 5; ++f) nstr += S.L[f];
        const bool staged = src0 >= 0 && src0 + (int64_t)nstr <= (int64_t)nb;
        outside = live && !staged && rend > (rw > 0 ? rw : 0) && (rw < wlen);
        i32x4 a, b;
        a.x = rw;
        a.y = rend;
        a.z = staged ? rw + LY::kS0 - (int32_t)src0 : 0;
        // string starts z_1..z_4 (record-relative); fields the layout lacks start at the end
        int32_t zs[5];
        int32_t z = LY::kS0;
#pragma unroll
        for (int f = 1; f < 5; ++f) {
            if (f < LY::kNF) z += (int32_t)S.L[f - 1] + 2;
            zs[f - 1] = z;
        }
        zs[4] = z + (int32_t)S.L[LY::kNF - 1];
#pragma unroll
        for (int f = LY::kNF; f < 5; ++f) zs[f - 1] = zs[4];
        a.w = zs[0];
        b.x = zs[1];
        b.y = zs[2];
        b.z = zs[3];
        b.w = zs[4] | (staged ? 0 : kNotStaged);
        reinterpret_cast<lds_i32x4*>(rt + kRecEnt * r)[0] = a;
        reinterpret_cast<lds_i32x4*>(rt + kRecEnt * r)[1] = b;
        sbase[r] = s0;
        // buckets bb (lane bb's range, 2^lg bytes) starting inside [rw, rend) ∩ [0, wlen)
        const int32_t s1 = rw > 0 ? rw : 0;
        const int32_t e1 = rend < wlen ? rend : wlen;
        if (live && s1 < e1) {
            for (int32_t bb = (s1 + (1 << lg) - 1) >> lg; (bb << lg) < e1; ++bb) bk[bb] = r;
        }
    }
    return __ballot(outside) != 0;
}

__device__ __forceinline__ int32_t zone_of(const RecEnt& E, int32_t X) {
    return (X >= E.z1) + (X >= E.z2) + (X >= E.z3) + (X >= E.z4);
}

// Zone boundaries inside a chunk: for the chunk at record-relative X (its first byte in string
// zone f0 = zone_of(X)), the starts z_f of strings f > f0 that fall on bytes 1..15 of the chunk
// (before the record's composed end), as 4-bit byte offsets: nibble f-1 = z_f - X, 0 = none.  The
// bytes from z_f on come from zone f (2 bytes further along the input per zone).
__device__ __forceinline__ uint32_t zone_marks(const RecEnt& E, int32_t X) {
    const int32_t last = min(X + 15, E.rend - E.rw - 1);
    uint32_t m = 0;
    m |= (E.z1 > X && E.z1 <= last) ? (uint32_t)(E.z1 - X) : 0u;
    m |= (E.z2 > X && E.z2 <= last) ? (uint32_t)(E.z2 - X) << 4 : 0u;
    m |= (E.z3 > X && E.z3 <= last) ? (uint32_t)(E.z3 - X) << 8 : 0u;
    m |= (E.z4 > X && E.z4 <= last) ? (uint32_t)(E.z4 - X) << 12 : 0u;
    return m;
}

// bytes b0..15 of v replaced by w's (b0 in 1..16; 16: none): byte masks from two 64-bit shifts,
// one v_bfi per dword
__device__ __forceinline__ u32x4 merge_tail(u32x4 v, u32x4 w, int32_t b0) {
    const uint32_t s = 8u * (uint32_t)b0;
    const uint64_t m01 = s >= 64 ? 0ull : ~0ull << s;
    const uint64_t m23 = s >= 128 ? 0ull : (s <= 64 ? ~0ull : ~0ull << (s - 64));
    const uint32_t m[4] = {(uint32_t)m01, (uint32_t)(m01 >> 32), (uint32_t)m23, (uint32_t)(m23 >> 32)};
    u32x4 r;
#pragma unroll
    for (int j = 0; j < 4; ++j) r[j] = (v[j] & ~m[j]) | (w[j] & m[j]);
    return r;
}

__device__ __forceinline__ u32x4 align4(uint32_t e0, uint32_t e1, uint32_t e2, uint32_t e3, uint32_t e4, uint32_t s) {
    u32x4 v;
    v.x = __builtin_amdgcn_alignbyte(e1, e0, s);
    v.y = __builtin_amdgcn_alignbyte(e2, e1, s);
    v.z = __builtin_amdgcn_alignbyte(e3, e2, s);
    v.w = __builtin_amdgcn_alignbyte(e4, e3, s);
    return v;
}

// Every chunk of the lane from the staged input, string bytes exact (chunks of not-staged records
// get don't-care data, redone by chunk_pass_global; literal bytes are don't-care until the literal
// pass).  Phases, so the LDS latency is paid a few times per window, not per chunk: source offsets
// (walking the record table, next entry prefetched), all source reads, v_alignbyte, then the rare
// chunks with a string start inside (zone_marks) merge their tail from the next zone, then one
// ds_write_b128 per chunk.
// Lane l owns the kk chunks [l kk, (l+1) kk) of the window: kk = 8 for a full window, fewer for
// a window that carries less (kk a power of two, so a lane never straddles a padded 256-B row).
template <class LY>
__device__ __forceinline__ void chunk_pass(lds_u8* wout, lds_cu8* inb, lds_i32* rt, lds_i32* bk, int32_t wlen,
                                           int32_t nb, int kk, int lg, int lane) {
    SBE_TILE_SHAPE(LY);
    const int32_t imax = (nb + kInSlack) / 4 - 5;
    int32_t r = bk[lane];
    RecEnt E = rec_load(rt, r);
    RecEnt N = rec_load(rt, r + 1 < kRpt ? r + 1 : r);
    int32_t u[kCpl];
    const int32_t lb = lane << lg;  // the lane's first byte
#pragma unroll
    for (int k = 0; k < kCpl; ++k) {
        if (k >= kk) break;
        const int32_t p = lb + 16 * k;
        if (p >= E.rend && r + 1 < kRpt) {
            do {  // records shorter than a chunk step: rare second iteration
                ++r;
                E = N;
                N = rec_load(rt, r + 1 < kRpt ? r + 1 : r);
            } while (p >= E.rend && r + 1 < kRpt);
        }
        u[k] = p - E.sh0 - 2 * zone_of(E, p - E.rw);
    }
#if SBE_CHUNK_UA
    u32x4 w[kCpl];
#else
    uint32_t d[kCpl][5];
#endif
#pragma unroll
    for (int k = 0; k < kCpl; ++k) {
        if (k >= kk) break;
#if SBE_CHUNK_UA
        w[k] = lds_chunk_ua(inb, u[k], imax - 1);
#else
        int32_t i = u[k] >> 2;
        i = i < -kInSlack / 4 ? -kInSlack / 4 : (i > imax - 1 ? imax - 1 : i);
        lds_dw5(inb, i, d[k]);
#endif
    }
    lds_u8* const wl = wout + lb + (lb >> 8) * kRowPad;  // padded rows never split a lane
#pragma unroll
    for (int k = 0; k < kCpl; ++k) {
        if (k >= kk) break;
#if SBE_CHUNK_UA
        const u32x4 v = w[k];
#else
        const u32x4 v = align4(d[k][0], d[k][1], d[k][2], d[k][3], d[k][4], (uint32_t)u[k] & 3u);
#endif
        if (lb + 16 * k < wlen) *reinterpret_cast<lds_u32x4*>(wl + 16 * k) = v;
    }
}

// Zone fix-up: the bulk passes compose every chunk from the zone (string) of its first byte; a
// chunk with a string start on bytes 1..15 gets its tail from the later zone(s) here.  Work items
// are the (record, string start) pairs of the record table, kNF - 1 per record (z1..z4 for a
// TopicMessage: two item passes per window; one for the Lite layouts); the item of a chunk's first interior string start recomputes the whole chunk (its
// zone, then every later string start inside it merged over the tail) and rewrites it, the others
// do nothing.  So the merges cost
// two item passes per window instead of a merge step at every chunk position of every lane.
// Records of the table outside the window, empty ones (rend <= rw) and not-staged ones
// (chunk_pass_global composes those whole) have no items.
template <class LY>
__device__ __forceinline__ void zone_fixup(lds_u8* wout, lds_cu8* inb, lds_i32* rt, int32_t wlen, int32_t nb,
                                           int lane, int ra, int rb) {
    SBE_TILE_SHAPE(LY);
    const int32_t imax = (nb + kInSlack) / 4 - 5;
    constexpr int kZ = LY::kNF - 1;  // interior string starts per record (z_1 .. z_{kNF-1})
    static_assert(kZ >= 1 && kZ <= 4, "layouts have 2..5 strings");
    // 64-record tiles: the window's records [ra, rb) only (a window holds part of a tile: fewer
    // item passes); 32-record tiles: all of them (measured no slower than the restriction)
    const int r0 = kRpt == 64 ? ra : 0, r1 = kRpt == 64 ? rb : kRpt;
    const int nitems = kZ * (r1 - r0);
#pragma unroll
    for (int i0 = 0; i0 < kZ * kRpt; i0 += kWave) {
        if (i0 >= nitems) break;
        const int i = i0 + lane, j = r0 + i / kZ, f = i % kZ;  // string start z_{f+1} of record j
        if (j >= r1) continue;
        const RecEnt E = rec_load(rt, j);
        const int32_t zf = f == 0 ? E.z1 : f == 1 ? E.z2 : f == 2 ? E.z3 : E.z4;
        const int32_t zp = f == 0 ? 0 : f == 1 ? E.z1 : f == 2 ? E.z2 : E.z3;
        const int32_t P = E.rw + zf;  // window position of the string start
        const int32_t C = P >> 4;     // its chunk
        const bool own = (P & 15) != 0 && P < E.rend && P >= 0 && 16 * C < wlen && !(E.z5 & kNotStaged) &&
                         (f == 0 || E.rw + zp <= 16 * C);
        if (own) {
            // the chunk's first byte is in zone f (z_f <= its start < z_{f+1} = P): source u0; zone
            // f+1 from byte P - 16 C on reads 2 bytes further back, zone f+2 (a string start at
            // P2 in the same chunk: string f+1 shorter than 14 bytes) 4, later ones from the LDS
            const int32_t u0 = 16 * C - E.sh0 - 2 * f;
            int32_t q = u0 >> 2;
            q = q < 1 - kInSlack / 4 ? 1 - kInSlack / 4 : (q > imax ? imax : q);
            lds_cu32* src = reinterpret_cast<lds_cu32*>(inb) + q - 1;
            uint32_t d[6];
#pragma unroll
            for (int k = 0; k < 6; ++k) d[k] = src[k];
            const uint32_t sh = (uint32_t)u0 & 3u;
            u32x4 v = align4(d[1], d[2], d[3], d[4], d[5], sh);
            const bool hi = sh >= 2;  // u0 - 2 = 4 q + (sh - 2), or 4 (q - 1) + (sh + 2)
            v = merge_tail(v, align4(hi ? d[1] : d[0], hi ? d[2] : d[1], hi ? d[3] : d[2], hi ? d[4] : d[3],
                                     hi ? d[5] : d[4], hi ? sh - 2 : sh + 2), P - 16 * C);
            const int32_t cend = min(16 * C + 16, E.rend);
            const int32_t P2 = E.rw + (f == 0 ? E.z2 : f == 1 ? E.z3 : E.z4);
            const bool has2 = f < 3 && P2 < cend;
            if (__ballot(has2)) {
                v = merge_tail(v, align4(d[0], d[1], d[2], d[3], d[4], sh), has2 ? P2 - 16 * C : 16);
                const int32_t P3 = E.rw + (f == 0 ? E.z3 : E.z4);
                const bool has3 = f < 2 && P3 < cend;
                if (__ballot(has3)) {
                    v = merge_tail(v, chunk_lds(inb, u0 - 6, imax), has3 ? P3 - 16 * C : 16);
                    const bool has4 = f == 0 && E.rw + E.z4 < cend;
                    if (__ballot(has4)) v = merge_tail(v, chunk_lds(inb, u0 - 8, imax), has4 ? E.rw + E.z4 - 16 * C : 16);
                }
            }
            *reinterpret_cast<lds_u32x4*>(wout + wout_addr(16 * C)) = v;
        }
    }
}

// the chunks of records whose strings are not all staged, from HBM (rare: a record straddling a
// window of a multi-window tile, or valid records behind E109 records with large strings)
typedef __attribute__((address_space(3))) uint64_t lds_u64;
template <class LY>
__device__ __noinline__ void chunk_pass_global(lds_u8* wout, lds_i32* rt, lds_i32* bk, const lds_u64* sbase,
                                               int32_t wlen, int kk, int lg, int lane) {
    SBE_TILE_SHAPE(LY);
    int32_t r = bk[lane];
    RecEnt E = rec_load(rt, r);
    const int32_t lb = lane << lg;
    lds_u8* const wl = wout + lb + (lb >> 8) * kRowPad;
    for (int k = 0; k < kk; ++k) {
        const int32_t p = lb + 16 * k;
        if (p >= wlen) break;
        while (p >= E.rend && r + 1 < kRpt) {
            ++r;
            E = rec_load(rt, r);
        }
        if (!(E.z5 & kNotStaged)) continue;
        const int32_t X = p - E.rw;
        const uint64_t s0 = sbase[r];
        const uint32_t nstr = (uint32_t)((E.z5 & ~kNotStaged) - LY::kOvh);
        const uint64_t lo4 = s0 & ~3ull, hi4 = (s0 + (nstr ? nstr - 1 : 0)) & ~3ull;
        // string f's byte at record-relative x sits at s0 + x - kS0 - 2f
        const int64_t at0 = (int64_t)X - LY::kS0;
        u32x4 v = chunk_glb(s0 + (uint64_t)(at0 - 2 * zone_of(E, X)), lo4, hi4);
        for (uint32_t m = zone_marks(E, X); m; ) {
            const int32_t nib = __builtin_ctz(m) >> 2;
            const int32_t b0 = (int32_t)((m >> (4 * nib)) & 15u);
            m &= ~(15u << (4 * nib));
            v = merge_tail(v, chunk_glb(s0 + (uint64_t)(at0 - 2 * (nib + 1)), lo4, hi4), b0);
        }
        *reinterpret_cast<lds_u32x4*>(wl + 16 * k) = v;
    }
}

// The literal words of one record: lit_word's inputs, small enough to pass by value.
struct LitIn {
    uint64_t ts;   // timestamp (default applied) / Lite sequence
    int64_t term, sess;
    uint32_t tid, tmpl;
    uint32_t L[5];
};

// Dword j (compile-time after unrolling) of a record's literal prefix (see lit_word).
template <class LY>
__device__ __forceinline__ uint32_t lit_word_v(const LitIn& I, int j) {
    if (j < LY::kPre / 4) {
        switch (j) {
            case 0: return SBE_SESSION_BLOCK_LEN | (SBE_SESSION_TEMPLATE_ID << 16);
            case 1: return SBE_CLUSTER_SCHEMA_ID | (SBE_CLUSTER_SCHEMA_VERSION << 16);
            case 2: return (uint32_t)(uint64_t)I.term;
            case 3: return (uint32_t)((uint64_t)I.term >> 32);
            case 4: return (uint32_t)(uint64_t)I.sess;
            case 5: return (uint32_t)((uint64_t)I.sess >> 32);
            default: return 0u;
        }
    }
    j -= LY::kPre / 4;
    if (j == 0) return (uint32_t)LY::kBlk | ((LY::kTM ? SBE_TM_TEMPLATE_ID : I.tmpl) << 16);
    if (j == 1) return SBE_TOPIC_SCHEMA_ID | (1u << 16);
    if (LY::kTM) return j == 2 ? (uint32_t)I.ts : (j == 3 ? (uint32_t)(I.ts >> 32) : 0u);
    return j == 2 ? I.tid : (j == 3 ? (uint32_t)I.ts : (uint32_t)(I.ts >> 32));
}

// the literal prefix and the u16 lengths (TopicMessage.h:515-1231) of a record whose literal bytes
// may be clipped by the window or the capacity: dword writes with byte-wise edges (rare, out of line)
template <class LY>
__device__ __noinline__ void literal_clip(lds_u8* wout, RecEnt E, LitIn I, int32_t wlen, int q) {
    SBE_TILE_SHAPE(LY);
    const int32_t hi_all = E.rend < wlen ? E.rend : wlen;
    const int32_t lo_all = E.rw > 0 ? E.rw : 0;
    if (q == 0) {
        constexpr int kW = LY::kLit / 4;
        const int32_t a = E.rw & 3, d0 = E.rw - a;
        const int32_t hi = E.rw + LY::kLit < hi_all ? E.rw + LY::kLit : hi_all;
#pragma unroll
        for (int j = 0; j <= kW; ++j) {
            const uint32_t cur = j < kW ? lit_word_v<LY>(I, j) : 0u, prv = j > 0 ? lit_word_v<LY>(I, j - 1) : 0u;
            const uint32_t v = a ? __builtin_amdgcn_alignbyte(cur, prv, 4u - (uint32_t)a) : cur;
            put_clip(wout, d0 + 4 * j, v, lo_all, hi);
        }
    }
    if (q == (kLpr > 1 ? 1 : 0)) {
#pragma unroll
        for (int f = 0; f < LY::kNF; ++f) {
            const int32_t P = E.rw + (f == 0 ? LY::kLit : zat(E, f - 1) - 2);
            const uint32_t L = I.L[f] & 0xffffu;
            if (P >= lo_all && P < hi_all) wout[wout_addr(P)] = (uint8_t)L;
            if (P + 1 >= lo_all && P + 1 < hi_all) wout[wout_addr(P + 1)] = (uint8_t)(L >> 8);
        }
    }
}

// the 4 bytes of v at consecutive byte addresses from p
__device__ __forceinline__ void put_b4(lds_u8* p, uint32_t v) {
    p[0] = (uint8_t)v;
    p[1] = (uint8_t)(v >> 8);
    p[2] = (uint8_t)(v >> 16);
    p[3] = (uint8_t)(v >> 24);
}

// The literal prefix and the u16 lengths of every record of the window.  A record whose composed
// bytes lie whole inside the window (the common case) writes them as byte stores (no alignment
// assumption, no clipping; a dword that crosses a padded row goes byte by byte); others go through
// literal_clip.
template <class LY>
__device__ __forceinline__ void literal_pass(const EncArgs& ea, lds_u8* wout, lds_i32* rt, const TileSt& S,
                                             int32_t wlen, int lane) {
    SBE_TILE_SHAPE(LY);
    const int q = lane % kLpr, r = lane / kLpr;
    if (!S.rec_out) return;
    const RecEnt E = rec_load(rt, r);
    if (E.rend <= (E.rw > 0 ? E.rw : 0) || E.rw >= wlen) return;  // nothing of the record in this window
    LitIn I;
    I.ts = S.ts;
    I.tid = S.tid;
    I.term = ea.term_id;
    I.sess = ea.sess_id;
    I.tmpl = ea.tmpl;
#pragma unroll
    for (int f = 0; f < 5; ++f) I.L[f] = S.L[f];
    const bool whole = E.rw >= 0 && E.rend <= wlen && S.pe_rec == S.rs + S.rec_out;
    if (!whole) {
        literal_clip<LY>(wout, E, I, wlen, q);
        return;
    }
    if (q == 0) {
#pragma unroll
        for (int j = 0; j < LY::kLit / 4; ++j) {
            const uint32_t w = lit_word_v<LY>(I, j);
            const int32_t x = E.rw + 4 * j;
            if (((x ^ (x + 3)) >> 8) == 0) {
                put_b4(wout + wout_addr(x), w);
            } else {
#pragma unroll
                for (int k = 0; k < 4; ++k) wout[wout_addr(x + k)] = (uint8_t)(w >> (8 * k));
            }
        }
    }
    if (q == (kLpr > 1 ? 1 : 0)) {
#pragma unroll
        for (int f = 0; f < LY::kNF; ++f) {
            // the length bytes inside the record's composed bytes (a REF_TRUNCATE8 record ends 8
            // bytes short of the wire record, cutting trailing lengths)
            const int32_t P = E.rw + (f == 0 ? LY::kLit : zat(E, f - 1) - 2);
            const uint32_t L = I.L[f];
            if (P < E.rend) wout[wout_addr(P)] = (uint8_t)L;
            if (P + 1 < E.rend) wout[wout_addr(P + 1)] = (uint8_t)(L >> 8);
        }
    }
}

template <class LY>
__device__ __forceinline__ void pack_window(const EncArgs& ea, lds_u8* wout, lds_u8* inb, lds_i32* rt, lds_i32* bk,
                                            uint64_t* sbase, const TileSt& S, int32_t wrel, int32_t wlen,
                                            uintptr_t swb, int32_t nb, int lane, int ra = 0, int rb = LY::kRpt) {
    SBE_TILE_SHAPE(LY);
    // chunks per lane for this window: 1, 2, 4, 8 or 16 (the lane's range: 16 kk = 2^lg bytes)
    const int kk = wlen <= 1024 ? 1 : wlen <= 2048 ? 2 : wlen <= 4096 ? 4 : wlen <= 8192 ? 8 : kCpl;
    const int lg = kk == 1 ? 4 : kk == 2 ? 5 : kk == 4 ? 6 : kk == 8 ? 7 : 8;
    static_assert(kCpl == 16 || kCpl == 8 || kCpl == 4, "chunk ownership sizes");
    const bool outside = build_tables<LY>(rt, bk, sbase, S, wrel, wlen, swb, nb, ra, rb, lg, lane);
    wsync();
    chunk_pass<LY>(wout, inb, rt, bk, wlen, nb, kk, lg, lane);
    if (outside) chunk_pass_global<LY>(wout, rt, bk, (const lds_u64*)sbase, wlen, kk, lg, lane);
    wsync();
    zone_fixup<LY>(wout, inb, rt, wlen, nb, lane, ra, rb);
    wsync();
    literal_pass<LY>(ea, wout, rt, S, wlen, lane);
}

// ---- record-lane composition (the fast path) ---------------------------------------------
// For a window holding whole, staged, unclipped records [ra, rb): lane 2j+q composes half of
// record j's own chunks (the 16-byte chunks whose first byte lies in the record; a chunk's string
// bytes always belong to that record, string bytes starting >= 26 B in): zone of the chunk's
// first byte, five LDS dword reads and four v_alignbyte, later zones merged over the tail where a
// string starts inside the chunk; then the record's literal bytes (session / SBE header, fixed
// block, u16 lengths), split over the record's two lanes.  No record table, no walk: every lane
// works from its own record's registers.
template <class LY>
__device__ __forceinline__ bool compose_records(const EncArgs& ea, lds_u8* wout, lds_cu8* inb, lds_i32* rt,
                                                const TileSt& S, int32_t wrel, int32_t wlen, uintptr_t swb, int32_t nb,
                                                int lane, int ra, int rb, Ph& ph, bool spread = false) {
    SBE_TILE_SHAPE(LY);
    const int q = lane % kLpr, r = lane / kLpr;
    const bool live = S.rec_out != 0 && r >= ra && r < rb;
    const int32_t rw = (int32_t)S.rs - wrel;  // record start in the window
    const int32_t rl = (int32_t)S.rec_out;
    const int64_t src0l = (int64_t)(S.in_tile + S.in0) - (int64_t)swb;  // staged position of string 0
    uint32_t nstr = 0;
#pragma unroll
    for (int f = 0; f < LY::kNF; ++f) nstr += S.L[f];
    const bool ok = !live || (src0l >= 0 && src0l + (int64_t)nstr <= (int64_t)nb && S.pe_rec == S.rs + S.rec_out &&
                              rw >= 0 && rw + rl <= wlen);
    if (__ballot(!ok)) return false;
    const int32_t src0 = (int32_t)src0l - LY::kS0;  // input position of zone-0 byte x: src0 + x
    // record-relative string starts z1..z4 (absent fields start at the end of the last string)
    int32_t zs[5];
    {
        int32_t z = LY::kS0;
#pragma unroll
        for (int f = 1; f < 5; ++f) {
            if (f < LY::kNF) z += (int32_t)S.L[f - 1] + 2;
            zs[f - 1] = z;
        }
        zs[4] = z + (int32_t)S.L[LY::kNF - 1];
#pragma unroll
        for (int f = LY::kNF; f < 5; ++f) zs[f - 1] = zs[4];
    }
    const int32_t z1 = zs[0], z2 = zs[1], z3 = zs[2], z4 = zs[3];
    // this lane's chunks: the first (q = 0) or second half of the record's own chunks (kLpr = 1:
    // all of them)
    const int32_t c0 = (rw + 15) >> 4, nc = live ? ((rw + rl + 15) >> 4) - c0 : 0;
    const int32_t h = kLpr == 2 ? (nc + 1) >> 1 : nc;
    int32_t cb = c0 + (q ? h : 0), n_mine = q ? nc - h : h;
    // the record this lane composes chunks of (its own unless rebalanced)
    int32_t brw = rw, bsrc0 = src0, bz1 = z1, bz2 = z2, bz3 = z3, bz4 = z4;
    // Session frames and Lite records: rebalance only when it shortens the two-lane split's longest
    // lane (records of equal lengths just over 2 kCpl chunks, e.g. 280-B frames, are better off
    // split in two).  The plain TopicMessage layout keeps the unconditional rebalance: its windows
    // never gain from the check, and the extra code measured +0.6 % on the fixed-256 pack.
    constexpr bool kGuard = !(LY::kTM && LY::kPre == 0);
    bool rebal = false;
    uint32_t T = 0;
#ifndef SBE_REBAL_MIN  // A/B: chunks per lane above which a window is rebalanced
#define SBE_REBAL_MIN kCpl
#endif
    // spread (the serve kernel: a lone wave with few records): rebalance whenever some lane has
    // more than one chunk, so the chunks of a few records use the whole wave
    if (__ballot(n_mine > (spread ? 1 : SBE_REBAL_MIN))) {
        const bool lead = q == 0 && nc > 0;
        const uint32_t C = lane_u32(wave_incl_scan(lead ? (uint32_t)nc : 0u, lane), kWave - 1);
        const uint32_t nrec = (uint32_t)__builtin_popcountll(__ballot(lead));
        // T chunks per lane: the smallest of T0 .. T0 + 3 (T0 = ceil(C / 64)) whose records' runs
        // of ceil(nc_j / T) lanes fit the wave, from one scan of the four lane counts packed in
        // bytes (each sum <= C / T0 + records <= 128, so no byte carries into the next); else
        // ceil(C / (64 - records)), which always fits (sum of ceil(nc_j / T) <= C / T + records);
        // no spare lane: no rebalance.  Variable-length TopicMessage windows (~21 records, ~390
        // chunks) take T0 + 1 where the bound gives 10-12.
        const uint32_t T0 = (C + kWave - 1) / kWave;
        uint32_t pk = 0;
        if (lead) {
#pragma unroll
            for (uint32_t k = 0; k < 4; ++k) pk |= ceil_div_small((uint32_t)nc, T0 + k) << (8 * k);
        }
        const uint32_t S4 = lane_u32(wave_incl_scan(pk, lane), kWave - 1);
        T = nrec < (uint32_t)kWave ? (C + (kWave - nrec) - 1) / (kWave - nrec) : 0u;
#pragma unroll
        for (int k = 3; k >= 0; --k)
            if (((S4 >> (8 * k)) & 0xffu) <= (uint32_t)kWave) T = T0 + (uint32_t)k;
        const uint32_t mx = lane_u32(wave_incl_max((uint32_t)(n_mine > 0 ? n_mine : 0)), kWave - 1);
        rebal = T != 0 && (kGuard && !spread ? T < mx : true);
    }
    if (rebal) {
        // records of unequal lengths (variable-length records, or one long record): two lanes per
        // record would let the longest record set the wave's loop count.  Rebalance: T chunks per
        // lane with T = ceil(C / (64 - records)), record j served by ceil(nc_j / T) consecutive
        // lanes (at most 64 in all); a lane finds its record by a max-scan of the lanes where the
        // records' runs start, then reads that record's registers from its lead lane.
        const bool lead = q == 0 && nc > 0;
        const uint32_t L = lead ? ceil_div_small((uint32_t)nc, T) : 0u;
        const uint32_t incL = wave_incl_scan(L, lane);
        const uint32_t A = incL - L;  // first lane serving this lane's record (lead lanes)
        const uint32_t used = lane_u32(incL, kWave - 1);
        // lane A of every record learns the record's lead lane + 1 (0: no record starts there),
        // through the record-table area (written again below)
        rt[lane] = 0;
        wsync();
        if (lead) rt[A] = lane + 1;
        wsync();
        const uint32_t start = (uint32_t)rt[lane];
        wsync();
        const uint32_t owner1 = wave_incl_max(start);  // lead lane + 1 of the record this lane serves
        const int owner = (int)owner1 - 1;
        const bool serve = (uint32_t)lane < used && owner >= 0;
        const int src = owner >= 0 ? owner : lane;
        const int32_t oA = __shfl((int32_t)A, src, kWave), oc0 = __shfl(c0, src, kWave), onc = __shfl(nc, src, kWave);
        brw = __shfl(rw, src, kWave);
        bsrc0 = __shfl(src0, src, kWave);
        bz1 = __shfl(z1, src, kWave);
        bz2 = __shfl(z2, src, kWave);
        bz3 = __shfl(z3, src, kWave);
        bz4 = __shfl(z4, src, kWave);
        const int32_t part = lane - oA;
        cb = oc0 + part * (int32_t)T;
        n_mine = serve ? min((int32_t)T, onc - part * (int32_t)T) : 0;
        n_mine = n_mine > 0 ? n_mine : 0;
    }
    const int32_t imax = (nb + kInSlack) / 4 - 5;
    // groups of kG chunks, all their LDS reads in flight together: 4 while some lane has 4 left,
    // then a group of 2 and one of 1 as the longest lane needs them (a rebalanced window's T is
    // rarely a multiple of 4)
    auto group = [&](auto kGc, int32_t i0) {
        constexpr int kG = decltype(kGc)::value;
        int32_t u[kG];
#if SBE_CHUNK_UA
        u32x4 w[kG];
#else
        uint32_t d[kG][5];
#endif
#pragma unroll
        for (int k = 0; k < kG; ++k) {
            const int32_t X = 16 * (cb + i0 + k) - brw;
            const int32_t f = (X >= bz1) + (X >= bz2) + (X >= bz3) + (X >= bz4);
            u[k] = bsrc0 + X - 2 * f;
#if SBE_CHUNK_UA
            w[k] = lds_chunk_ua(inb, u[k], imax - 1);
#else
            int32_t i = u[k] >> 2;
            i = i < -kInSlack / 4 ? -kInSlack / 4 : (i > imax - 1 ? imax - 1 : i);
            lds_dw5(inb, i, d[k]);
#endif
        }
#pragma unroll
        for (int k = 0; k < kG; ++k) {
            // the zone of the chunk's first byte; string starts inside it: zone_fixup
#if SBE_CHUNK_UA
            const u32x4 v = w[k];
#else
            const u32x4 v = align4(d[k][0], d[k][1], d[k][2], d[k][3], d[k][4], (uint32_t)u[k] & 3u);
#endif
            if (i0 + k < n_mine) {
                const int32_t p = 16 * (cb + i0 + k);
                *reinterpret_cast<lds_u32x4*>(wout + wout_addr(p)) = v;
            }
        }
    };
    int32_t i0 = 0;
    for (; __ballot(i0 + 3 < n_mine); i0 += 4) group(std::integral_constant<int, 4>{}, i0);
    if (__ballot(i0 + 1 < n_mine)) {
        group(std::integral_constant<int, 2>{}, i0);
        i0 += 2;
    }
    if (__ballot(i0 < n_mine)) group(std::integral_constant<int, 1>{}, i0);
    if (q == 0) {  // the record table entry zone_fixup reads (RecEnt; no record clipped here)
        i32x4 ea4, eb4;
        ea4.x = rw;
        ea4.y = live ? rw + rl : rw;
        ea4.z = rw - src0;
        ea4.w = z1;
        eb4.x = z2;
        eb4.y = z3;
        eb4.z = z4;
        eb4.w = zs[4];
        reinterpret_cast<lds_i32x4*>(rt + kRecEnt * r)[0] = ea4;
        reinterpret_cast<lds_i32x4*>(rt + kRecEnt * r)[1] = eb4;
    }
    wsync();
    ph.lap(1);
    zone_fixup<LY>(wout, inb, rt, wlen, nb, lane, ra, rb);
    wsync();
    ph.lap(2);
    if (!live) return true;
    // literal bytes: q = 0 the header prefix (TopicMessage.h:221-238, :362-437), q = 1 the lengths
    // (:515-1231; a REF_TRUNCATE8 record ends 8 bytes short of the wire record, cutting trailing ones)
    LitIn I;
    I.ts = S.ts;
    I.tid = S.tid;
    I.term = ea.term_id;
    I.sess = ea.sess_id;
    I.tmpl = ea.tmpl;
    // The literal bytes split over the record's two lanes, one instruction stream for both (no
    // divergent header / lengths branches): part p = q writes half of the header's aligned dwords
    // (p = 0 the bytes before the first aligned one, p = 1 those after the last) and the lengths
    // of fields f = 2k + p, each as one ds_write_b16 where it is 2-aligned.  kLpr = 1: the
    // record's lane writes both parts.
    constexpr int kW = LY::kLit / 4, kH = (kW + 1) / 2;
    uint32_t w[kW];
#pragma unroll
    for (int j = 0; j < kW; ++j) w[j] = lit_word_v<LY>(I, j);
    const uint32_t a = (uint32_t)(-rw) & 3u;  // header bytes before the first 4-aligned position
    const int32_t xa = rw + (int32_t)a;
    const int nA = a ? kW - 1 : kW;            // whole aligned dwords of the header
    auto part = [&](int p) {
        // dword k of the aligned run (k compile-time per unrolled step, lane-dependent by p)
#pragma unroll
        for (int k = 0; k < kH; ++k) {
            const int kk = p ? kH + k : k;
            uint32_t v = 0;
#pragma unroll
            for (int j = 0; j < kW; ++j)
                if (j == kk) v = a ? __builtin_amdgcn_alignbyte(w[j + 1 < kW ? j + 1 : j], w[j], a) : w[j];
            if (kk < nA) *reinterpret_cast<lds_u32*>(wout + wout_addr(xa + 4 * kk)) = v;
        }
        if (a) {  // p = 0: the a bytes before the run; p = 1: the 4 - a bytes after it
            const uint32_t src = p ? w[kW - 1] : w[0];
            const int32_t x0 = p ? rw + LY::kLit - 4 + (int32_t)a : rw;
            const uint32_t sh0 = p ? a : 0u, cnt = p ? 4u - a : a;
#pragma unroll
            for (uint32_t t = 0; t < 3; ++t)
                if (t < cnt) wout[wout_addr(x0 + (int32_t)t)] = (uint8_t)(src >> (8 * (sh0 + t)));
        }
#pragma unroll
        for (int k = 0; k < (LY::kNF + 1) / 2; ++k) {
            const int f = 2 * k + p;
            if (f >= LY::kNF) continue;
            int32_t P = LY::kLit;
            uint32_t L = S.L[0];
#pragma unroll
            for (int g = 1; g < LY::kNF; ++g)
                if (g == f) {
                    P = zs[g - 1] - 2;
                    L = S.L[g];
                }
            const int32_t X = rw + P;
            if (P + 1 < rl && ((X & 1) == 0)) {
                *reinterpret_cast<__attribute__((address_space(3))) uint16_t*>(wout + wout_addr(X)) = (uint16_t)L;
            } else {
                if (P < rl) wout[wout_addr(X)] = (uint8_t)L;
                if (P + 1 < rl) wout[wout_addr(X + 1)] = (uint8_t)(L >> 8);
            }
        }
    };
    if (kLpr == 2) {
        part(q);
    } else {
        part(0);
        part(1);
    }
    return true;
}

// A tile whose output exceeds the window is split at record boundaries: window [ra, rb) holds
// whole records only (none straddles, so all of them are staged), output bytes [wrel, wrel+wlen)
// relative to T0 with wrel the 16-B aligned start below record ra's first byte A, and staged
// input [swb, swb+nb) = the strings of records [ra, rb).  A tile with a record longer than the
// window minus 16 bytes takes the byte-window path instead (tile_big).
struct Win {
    int ra, rb;
    int32_t wrel, wlen;
    uint32_t A;
    uintptr_t swb;
    int32_t nb;
};

template <class LY>
__device__ __forceinline__ bool tile_big(const TileSt& S, int lane) {
    SBE_TILE_SHAPE(LY);
    return __ballot(lane % kLpr == 0 && S.rec_out > (uint32_t)(kEW - 16)) != 0;
}

template <class LY>
__device__ __forceinline__ Win tile_window(const TileSt& S, int ra, int lane, uintptr_t sink) {
    SBE_TILE_SHAPE(LY);
    Win W;
    const int q = lane % kLpr, r = lane / kLpr;
    W.ra = ra;
    W.A = lane_u32(S.rs, ra * kLpr);
    W.wrel = (int32_t)W.A - (int32_t)((S.T0 + W.A) & 15u);
    // records from ra whose (capacity-clipped) end fits: ends are non-decreasing, so a prefix
    const bool fits = q == 0 && r >= ra && (int32_t)S.pe_rec - W.wrel <= kEW;
    const int cnt = __builtin_popcountll(__ballot(fits));
    W.rb = ra + (cnt > 0 ? cnt : 1);
    const uint32_t B = lane_u32(S.pe_rec, (W.rb - 1) * kLpr);
    W.wlen = (int32_t)B - W.wrel;
    const uint64_t ia = lane_u64(S.in0, ra * kLpr);
    const uint64_t ib = W.rb < kRpt ? lane_u64(S.in0, W.rb * kLpr) : (uint64_t)S.agg_in;
    W.swb = (S.in_tile + ia) & ~(uintptr_t)15;
    const uintptr_t end = (S.in_tile + ib + 15) & ~(uintptr_t)15;
    W.nb = (int32_t)(end - W.swb < (uintptr_t)kEWIn ? end - W.swb : (uintptr_t)kEWIn);
    if (W.nb == 0) W.swb = sink;  // stage_issue reads 16 bytes at swb even then
    return W;
}

// The pack loop's LDS (one workgroup): output window, staged input, record / bucket tables.
template <class LY, bool kPacked>
struct PackLds {
    __attribute__((aligned(16))) uint8_t wout[kWoutBytes];
    __attribute__((aligned(16))) uint8_t win[kPacked ? kWinBytes : 16];
    __attribute__((aligned(16))) int32_t rt[kPacked ? LY::kRpt * kRecEnt : 4];
    int32_t bk[kPacked ? kWave : 1];
    uint64_t sbase[kPacked ? LY::kRpt : 1];
};

// Tiles first, first + G, ... of the batch (the pack kernel: first = blockIdx.x, G = gridDim.x;
// the serve kernel: 0, 1 for a one-tile batch).
template <class LY, bool kPacked, int kLen>
__device__ __forceinline__ void enc_pack_run(const EncArgs& a, uint64_t first, uint64_t G, PackLds<LY, kPacked>& L) {
    SBE_TILE_SHAPE(LY);
    lds_u8* const wout = (lds_u8*)L.wout;
    lds_u8* const win_in = (lds_u8*)L.win + kInSlack;
    lds_i32* const rt = (lds_i32*)L.rt;
    lds_i32* const bk = (lds_i32*)L.bk;
    uint64_t* const sbase = L.sbase;
    const int lane = threadIdx.x;
    const uint64_t ntiles = (a.n + kRpt - 1) / kRpt;
    uint64_t t = first;
    if (t >= ntiles) return;
    Ph ph;
    ph.start();

    uint64_t sb_next = 0, sp_out = 0, sp_in = 0;
    TileIn x = tile_load<LY, kPacked>(a, t, lane, sb_next);
    TileSt S = tile_prepare<LY, kPacked, kLen>(a, x, t, lane, sp_out, sp_in);
    uint4 I[kStageRegs];
    const uintptr_t sink = reinterpret_cast<uintptr_t>(a.sink);
    Win W{0, kRpt, 0, 0, 0, sink, 0};
    bool fast = kPacked && !S.wrapped && !tile_big<LY>(S, lane);
    if (fast) W = tile_window<LY>(S, 0, lane, sink);
    if (kPacked) {
        stage_issue<LY::kNtIn>(W.swb, W.nb, lane, I);
        stage_write(win_in, W.nb, lane, I);
    }
    uint64_t tn = t + G;
    x = tile_load<LY, kPacked>(a, tn < ntiles ? tn : ntiles - 1, lane, sb_next);

    // Steady state, per window: [next window of this tile, or the next tile (prepare, lengths of
    // the one after): staging loads] [compose + store this window] [next window's staged input →
    // LDS].  The staging registers are written to LDS after this window's stores, so that wait
    // leaves exactly those stores in flight.
    for (;;) {
        const bool more_win = fast && W.rb < kRpt && W.wrel + W.wlen < (int32_t)S.len;
        const bool have_next = more_win || tn < ntiles;
        TileSt Sn;
        Win Wn{0, kRpt, 0, 0, 0, sink, 0};
        bool fast_n = false;
        if (more_win) {
            Wn = tile_window<LY>(S, W.rb, lane, sink);
            fast_n = true;
        } else if (have_next) {
            Sn = tile_prepare<LY, kPacked, kLen>(a, x, tn, lane, sp_out, sp_in);
            ph.lap(7);
            const uint64_t t2 = tn + G;
            x = tile_load<LY, kPacked>(a, t2 < ntiles ? t2 : ntiles - 1, lane, sb_next);
            fast_n = kPacked && !Sn.wrapped && !tile_big<LY>(Sn, lane);
            if (fast_n) Wn = tile_window<LY>(Sn, 0, lane, sink);
        }
        if (have_next && kPacked) stage_issue<LY::kNtIn>(Wn.swb, Wn.nb, lane, I);
        ph.lap(0);
        // current window (fast) or the whole tile window by window
        if (fast) {
            if (!compose_records<LY>(a, wout, win_in, rt, S, W.wrel, W.wlen, W.swb, W.nb, lane, W.ra, W.rb, ph)) {
                pack_window<LY>(a, wout, win_in, rt, bk, sbase, S, W.wrel, W.wlen, W.swb, W.nb, lane, W.ra, W.rb);
                ph.lap(6);
            } else {
                ph.lap(3);
            }
            wsync();
            store_window<(LY::kStoreRows0 < kStoreRows ? LY::kStoreRows0 : kStoreRows)>(a.out, wout, S.T0 + W.A, S.T0 + (int64_t)W.wrel,
                                          S.T0 + (int64_t)(W.wrel + W.wlen), lane);
            wsync();
            ph.lap(4);
        } else {
            const int32_t wrel0 = -(int32_t)(S.T0 & 15);
            for (int32_t wrel = wrel0; wrel < (int32_t)S.len; wrel += kEW) {
                const int32_t we_rel = wrel + kEW < (int32_t)S.len ? wrel + kEW : (int32_t)S.len;
                uintptr_t sw = 0;
                int32_t nbw = 0;
                if (kPacked && !S.wrapped) {
                    stage_range<LY>(S, wrel, lane, sw, nbw);
                    // I holds the next item's prefetch: stage this window in batches of 3 chunks
                    for (int k0 = 0; k0 < kStageRegs; k0 += 3) {
                        uint4 J[3];
#pragma unroll
                        for (int k = 0; k < 3; ++k) {
                            const uint32_t ch = lane + kWave * (k0 + k);
                            J[k] = (int32_t)(16 * ch) < nbw ? gload128(sw + 16u * ch) : make_uint4(0, 0, 0, 0);
                        }
#pragma unroll
                        for (int k = 0; k < 3; ++k) {
                            const uint32_t ch = lane + kWave * (k0 + k);
                            if ((int32_t)(16 * ch) < nbw) lds_store16(win_in + 16 * ch, J[k]);
                        }
                    }
                }
                if (kPacked && !S.wrapped) {
                    pack_window<LY>(a, wout, win_in, rt, bk, sbase, S, wrel, we_rel - wrel, sw, nbw, lane);
                } else {  // gather mode, or a kLenPub tile whose outputs are shorter than its inputs
                    wsync();
                    compose<LY, false>(a, wout, win_in, S, wrel, we_rel, sw, nbw);
                }
                wsync();
                store_window(a.out, wout, S.T0, S.T0 + (int64_t)wrel, S.T0 + (uint64_t)we_rel, lane);
                wsync();
            }
            ph.lap(6);
        }
        if (!have_next) break;
        if (kPacked) stage_write(win_in, Wn.nb, lane, I);  // after the compose above read win_in
        wsync();
        ph.lap(5);
        if (!more_win) {
            S = Sn;
            tn += G;
        }
        W = Wn;
        fast = fast_n;
    }
    ph.put(lane);
}

// ---- virtual tiles: every window full -----------------------------------------------------
// The tiles are cut into chunks of CT consecutive tiles, dealt to the workgroups round robin
// (chunk c to workgroup c mod G, as the tile loop deals tiles).  A workgroup walks its chunk's
// records in order with running output / input offsets: each step takes the kRpt records from the
// first one not yet written (a "virtual tile", at any record index) and writes ONE output window,
// the records from its first that fit kEW bytes, so every window but a chunk's last is full.
// (Tile-aligned steps leave a tile's last window part full: a 32-record tile of ~380-B records is
// a full 8 KiB window and a ~4 KiB one, and a window costs about the same whatever it holds.)  The
// records after the window start the next step; their lengths are loaded one step ahead, like the
// tiles'.  Chunks rather than one contiguous range per workgroup: the windows in flight at once
// then lie CT tiles apart, not n / G records (contiguous ranges measured the fixed-256 pack 10 %
// slower, profiles/r04_ab_vt.log; chunks did not recover it, see SBE_PACK_VT).  A virtual tile
// the fast path cannot take (a record longer than a window, gather mode, a PUBLISH_TOPIC length
// wrap) is written whole, window by window.
#ifndef SBE_VT_CHUNK  // tiles per chunk (0: one contiguous range per workgroup, the batch kernel's)
#define SBE_VT_CHUNK 0
#endif
template <class LY, bool kPacked>
__device__ __forceinline__ TileIn vt_load(const EncArgs& a, uint64_t r0, int lane) {
    SBE_TILE_SHAPE(LY);
    TileIn x;
    uint64_t r = r0 + (uint64_t)(lane / kLpr);
    r = r < a.n ? r : a.n - 1;  // unconditional loads at a clamped index (tile_load)
#pragma unroll
    for (int f = 0; f < 5; ++f) x.L[f] = f < LY::kNF ? a.str_len[LY::kNF * r + f] : 0u;
    x.ts = a.timestamp[r];
    x.tid = LY::kTM ? 0u : a.topic_id[r];
    x.to = x.ti = x.po = x.pi = 0;
    x.pcount = 0;
    return x;
}

// The lengths of chunk start tile t's first records plus the terms of its base: the tile's prefix
// inside its superblock (sbe_enc_sums) and, per lane, its share of the superblock totals from
// sb_next up to the tile's superblock (a workgroup's chunks come in increasing order, so each
// superblock total is loaded once).
template <class LY, bool kPacked>
__device__ __forceinline__ TileIn vt_chunk_load(const EncArgs& a, uint64_t t, int lane, uint64_t& sb_next) {
    SBE_TILE_SHAPE(LY);
    TileIn x = vt_load<LY, kPacked>(a, t * kRpt, lane);
    x.to = a.tsum[2 * t];
    x.ti = kPacked ? a.tsum[2 * t + 1] : 0ull;
    const uint64_t sbt = t / kTilesPerSb;
    uint64_t po = 0, pi = 0;
    for (uint64_t s = sb_next + (uint64_t)lane; s < sbt; s += kWave) {
        po += a.bsum[2 * s];
        if (kPacked) pi += a.bsum[2 * s + 1];
    }
    x.po = po;
    x.pi = pi;
    sb_next = sbt > sb_next ? sbt : sb_next;
    return x;
}

#ifdef SBE_VT_GUARD
// Debug build only: the first out-of-range window of the virtual-tile loop, recorded instead of
// stored (read with sbe_debug_vt_guard).
__device__ uint64_t g_vt_guard[16];
#endif

template <class LY, bool kPacked, int kLen>
__device__ __forceinline__ void enc_pack_run_vt(const EncArgs& a, uint64_t first, uint64_t G, PackLds<LY, kPacked>& L,
                                                uint64_t chunk_tiles = SBE_VT_CHUNK, bool spread = false) {
    SBE_TILE_SHAPE(LY);
    lds_u8* const wout = (lds_u8*)L.wout;
    lds_u8* const win_in = (lds_u8*)L.win + kInSlack;
    lds_i32* const rt = (lds_i32*)L.rt;
    lds_i32* const bk = (lds_i32*)L.bk;
    uint64_t* const sbase = L.sbase;
    const int lane = threadIdx.x;
    const uint64_t ntiles = (a.n + kRpt - 1) / kRpt;
    const uint64_t CT = chunk_tiles > 0 ? chunk_tiles : (ntiles + G - 1) / G;
    const uint64_t nch = (ntiles + CT - 1) / CT;
    uint64_t c = first;
    if (c >= nch) return;
    const uint64_t CR = CT * kRpt;  // records per chunk
    auto chunk_end = [&](uint64_t cc) { return cc * CR + CR < a.n ? cc * CR + CR : a.n; };
    Ph ph;
    ph.start();
    uint64_t sb_next = 0, sp_out = 0, sp_in = 0;
    uint64_t bo = 0, bi = 0;
    // a new chunk's base: the superblock totals loaded with its lengths, then its tile prefix
    auto chunk_base = [&](const TileIn& x_) {
        sp_out += wave_sum64(x_.po);
        if (kPacked) sp_in += wave_sum64(x_.pi);
        bo = uniform64(sp_out + x_.to);
        bi = kPacked ? uniform64(sp_in + x_.ti) : 0ull;
    };
    const uintptr_t sink = reinterpret_cast<uintptr_t>(a.sink);
    // records written by the step of tile S with window W; bo / bi move past them
    auto advance = [&](const TileSt& S_, const Win& W_, bool fast_) -> uint32_t {
        const uint32_t k = fast_ ? (uint32_t)W_.rb : (uint32_t)kRpt;
        if (k < (uint32_t)kRpt) {
            bo += lane_u32(S_.rs, (int)k * kLpr);
            if (kPacked) bi += lane_u64(S_.in0, (int)k * kLpr);
        } else {
            bo += S_.agg_out;
            if (kPacked) bi += S_.tot_in;
        }
        return k;
    };
    uint64_t r_hi = chunk_end(c);
#ifdef SBE_VT_GUARD
    uint64_t tot_in_all = 0;
    {
        const uint64_t nsb_all = (a.n + kSbRec - 1) / kSbRec;
        uint64_t si = 0;
        for (uint64_t j = (uint64_t)lane; j < nsb_all; j += kWave) si += a.bsum[2 * j + 1];
        tot_in_all = uniform64(wave_sum64(si));
    }
    // true (and the first such window recorded) when a window would store past the capacity or
    // stage outside the packed arena
    auto bad = [&](uint64_t code, const TileSt& S_, int64_t wrel_, int64_t wlen_, uintptr_t swb_, int64_t nb_,
                   uint64_t r_) -> bool {
        const uintptr_t a0 = reinterpret_cast<uintptr_t>(a.arena);
        bool b = wlen_ < 0 || wlen_ > kEW + 16 || (int64_t)S_.T0 + wrel_ + wlen_ > (int64_t)a.cap ||
                 (int64_t)S_.T0 + wrel_ < -16 || nb_ < 0 || nb_ > kEWIn;
        if (kPacked && nb_ > 0 && (swb_ + 16 < a0 || swb_ + (uintptr_t)nb_ > a0 + tot_in_all + 16)) b = true;
        if (!b) return false;
        if (lane == 0 && atomicCAS((unsigned long long*)&g_vt_guard[0], 0ull, code) == 0ull) {
            g_vt_guard[1] = first;
            g_vt_guard[2] = r_;
            g_vt_guard[3] = S_.T0;
            g_vt_guard[4] = (uint64_t)wrel_;
            g_vt_guard[5] = (uint64_t)wlen_;
            g_vt_guard[6] = swb_ - a0;
            g_vt_guard[7] = (uint64_t)nb_;
            g_vt_guard[8] = tot_in_all;
            g_vt_guard[9] = r_hi;
            g_vt_guard[10] = S_.agg_out;
            g_vt_guard[11] = S_.in_tile - a0;
            g_vt_guard[12] = a.n;
        }
        return true;
    };
#endif
    TileIn x = vt_chunk_load<LY, kPacked>(a, c * CT, lane, sb_next);
    chunk_base(x);
    uint64_t rn = c * CR;
    TileSt S = tile_prepare_at<LY, kPacked, kLen>(a, x, rn, r_hi, lane, bo, bi);
    uint4 I[kStageRegs];
    Win W{0, kRpt, 0, 0, 0, sink, 0};
    bool fast = kPacked && !S.wrapped && !tile_big<LY>(S, lane);
    if (fast) W = tile_window<LY>(S, 0, lane, sink);
#ifdef SBE_VT_GUARD
    if (fast && bad(1, S, W.wrel, W.wlen, W.swb, W.nb, rn)) return;
#endif
    rn += advance(S, W, fast);
    if (kPacked) {
        stage_issue<LY::kNtIn>(W.swb, W.nb, lane, I);
        stage_write(win_in, W.nb, lane, I);
    }
    // the next step: the rest of this chunk, or the workgroup's next chunk (its base from the
    // superblock totals loaded with its lengths)
    uint64_t cn = c + G;
    bool nxt_new = rn >= r_hi;
    if (nxt_new) {
        rn = cn * CR;
        x = vt_chunk_load<LY, kPacked>(a, (cn < nch ? cn : nch - 1) * CT, lane, sb_next);
    } else {
        x = vt_load<LY, kPacked>(a, rn, lane);
    }

    for (;;) {
        const bool have_next = !nxt_new || cn < nch;
        TileSt Sn;
        Win Wn{0, kRpt, 0, 0, 0, sink, 0};
        bool fast_n = false, nxt_new_n = false;
        uint64_t rnn = rn;
        if (have_next) {
            if (nxt_new) {
                c = cn;
                cn = c + G;
                r_hi = chunk_end(c);
                chunk_base(x);
            }
            Sn = tile_prepare_at<LY, kPacked, kLen>(a, x, rn, r_hi, lane, bo, bi);
            ph.lap(7);
            fast_n = kPacked && !Sn.wrapped && !tile_big<LY>(Sn, lane);
            if (fast_n) Wn = tile_window<LY>(Sn, 0, lane, sink);
#ifdef SBE_VT_GUARD
            if (fast_n && bad(2, Sn, Wn.wrel, Wn.wlen, Wn.swb, Wn.nb, rn)) return;
#endif
            rnn = rn + advance(Sn, Wn, fast_n);
            nxt_new_n = rnn >= r_hi;
            if (nxt_new_n) {
                rnn = cn * CR;
                x = vt_chunk_load<LY, kPacked>(a, (cn < nch ? cn : nch - 1) * CT, lane, sb_next);
            } else {
                x = vt_load<LY, kPacked>(a, rnn, lane);
            }
        }
        if (have_next && kPacked) stage_issue<LY::kNtIn>(Wn.swb, Wn.nb, lane, I);
        ph.lap(0);
        if (fast) {
            if (!compose_records<LY>(a, wout, win_in, rt, S, W.wrel, W.wlen, W.swb, W.nb, lane, W.ra, W.rb, ph, spread)) {
                pack_window<LY>(a, wout, win_in, rt, bk, sbase, S, W.wrel, W.wlen, W.swb, W.nb, lane, W.ra, W.rb);
                ph.lap(6);
            } else {
                ph.lap(3);
            }
            wsync();
            store_window<(LY::kStoreRows0 < kStoreRows ? LY::kStoreRows0 : kStoreRows)>(a.out, wout, S.T0 + W.A, S.T0 + (int64_t)W.wrel,
                                          S.T0 + (int64_t)(W.wrel + W.wlen), lane);
            wsync();
            ph.lap(4);
        } else {  // the whole virtual tile, window by window (records longer than a window, gather mode)
            const int32_t wrel0 = -(int32_t)(S.T0 & 15);
            for (int32_t wrel = wrel0; wrel < (int32_t)S.len; wrel += kEW) {
                const int32_t we_rel = wrel + kEW < (int32_t)S.len ? wrel + kEW : (int32_t)S.len;
                uintptr_t sw = 0;
                int32_t nbw = 0;
                if (kPacked && !S.wrapped) {
                    stage_range<LY>(S, wrel, lane, sw, nbw);
#ifdef SBE_VT_GUARD
                    if (bad(4, S, wrel, we_rel - wrel, sw, nbw, rn)) return;
#endif
                    for (int k0 = 0; k0 < kStageRegs; k0 += 3) {
                        uint4 J[3];
#pragma unroll
                        for (int k = 0; k < 3; ++k) {
                            const uint32_t ch = lane + kWave * (k0 + k);
                            J[k] = (int32_t)(16 * ch) < nbw ? gload128(sw + 16u * ch) : make_uint4(0, 0, 0, 0);
                        }
#pragma unroll
                        for (int k = 0; k < 3; ++k) {
                            const uint32_t ch = lane + kWave * (k0 + k);
                            if ((int32_t)(16 * ch) < nbw) lds_store16(win_in + 16 * ch, J[k]);
                        }
                    }
                }
                if (kPacked && !S.wrapped) {
                    pack_window<LY>(a, wout, win_in, rt, bk, sbase, S, wrel, we_rel - wrel, sw, nbw, lane);
                } else {
                    wsync();
                    compose<LY, false>(a, wout, win_in, S, wrel, we_rel, sw, nbw);
                }
                wsync();
                store_window(a.out, wout, S.T0, S.T0 + (int64_t)wrel, S.T0 + (uint64_t)we_rel, lane);
                wsync();
            }
            ph.lap(6);
        }
        if (!have_next) break;
        if (kPacked) stage_write(win_in, Wn.nb, lane, I);  // after the compose above read win_in
        wsync();
        ph.lap(5);
        S = Sn;
        W = Wn;
        fast = fast_n;
        rn = rnn;
        nxt_new = nxt_new_n;
    }
    ph.put(lane);
}

// The batch pack kernel keeps the tile loop: per window, the virtual-tile loop re-prepares a tile
// (lengths, scans, offsets) where the tile loop reuses the tile's state for its second window, and
// that costs about what the full windows save (A/B in one process, pack µs tile → virtual tiles:
// fixed-256 97 → 103-114, config 4 728 → 722-827, session 135 → 134-151, OrderRequestLite 145 →
// 160, CommitOffsetLite 41 → 40-44 over chunk sizes 1-8 and contiguous ranges;
// profiles/r04_ab_vt_chunks.log).  The serve kernel uses the virtual-tile loop (running offsets,
// no tile sums).  SBE_PACK_VT=1 selects it for the batch kernel (A/B).
#ifndef SBE_PACK_VT  // A/B builds: 1 = always the virtual-tile loop, 2 = never; 0 = chosen per launch
#define SBE_PACK_VT 0
#endif
// Which loop pays is a matter of the windows a tile takes: a tile whose output ends in a part-full
// window pays that window's fixed cost (staging issue, store rows, fix-up passes) for little, and
// the virtual-tile loop (one contiguous record range per workgroup), whose windows are all full,
// wins; a tile of whole windows keeps the tile loop, which re-prepares nothing.  Measured on
// rotated inputs, pack us tile -> virtual tiles (profiles/r06_ab_vt.log; the tile's average output
// and its last window's fill in brackets): config 4's variable-length records 729.9 -> 695.3
// (12.4 KiB, 0.54), session frames 136.2 -> 130.4 (17.9 KiB, 0.23), 626-B records 648.4 -> 622.0
// (20 KiB, 0.45); fixed-256 95.6 -> 105.3 (8 KiB, one window), 502-B records 578.5 -> 600.0 (16 KiB,
// 0.96), OrderRequestLite 143.7 -> 156.1 (21.3 KiB, 0.65), CommitOffsetLite 43.6 -> 44.2 (one
// window).  So the kernel takes the virtual-tile loop when the average tile of the first
// superblock (sbe_enc_sums' totals: a uniform read, the same choice in every workgroup) needs more
// than one window and its last one is under 60 % full.
template <class LY>
__device__ __forceinline__ bool vt_pays(const EncArgs& a) {
    SBE_TILE_SHAPE(LY);
    const uint64_t n0 = a.n < (uint64_t)kSbRec ? a.n : (uint64_t)kSbRec;
    if (n0 < (uint64_t)kRpt) return false;
    const uint64_t t = uniform64(a.bsum[0]) * kRpt / n0;  // average output bytes of a tile
    if (t <= (uint64_t)kEW) return false;
    const uint64_t last = t - (t - 1) / kEW * kEW;        // bytes in the tile's last window
    return 10 * last < 6 * (uint64_t)kEW;
}
template <class LY, bool kPacked, int kLen>
__global__ __launch_bounds__(kWave, SBE_PACK_MIN_WAVES) void sbe_enc_pack(EncArgs a) {
    __shared__ PackLds<LY, kPacked> lds;
    if (SBE_PACK_VT == 1 || (SBE_PACK_VT == 0 && kPacked && vt_pays<LY>(a)))
        enc_pack_run_vt<LY, kPacked, kLen>(a, blockIdx.x, gridDim.x, lds, SBE_VT_CHUNK);
    else
        enc_pack_run<LY, kPacked, kLen>(a, blockIdx.x, gridDim.x, lds);
}

#include "seqnum.hpp"
#include "order_json.hpp"

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
    uint64_t* seq;  // parse mode, optional: sequence_number of the flagged TopicMessages
};

// Reads of one record: LDS window [wb, we) where staged, global memory elsewhere.
// Reads of one record.  LdsRec: the record lies inside the staged LDS window (the common case;
// 32-bit window offsets, no global path).  GlbRec: any other record, read from HBM.
struct LdsRec {
    const uint32_t* win;
    uint32_t base;  // record start, byte offset in the window
    __device__ __forceinline__ uint32_t adw(uint32_t p) const {  // dword holding record byte p (p & ~3 rel. to window)
        return lds_dw(win, (base + p) >> 2);
    }
    __device__ __forceinline__ uint32_t abs_align(uint32_t p) const { return (base + p) & 3u; }
    __device__ __forceinline__ uint32_t bytes(uint32_t p, uint32_t nb) const {
        const uint32_t ap = base + p, sh = ap & 3u;
        const uint32_t lo = lds_dw(win, ap >> 2);
        uint32_t v = lo >> (8 * sh);
        if (sh + nb > 4) v = __builtin_amdgcn_alignbyte(lds_dw(win, (ap >> 2) + 1), lo, sh);
        return v & byte_mask_bits(nb);
    }
    __device__ __forceinline__ uint16_t u16(uint32_t p) const { return (uint16_t)bytes(p, 2); }
    __device__ __forceinline__ uint32_t u32(uint32_t p) const { return bytes(p, 4); }
    __device__ __forceinline__ uint64_t u64(uint32_t p) const {
        return (uint64_t)bytes(p, 4) | ((uint64_t)bytes(p + 4, 4) << 32);
    }
};
struct GlbRec {
    uintptr_t base;  // absolute address of the record's first byte
    __device__ __forceinline__ uint32_t adw(uint32_t p) const { return gload32((base + p) & ~(uintptr_t)3); }
    __device__ __forceinline__ uint32_t abs_align(uint32_t p) const { return (uint32_t)((base + p) & 3u); }
    __device__ __forceinline__ uint32_t bytes(uint32_t p, uint32_t nb) const {
        const uintptr_t ap = base + p, qa = ap & ~(uintptr_t)3;
        const uint32_t sh = (uint32_t)(ap & 3u);
        const uint32_t lo = gload32(qa);
        uint32_t v = lo >> (8 * sh);
        if (sh + nb > 4) v = __builtin_amdgcn_alignbyte(gload32(qa + 4), lo, sh);
        return v & byte_mask_bits(nb);
    }
    __device__ __forceinline__ uint16_t u16(uint32_t p) const { return (uint16_t)bytes(p, 2); }
    __device__ __forceinline__ uint32_t u32(uint32_t p) const { return bytes(p, 4); }
    __device__ __forceinline__ uint64_t u64(uint32_t p) const {
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
    // views[k] for a runtime k: compare-and-select, so the arrays stay in registers (a dynamic
    // index would put the whole descriptor in scratch memory)
    __device__ __forceinline__ void set_view(uint32_t k, uint32_t o, uint32_t l) {
#pragma unroll
        for (uint32_t j = 0; j < 5; ++j) {
            if (j == k) {
                off[j] = o;
                len[j] = l;
            }
        }
    }
    __device__ __forceinline__ void fail(uint32_t st, uint32_t param) {
        clear();
        status = st;
        off[0] = param;
    }
    template <typename R_t>
    __device__ __forceinline__ void set_hdr(const R_t& R, uint32_t p) {
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

// "_sequence_number" anywhere in [p, p+n) of the record (flag only; src/sbe_encoder.cpp:1031-1125).
// Any occurrence fully covers one 4-aligned dword, which then equals key[j..j+4) for j = (4 - s%4)%4:
// one aligned dword per 4 payload bytes, compared with those four slices; a hit is verified.
constexpr uint32_t kSeqK0 = 0x7165735fu, kSeqK1 = 0x636e6575u, kSeqK2 = 0x756e5f65u, kSeqK3 = 0x7265626du;
constexpr uint32_t kSeqS1 = 0x75716573u, kSeqS2 = 0x65757165u, kSeqS3 = 0x6e657571u;  // key[1..5), [2..6), [3..7)

// candidate test of the aligned dword w at record offset q
template <typename R_t>
__device__ __forceinline__ bool seq_key_at(const R_t& R, uint32_t q, uint32_t w, uint32_t p, uint32_t n) {
    constexpr uint32_t K = 16;  // strlen("_sequence_number")
    if (!(w == kSeqK0 || w == kSeqS1 || w == kSeqS2 || w == kSeqS3)) return false;
    const uint32_t j = w == kSeqK0 ? 0u : w == kSeqS1 ? 1u : w == kSeqS2 ? 2u : 3u;
    if (q < p + j || q - j + K > p + n) return false;
    const uint32_t st = q - j;
    return R.u32(st) == kSeqK0 && R.u32(st + 4) == kSeqK1 && R.u32(st + 8) == kSeqK2 && R.u32(st + 12) == kSeqK3;
}

// 0x80 in exactly the bytes of w equal to '\\' (no borrow noise: the escape flag is per byte)
__device__ __forceinline__ uint32_t bs_bytes_exact(uint32_t w) {
    const uint32_t x = w ^ 0x5c5c5c5cu;
    return ~(((x & 0x7f7f7f7fu) + 0x7f7f7f7fu) | x | 0x7f7f7f7fu);
}
// 0x80 in the bytes of the aligned dword at window/record offset A that lie inside [a0, a1)
__device__ __forceinline__ uint32_t range_bytes(uint32_t A, uint32_t a0, uint32_t a1) {
    const uint32_t lo = a0 > A ? min(a0 - A, 4u) : 0u, hi = a1 > A ? min(a1 - A, 4u) : 0u;
    const uint64_t m = ((1ull << (8 * hi)) - 1) & ~((1ull << (8 * lo)) - 1);
    return (uint32_t)m & 0x80808080u;
}

// SBE_FL_SEQ_KEY / SBE_FL_SEQ_ESC of the payload [p, p+n) of a record read from HBM: every dword
// overlapping the payload is read aligned (the first and last may reach outside it, never outside
// the 4-byte unit of a payload byte)
template <typename R_t>
__device__ uint32_t has_seq_key(const R_t& R, uint32_t p, uint32_t n) {
    if (n < 16) return 0u;
    uint32_t fl = 0;
    for (uint32_t q = p - R.abs_align(p); q < p + n; q += 4) {
        const uint32_t w = R.adw(q);
        if (bs_bytes_exact(w) & range_bytes(q, p, p + n)) fl |= SBE_FL_SEQ_ESC;
        if (q >= p && seq_key_at(R, q, w, p, n)) fl |= SBE_FL_SEQ_KEY;
    }
    return fl;
}

// Suspect bytes, accumulated branch-free over a lane's chunks (the decode kernel is issue-bound:
// every VALU / SALU instruction of the scan costs its slot, so the common no-hit case is pure
// VALU, no compares into masks, no per-chunk branch):
//   km = min over the dwords w of min(w ^ K0, w ^ S1, w ^ S2, w ^ S3): 0 iff some dword equals a
//        key slice (the candidates of seq_key_at);
//   bz |= (x - 0x01010101) & ~x with x = w ^ 0x5c5c5c5c: bit 7 of some byte set iff some byte is a
//        backslash (borrow noise only sits above a real zero byte, so it is exact as an any-test).
// Both are membership tests over the chunk's dwords.  A suspect lane then
// rescans its chunks with the exact per-dword tests (rare: real key slices or escapes).
struct Suspect {
    uint32_t km = ~0u, bz = 0u;
    __device__ __forceinline__ void add(uint4 v) {
        const uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            km = min(km, min(min(w[j] ^ kSeqK0, w[j] ^ kSeqS1), min(w[j] ^ kSeqS2, w[j] ^ kSeqS3)));
            const uint32_t x = w[j] ^ 0x5c5c5c5cu;
            bz |= (x - 0x01010101u) & ~x;
        }
    }
    __device__ __forceinline__ bool any() const { return km == 0u || (bz & 0x80808080u) != 0u; }
};

// 0 iff some dword of v equals one of the four key slices (the candidates of seq_key_at)
__device__ __forceinline__ uint32_t slice_dist(uint32_t w) {
    const uint32_t a = min(w ^ kSeqK0, w ^ kSeqS1), b = min(w ^ kSeqS2, w ^ kSeqS3);
    return min(a, b);
}
__device__ __forceinline__ bool has_slice(uint4 v) {
    return min(min(slice_dist(v.x), slice_dist(v.y)), min(slice_dist(v.z), slice_dist(v.w))) == 0u;
}

__device__ __forceinline__ uint32_t bs_any(uint32_t w) {  // 0x80 in some byte iff w holds a '\\' (plus noise above it)
    const uint32_t x = w ^ 0x5c5c5c5cu;
    return (x - 0x01010101u) & ~x;
}
__device__ __forceinline__ uint32_t q_bytes(uint32_t w) {  // 0x80 in each byte of w equal to 'q' (plus borrow noise above a hit)
    const uint32_t x = w ^ 0x71717171u;
    return (x - 0x01010101u) & ~x;
}

// Staged records: every key dword contains 'q' (key[3]), so a 16-byte chunk (one ds_read_b128) without a 'q'
// byte holds no candidate.  Only flagged chunks run the exact per-dword test.  Per lane: tiles of
// records up to kSeqLaneRec bytes, and the fallback of window_exact (two hits in one lane).
// SBE_SEQ_LANE_K: chunk reads in flight per step.  4, 6 and 8 measured no faster (config 3 decode
// 60.1 -> 61.1 / 63.2 / 72.0 us, profiles/r04_ab_seqlane_k.log): the other waves already hide the
// LDS latency; the scan costs instructions, not waits.
#ifndef SBE_SEQ_LANE_K
#define SBE_SEQ_LANE_K 2
#endif
__device__ uint32_t has_seq_key_lane(const LdsRec& R, uint32_t p, uint32_t n) {
    if (n < 16) return 0u;
    constexpr uint32_t K = SBE_SEQ_LANE_K;  // chunks whose LDS reads are in flight together
    const uint32_t a0 = R.base + p, a1 = a0 + n;  // window byte range
    const uint32_t c1 = (a1 + 15) >> 4;
    uint32_t fl = 0;
    for (uint32_t c = a0 >> 4; c < c1; c += K) {
        // a group's reads past the payload's last chunk re-read that chunk (clamped address, no
        // branch between the reads): a duplicate can only repeat a suspect, never hide one
        uint4 v[K];
#pragma unroll
        for (uint32_t k = 0; k < K; ++k) v[k] = lds_read_chunk_raw(R.win, min(c + k, c1 - 1));
        // any-tests (exact as "some byte matches": borrow noise only sits above a real match); the
        // exact per-dword tests below run only for a group that holds a 'q' forming a key slice,
        // or a backslash anywhere in its bytes (the range test there decides whether it is inside
        // the payload)
        uint32_t t = 0, b = 0;
#pragma unroll
        for (uint32_t k = 0; k < K; ++k) {
            t |= q_bytes(v[k].x) | q_bytes(v[k].y) | q_bytes(v[k].z) | q_bytes(v[k].w);
            b |= bs_any(v[k].x) | bs_any(v[k].y) | bs_any(v[k].z) | bs_any(v[k].w);
        }
        bool sus = (b & 0x80808080u) != 0u;
        if (t & 0x80808080u) {
#pragma unroll
            for (uint32_t k = 0; k < K; ++k) sus |= has_slice(v[k]);
        }
        if (sus) {
#pragma nounroll
            for (uint32_t k = 0; k < 4 * K; ++k) {
                const uint32_t A = 16 * c + 4 * k;  // window offset of an aligned dword
                if (A + 4 <= a0 || A >= a1) continue;
                const uint32_t w = lds_dw(R.win, A >> 2);
                if (bs_bytes_exact(w) & range_bytes(A, a0, a1)) fl |= SBE_FL_SEQ_ESC;
                if (A < a0 || A + 4 > a1) continue;
                const uint32_t q = A - R.base;
                if (seq_key_at(R, q, w, p, n)) fl |= SBE_FL_SEQ_KEY;
            }
        }
    }
    return fl;
}

// Staged records are not scanned while parsing.  Tiles of short records (all <= kSeqLaneRec bytes):
// each lane scans its own payload afterwards (has_seq_key_lane; payloads are a minority of the
// window's bytes and the lanes' loops are about equally long).  Tiles with longer records: dec_stage
// classifies every staged 16-byte chunk from its staging registers (Suspect, one bit per chunk of
// the lane; no LDS pass, no divergence between records of different lengths), and dec_window
// resolves the pending payloads from those bits: none set in the wave (the usual case) clears them
// all; else the flagged chunks alone get the exact tests (window_exact) and each lane looks its
// payload up in the hit list.
#ifndef SBE_SEQ_LANE_REC
#define SBE_SEQ_LANE_REC 320
#endif
constexpr uint32_t kSeqLaneRec = SBE_SEQ_LANE_REC;
// _sequence_number flag of a payload: SBE_FL_SEQ_KEY or 0; staged payloads return kFlSeqPending
constexpr uint32_t kFlSeqPending = 0x80u;
template <typename R_t>
__device__ __forceinline__ uint32_t seq_key_state(const R_t& R, uint32_t p, uint32_t n) {
    return has_seq_key(R, p, n);
}
template <>
__device__ __forceinline__ uint32_t seq_key_state<LdsRec>(const LdsRec&, uint32_t, uint32_t n) {
    return n >= 16 ? kFlSeqPending : 0u;
}

// Exact tests of the flagged chunks (bit k of sm: chunk lane + 64 k) of a staged window of nbytes:
// every backslash byte and every verified key start (16 bytes at that window offset, inside the
// window) is a hit.  Each lane keeps the position of its first hit in `hit` (~0u: none; kHitEsc
// marks a backslash) and sets `more` if it found a second one.
__device__ __forceinline__ uint32_t win_bytes4(const uint32_t* win, uint32_t s) {  // 4 bytes at window offset s
    const uint32_t lo = lds_dw(win, s >> 2), sh = s & 3u;
    return sh ? __builtin_amdgcn_alignbyte(lds_dw(win, (s >> 2) + 1), lo, sh) : lo;
}
constexpr uint32_t kHitEsc = 0x80000000u;  // hit kind bit: a '\\' byte (else a key start)
__device__ __noinline__ void window_exact(const uint32_t* win, uint32_t sm, uint32_t nbytes, int lane,
                                          uint32_t& hit, bool& more) {
    hit = ~0u;
    more = false;
    for (; sm; sm &= sm - 1) {
        const uint32_t c = (uint32_t)lane + kWave * (uint32_t)__builtin_ctz(sm);
#pragma nounroll
        for (uint32_t j = 0; j < 4; ++j) {
            const uint32_t A = 16 * c + 4 * j;
            const uint32_t w = lds_dw(win, A >> 2);
            for (uint32_t m = bs_bytes_exact(w) & range_bytes(A, 0, nbytes); m; m &= m - 1) {
                const uint32_t x = (A + (__builtin_ctz(m) >> 3)) | kHitEsc;
                if (hit == ~0u) hit = x;
                else more = true;
            }
            if (!(w == kSeqK0 || w == kSeqS1 || w == kSeqS2 || w == kSeqS3)) continue;
            const uint32_t off = w == kSeqK0 ? 0u : w == kSeqS1 ? 1u : w == kSeqS2 ? 2u : 3u;
            if (A < off || A - off + 16 > nbytes) continue;
            const uint32_t st = A - off;
            if (win_bytes4(win, st) == kSeqK0 && win_bytes4(win, st + 4) == kSeqK1 &&
                win_bytes4(win, st + 8) == kSeqK2 && win_bytes4(win, st + 12) == kSeqK3) {
                if (hit == ~0u) hit = st;
                else more = true;
            }
        }
    }
}

// decode_topic_message_with_sbe (src/sbe_encoder.cpp:957-1143); record bytes [b, b+len)
template <typename R_t>
__device__ void dec_tm_parse(const R_t& R, uint32_t b, uint32_t len, Desc& d) {
    const uint32_t h0 = R.u32(b), h1 = R.u32(b + 4);
    const uint32_t blk = h0 & 0xffffu, ver = h1 >> 16;
    // 32-bit bounds: pos <= len holds after every step, so len - pos never wraps
    uint32_t pos = 8u + blk;
    if (pos > len) { d.fail(SBE_ST_ERR_TM_E100, 0); return; }
    d.clear();
#pragma unroll
    for (int f = 0; f < 4; ++f) {
        if (len - pos < 2) { d.fail(SBE_ST_ERR_TM_E100, 0); return; }
        const uint32_t L = R.u16(b + pos);
        if (L > len - pos - 2) { d.fail(SBE_ST_ERR_TM_E100, 0); return; }
        d.off[f] = b + pos + 2;
        d.len[f] = L;
        pos += 2 + L;
    }
    d.status = SBE_ST_TM;
    d.hdr[0] = (uint16_t)blk;
    d.hdr[1] = 1;
    d.hdr[2] = 1;
    d.hdr[3] = (uint16_t)ver;
    d.ts = R.u64(b + 8);
    if (b) d.flags |= SBE_FL_WRAPPED;
    d.flags |= seq_key_state(R, d.off[3], d.len[3]);
    const uint32_t L4 = len - pos >= 2 ? (uint32_t)R.u16(b + pos) : 0u;
    if (len - pos < 2 || L4 > len - pos - 2) {
        d.flags |= SBE_FL_HEADERS_E100;
    } else {
        d.off[4] = b + pos + 2;
        d.len[4] = L4;
    }
}

// bit k set iff record byte p + k is printable ([32, 126]), for k < nbytes (<= 64): 17 aligned
// dword reads (clamped to the record's last dword), four bytes classified per dword (SWAR), the
// four flags gathered with one multiply
template <typename R_t>
__device__ __forceinline__ uint64_t printable_mask64(const R_t& R, uint32_t p, uint32_t nbytes) {
    const uint32_t sh = R.abs_align(p);
    const uint32_t q0 = p - sh;  // record offset of the aligned dword holding byte p
    const uint32_t kmax = (sh + nbytes - 1) >> 2;
    uint64_t m = 0;
    uint32_t extra = 0;
#pragma unroll
    for (uint32_t k = 0; k < 17; ++k) {
        const uint32_t w = R.adw(q0 + 4 * (k < kmax ? k : kmax));
        const uint32_t lo7 = w & 0x7f7f7f7fu;
        const uint32_t pr = (lo7 + 0x60606060u) & ~(lo7 + 0x01010101u) & ~w & 0x80808080u;
        const uint32_t c = __builtin_amdgcn_udot4(pr >> 7, 0x08040201u, 0u, false);  // the four flags as bits 0-3
        if (k < 16) m |= (uint64_t)c << (4 * k);
        else extra = c;
    }
    if (sh) m = (m >> sh) | ((uint64_t)extra << (64 - sh));
    return nbytes >= 64 ? m : m & ((1ull << nbytes) - 1);
}

// The same for a staged record: the (up to) five 16-byte chunks holding [p, p + nbytes) as
// ds_read_b128 (a chunk stays whole in its LDS slot), classified on 80 bytes and shifted into place
// (5 LDS reads instead of 17 swizzled dword reads)
__device__ __forceinline__ uint32_t printable4(uint32_t w) {  // bit k: byte k of w is printable
    const uint32_t lo7 = w & 0x7f7f7f7fu;
    const uint32_t pr = (lo7 + 0x60606060u) & ~(lo7 + 0x01010101u) & ~w & 0x80808080u;
    // the four byte flags (bits 7, 15, 23, 31) gathered as bits 0-3 by one v_dot4_u32_u8 (weights
    // 1, 2, 4, 8) instead of a quarter-rate multiply and two shifts
    return __builtin_amdgcn_udot4(pr >> 7, 0x08040201u, 0u, false);
}
template <>
__device__ __forceinline__ uint64_t printable_mask64<LdsRec>(const LdsRec& R, uint32_t p, uint32_t nbytes) {
    const uint32_t A = R.base + p;  // window offset of byte p
    const uint32_t c0 = A >> 4, s = A & 15u, clast = (A + nbytes - 1) >> 4;
    uint64_t lo = 0;
    uint32_t hi = 0;
#pragma unroll
    for (uint32_t j = 0; j < 5; ++j) {
        const uint4 v = lds_read_chunk_raw(R.win, c0 + j < clast ? c0 + j : clast);
        const uint32_t m16 = printable4(v.x) | (printable4(v.y) << 4) | (printable4(v.z) << 8) | (printable4(v.w) << 12);
        if (j < 4) lo |= (uint64_t)m16 << (16 * j);
        else hi = m16;
    }
    const uint64_t m = s ? (lo >> s) | ((uint64_t)hi << (64 - s)) : lo;
    return nbytes >= 64 ? m : m & ((1ull << nbytes) - 1);
}

#ifndef SBE_ACK_FAST
#define SBE_ACK_FAST 1
#endif
// decode_acknowledgment_with_sbe (src/sbe_encoder.cpp:833-954)
template <typename R_t>
__device__ void dec_ack_heuristic(const R_t& R, uint32_t b, uint32_t len, Desc& d) {
    if (len < 16) { d.fail(SBE_ST_ERR_ACK_SHORT, (uint32_t)len); return; }
    d.clear();
    d.set_hdr(R, b);
    d.status = SBE_ST_ACK;
    d.ts = R.u64(b + 8);
    if (b) d.flags |= SBE_FL_WRAPPED;
    // Fast path (the common, well-formed Ack: u16-length-prefixed messageId, topic, correlationId
    // from byte 16, src/ack_decoder.cpp's layout): when every field byte is printable, every length
    // byte is not, each field is >= 3 bytes and the byte after the third field is not printable (or
    // is past the record), the first three maximal runs of the scan below are exactly the three
    // fields.  One 64-byte printable mask checks that for fields ending by byte 79; anything else
    // takes the general run scan.
    uint32_t nruns = 0;
#if SBE_ACK_FAST
    if (len >= 22) {
        const uint32_t L1 = R.u16(b + 16);
        const uint32_t p2 = 18 + L1;
        const uint32_t L2 = p2 + 2 <= len ? R.u16(b + p2) : 0u;
        const uint32_t p3 = p2 + 2 + L2;
        const uint32_t L3 = p3 + 2 <= len ? R.u16(b + p3) : 0u;
        const uint32_t end3 = p3 + 2 + L3;  // record offset after the third field
        const uint32_t span = (end3 < len ? end3 + 1 : end3) - 16;  // bytes [16, 16 + span) decide
        if (L1 >= 3 && L2 >= 3 && L3 >= 3 && end3 <= len && span <= 64) {
            const uint64_t m = printable_mask64(R, b + 16, span);
            auto ones = [](uint32_t n) { return n >= 64 ? ~0ull : (1ull << n) - 1; };
            // field bits: [2, 2 + L1), [4 + L1, 4 + L1 + L2), [6 + L1 + L2, 6 + L1 + L2 + L3) of the span
            const uint64_t want = (ones(L1) << 2) | (ones(L2) << (4 + L1)) | (ones(L3) << (6 + L1 + L2));
            if ((m & ones(span)) == want) {
                d.set_view(0, b + 18, L1);
                d.set_view(1, b + p2 + 2, L2);
                d.set_view(2, b + p3 + 2, L3);
                return;
            }
        }
    }
#endif
    // maximal runs of printable bytes over [16, len), 64 bytes per block as a bitmask; a run may
    // continue into the next block
    uint64_t run_start = 0, run_len = 0;
    for (uint32_t s0 = 16; s0 < len && nruns < 3; s0 += 64) {
        const uint32_t nb = len - s0 < 64u ? len - s0 : 64u;
        const uint64_t m = printable_mask64(R, b + s0, nb);
        uint32_t pos = 0;
        while (pos < nb && nruns < 3) {
            if (run_len == 0) {
                const uint64_t rest = m >> pos;
                if (rest == 0) break;  // nothing printable left in this block
                pos += (uint32_t)__builtin_ctzll(rest);
                run_start = s0 + pos;
            }
            const uint64_t zeros = ~(m >> pos);  // bits >= nb of m are clear: a run stops at nb
            const uint32_t o = zeros ? (uint32_t)__builtin_ctzll(zeros) : 64u - pos;
            const uint32_t take = o < nb - pos ? o : nb - pos;
            run_len += take;
            pos += take;
            if (pos < nb) {  // ended at a non-printable byte inside the block
                if (run_len >= 3) {
                    d.set_view(nruns, (uint32_t)(b + run_start), (uint32_t)run_len);
                    ++nruns;
                }
                run_len = 0;
            }
        }
    }
    if (nruns < 3 && run_len >= 3) {
        d.set_view(nruns, (uint32_t)(b + run_start), (uint32_t)run_len);
        ++nruns;
    }
    if (nruns < 1) d.flags |= SBE_FL_ID_DEFAULT;
    if (nruns < 2) d.flags |= SBE_FL_PAYLOAD_DEFAULT;
}

// parse_session_event / decode_session_event (src/sbe_encoder.cpp:618-647, :183-238, :285-318)
template <typename R_t>
__device__ void dec_session_event(const R_t& R, uint32_t len, Desc& d) {
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
template <typename R_t>
__device__ void dec_parse_message(const R_t& R, uint32_t len, Desc& d) {
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
template <typename R_t>
__device__ void dec_on_egress(const R_t& R, uint32_t len, Desc& d) {
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
#pragma unroll
        for (int f = 0; f < 3; ++f) {
            if (!ok) continue;
            const uint64_t L = R.u16(pos);
            if (L > 0) {
                if (pos + 2 + L > lim) {
                    ok = false;
                    continue;
                }
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

// The Lite templates' generated decode flyweights in field order (CommitOffsetLite.h:240-276,
// :337-420, :528-540; OrderRequestLite.h / OrderNotificationLite.h likewise): wrapForDecode(buf,
// 8, blockLength, version, len), topicId @8, sequence @12, getXAsString per var field (E100 past
// len).  The 12 fixed bytes must lie inside the record (the flyweight reads them unchecked).
template <typename R_t>
__device__ void dec_lite(const R_t& R, uint32_t len, Desc& d) {
    d.clear();
    if (len < 8) { d.status = SBE_ST_LITE_NOT_LITE; return; }
    const uint32_t h0 = R.u32(0), h1 = R.u32(4);
    const uint32_t blk = h0 & 0xffffu, tmpl = h0 >> 16, schema = h1 & 0xffffu;
    d.set_hdr(R, 0);
    const uint32_t nf = tmpl == SBE_COMMIT_OFFSET_LITE_TEMPLATE_ID ? 2u
                      : (tmpl == SBE_ORDER_REQUEST_LITE_TEMPLATE_ID || tmpl == SBE_ORDER_NOTIFICATION_LITE_TEMPLATE_ID) ? 3u
                                                                                                                   : 0u;
    if (schema != 1 || nf == 0) { d.status = SBE_ST_LITE_NOT_LITE; return; }
    uint32_t pos = 8u + blk;
    if (pos > len || len < 20) { d.status = SBE_ST_LITE_E100; return; }
#pragma unroll
    for (uint32_t f = 0; f < 3; ++f) {
        if (f >= nf) break;
        if (pos + 2 > len) {
#pragma unroll
            for (int k = 0; k < 5; ++k) d.off[k] = d.len[k] = 0;
            d.status = SBE_ST_LITE_E100;
            return;
        }
        const uint32_t L = R.u16(pos);
        pos += 2;
        if (pos + L > len) {
#pragma unroll
            for (int k = 0; k < 5; ++k) d.off[k] = d.len[k] = 0;
            d.status = SBE_ST_LITE_E100;
            return;
        }
        d.off[f] = pos;
        d.len[f] = L;
        pos += L;
    }
    d.status = SBE_ST_LITE;
    d.ts = R.u64(12);
    d.off[4] = R.u32(8);
}

template <uint32_t kW>
constexpr int dec_regs() {  // uint4 staging registers per lane (one window)
    static_assert(kW % (16 * kWave) == 0, "decode windows are whole 1 KiB staging rows");
    return (int)(kW / 16 / kWave);
}


template <uint32_t kMode, typename R_t>
__device__ __forceinline__ void dec_record(const R_t& R, uint32_t len, Desc& d) {
    if (kMode == SBE_DEC_ON_EGRESS)
        dec_on_egress(R, len, d);
    else if (kMode == SBE_DEC_LITE)
        dec_lite(R, len, d);
    else
        dec_parse_message(R, len, d);
}

// a record parsed straight from HBM (rare: see sbe_decode_kernel); not inlined, so its register
// needs stay out of the window loop's
template <uint32_t kMode>
__device__ __noinline__ Desc dec_record_glb(const uint8_t* in, uint64_t rs, uint32_t rl) {
    Desc d;
    d.clear();
    dec_record<kMode>(GlbRec{reinterpret_cast<uintptr_t>(in) + rs}, rl, d);
    return d;
}

// Stage window [wb, we) (16-B aligned, <= kWin bytes) into LDS: every 16-B load issued before
// the first LDS write, one HBM round trip per window.  Parse mode: returns the lane's Suspect bits
// (bit k: chunk lane + 64 k holds a key-slice dword or a backslash byte), classified from the
// staging registers (tiles with records over kSeqLaneRec bytes: `wide`), so the "_sequence_number"
// scan needs no LDS pass of its own.
// The decode's staging loads are nontemporal (the records are read once): against the default cache
// policy, rotated inputs, fixed-256 55.4 / 57.2 us, config 3 58.5 / 59.6, session frames 63.4 /
// 65.6, OrderRequestLite 66.5 / 71.0; one set re-read, fixed-256 56.3 / 58.4, config 4 410.9 / 430.9
// (profiles/r06_ab_decntl_{rot,warm}.log)
#ifndef SBE_DEC_NTL  // A/B builds: 0 = the decode's staging loads with the default cache policy
#define SBE_DEC_NTL 1
#endif
template <uint32_t kW>
__device__ __forceinline__ void dec_issue(const DecArgs& a, uint64_t wb, uint64_t we, int lane,
                                          uint4 (&I)[dec_regs<kW>()]) {
    const uint32_t nch = (uint32_t)((we - wb) >> 4);
    const uintptr_t src = reinterpret_cast<uintptr_t>(a.in) + wb;
#pragma unroll
    for (int k = 0; k < dec_regs<kW>(); ++k) {
        const uint32_t ch = lane + kWave * k;
        I[k] = ch < nch ? (SBE_DEC_NTL ? gload128_nt(src + 16ull * ch) : gload128(src + 16ull * ch))
                        : make_uint4(0, 0, 0, 0);
    }
}

template <uint32_t kMode, uint32_t kW>
__device__ __forceinline__ uint32_t dec_commit(uint32_t* win, uint64_t wb, uint64_t we, bool wide, int lane,
                                               const uint4 (&I)[dec_regs<kW>()]) {
    const uint32_t nch = (uint32_t)((we - wb) >> 4);
#pragma unroll
    for (int k = 0; k < dec_regs<kW>(); ++k) {
        const uint32_t ch = lane + kWave * k;
        if (ch < nch) lds_write_chunk(win, ch, I[k]);
    }
    uint32_t sm = 0;
#ifdef SBE_ABL_NOCLASS  // ablation builds only (wrong flags on payloads with a key or a backslash)
    if (false) {
#else
    if (kMode == SBE_DEC_PARSE_MESSAGE && wide) {
#endif
        // rows of chunks past the window are skipped (a tile's later window is often part full);
        // zero chunks of the last row are never suspect
        const uint32_t nrow = (nch + kWave - 1) / kWave;
#pragma unroll
        for (int k = 0; k < dec_regs<kW>(); ++k) {
            if ((uint32_t)k < nrow) {
                // (the key-slice compares as wave masks, v_cmp + s_or_b64 per dword instead of
                // xors and v_min3, read config 4 decode 407.0 -> 439.6 us: the scalar ors issue
                // from the same wave, profiles/r06_ab_cmp.log)
                Suspect S;
                S.add(I[k]);
                sm |= S.any() ? 1u << k : 0u;
            }
        }
    }
    return sm;
}

template <uint32_t kMode, uint32_t kW>
__device__ __forceinline__ uint32_t dec_stage(const DecArgs& a, uint32_t* win, uint64_t wb, uint64_t we, bool wide,
                                              int lane) {
    uint4 I[dec_regs<kW>()];
    dec_issue<kW>(a, wb, we, lane, I);
    return dec_commit<kMode, kW>(win, wb, we, wide, lane, I);
}

// One workgroup (one wave) per 64-record tile.  The tile's bytes are staged window by window:
// the first window starts at the tile's first byte, each later one at the first record not yet
// parsed; every lane parses its record from LDS in the window that holds it whole.  A record
// that no window can hold (larger than the window, or outside the tile's byte range when
// rec_off is not monotonic) is parsed from HBM.  Fixed 256-B records take one window per tile.
// The workgroup is one wave, whose LDS accesses execute in issue order: phase changes are
// compiler barriers.
// 3 waves per SIMD (<= 168 VGPRs): with 16 KiB of LDS per workgroup the CU holds 10 workgroups,
// which 3 waves/SIMD still allow.
// Parse the records that lie whole in the staged window [wb, we); in parse mode, then resolve the
// _sequence_number flags left pending from the window's Suspect bits sm (dec_stage).
template <uint32_t kMode>
__device__ __forceinline__ void dec_window(const uint32_t* win, uint64_t wb, uint64_t we, uint64_t rs, uint64_t rl,
                                           bool wide, uint32_t sm, bool& done, Desc& d, int lane) {
    bool here = false;
    if (!done && rs >= wb && rs + rl <= we) {
        dec_record<kMode>(LdsRec{win, (uint32_t)(rs - wb)}, (uint32_t)rl, d);
        done = true;
        here = true;
    }
    if (kMode == SBE_DEC_PARSE_MESSAGE) {
        const bool pend = here && (d.flags & kFlSeqPending);
        if (!wide) {
#ifdef SBE_TIMING_NOSEQ  // timing builds only (scripts/serve_probe.cpp): the per-lane scan skipped
            if (pend) d.flags &= ~kFlSeqPending;
#else
            if (pend)
                d.flags = (d.flags & ~kFlSeqPending) | has_seq_key_lane(LdsRec{win, (uint32_t)(rs - wb)}, d.off[3], d.len[3]);
#endif
        } else if (__ballot(pend)) {
            uint32_t hit = 0;
            if (__ballot(sm != 0)) {  // some staged chunk holds a key slice or a backslash
                uint32_t hpos;
                bool more;
                window_exact(win, sm, (uint32_t)(we - wb), lane, hpos, more);
                const uint32_t p0 = (uint32_t)(rs - wb) + d.off[3], p1 = p0 + d.len[3];
                if (__ballot(more)) {  // two hits among one lane's chunks: pending lanes scan themselves
                    if (pend) hit = has_seq_key_lane(LdsRec{win, (uint32_t)(rs - wb)}, d.off[3], d.len[3]);
                } else {
                    for (uint64_t m = __ballot(hpos != ~0u); m; m &= m - 1) {  // broadcast each hit
                        const uint32_t x = __builtin_amdgcn_readlane(hpos, __builtin_ctzll(m));
                        const uint32_t xa = x & ~kHitEsc;
                        if (x & kHitEsc) hit |= xa >= p0 && xa < p1 ? SBE_FL_SEQ_ESC : 0u;
                        else hit |= x >= p0 && x + 16 <= p1 ? SBE_FL_SEQ_KEY : 0u;
                    }
                }
            }
            if (pend) d.flags = (d.flags & ~kFlSeqPending) | hit;
        }
    }
}

#ifndef SBE_DEC_MINW
#define SBE_DEC_MINW 3
#endif
// One 64-record tile (the decode kernel: tile = blockIdx.x; the serve kernel: tile 0 of a one-tile
// batch); win is the workgroup's LDS window of kWin bytes.
#ifdef SBE_SERVE_PROF
__device__ uint64_t g_serve_prof[16];
#define SBE_SVP(k, t) tpk[(k) - 5] = __builtin_amdgcn_s_memrealtime()
#else
#define SBE_SVP(k, t) do { } while (0)
#endif
// The windows after a tile's first one (which is parsed): the second window's loads go out first
// when its start is known; then windows from the first record still to parse; records no window
// can hold are parsed from HBM.  I: free staging registers.
template <uint32_t kMode, uint32_t kWin>
__device__ __forceinline__ void dec_rest(const DecArgs& a, uint32_t* win, uint64_t T0, uint64_t end, uint64_t rs,
                                         uint64_t rl, bool wide, bool& done, Desc& d, int lane,
                                         uint4 (&I)[dec_regs<kWin>()]) {
    for (;;) {
        bool again = false;
        uint64_t wb = 0;
        for (;;) {
            const uint64_t m = __ballot(!done);
            if (m == 0) break;
            const int f = __builtin_ctzll(m);
            const uint64_t rsf = uniform64(__shfl(rs, f, kWave));
            const uint64_t rlf = uniform64(__shfl(rl, f, kWave));
            if ((rsf & 15) + rlf <= kWin && rsf + rlf <= end && rsf >= (T0 & ~15ull)) {
                wb = rsf & ~15ull;
                again = true;
                break;
            }
            if (lane == f) {
                d = dec_record_glb<kMode>(a.in, rs, (uint32_t)rl);
                done = true;
            }
        }
        if (!again) break;
        const uint64_t we = wb + kWin < end ? wb + kWin : end;
        wsync();
        dec_issue<kWin>(a, wb, we, lane, I);
        const uint32_t sm = dec_commit<kMode, kWin>(win, wb, we, wide, lane, I);
        wsync();
        dec_window<kMode>(win, wb, we, rs, rl, wide, sm, done, d, lane);
    }
}

// The descriptor SoA of record r, and ParseResult.sequence_number of flagged TopicMessages (rare:
// payloads with the key or a backslash), evaluated from HBM by the lanes that hold one.
template <uint32_t kMode, bool kServe>
__device__ __forceinline__ void dec_outputs(const DecArgs& a, uint64_t r, bool valid, uint64_t rs, const Desc& d) {
    if (valid) {
        dst_store(a.status + r, (uint8_t)d.status);
        dst_store(a.flags + r, (uint8_t)d.flags);
        dst_store(reinterpret_cast<uint64_t*>(a.hdr + 4 * r),
                  (uint64_t)((uint32_t)d.hdr[0] | ((uint32_t)d.hdr[1] << 16)) |
                      ((uint64_t)((uint32_t)d.hdr[2] | ((uint32_t)d.hdr[3] << 16)) << 32));
        dst_store(a.ts + r, d.ts);
    }
    // views [n][5]: each lane stores its record's 20 contiguous bytes per array (a dwordx4 and a
    // dword; the wave's stores cover 1280 contiguous bytes), no LDS transpose
    if (valid) {
        typedef uint32_t u32x4a4 __attribute__((ext_vector_type(4), aligned(4)));
        u32x4a4 o4, l4;
        o4.x = d.off[0]; o4.y = d.off[1]; o4.z = d.off[2]; o4.w = d.off[3];
        l4.x = d.len[0]; l4.y = d.len[1]; l4.z = d.len[2]; l4.w = d.len[3];
        __builtin_nontemporal_store(o4, reinterpret_cast<u32x4a4*>(a.view_off + 5 * r));
        __builtin_nontemporal_store(d.off[4], a.view_off + 5 * r + 4);
        __builtin_nontemporal_store(l4, reinterpret_cast<u32x4a4*>(a.view_len + 5 * r));
        __builtin_nontemporal_store(d.len[4], a.view_len + 5 * r + 4);
    }
    if (kMode == SBE_DEC_PARSE_MESSAGE && a.seq) {
        const bool cand = valid && d.status == SBE_ST_TM && (d.flags & kSeqCand);
        if (__ballot(cand) && cand)
            a.seq[r] = kServe ? json_seq_eval_call_serve(a.in + rs + d.off[3], d.len[3])
                              : json_seq_eval_call(a.in + rs + d.off[3], d.len[3]);
    }
}

// A record beyond 32-bit sizes is not an SBE frame we bound-check
template <uint32_t kMode>
__device__ __forceinline__ void dec_oversize(Desc& d) {
    d.status = kMode == SBE_DEC_ON_EGRESS ? SBE_ST_EG_NONE
             : kMode == SBE_DEC_LITE    ? SBE_ST_LITE_E100
                                        : SBE_ST_ERR_TM_E100;
}

template <uint32_t kMode, uint32_t kWin, bool kServe = false>
__device__ __forceinline__ void dec_tile(const DecArgs& a, uint64_t tile, uint32_t* win) {
#ifdef SBE_SERVE_PROF
    const uint64_t tp0 = __builtin_amdgcn_s_memrealtime();
    uint64_t tpk[4] = {tp0, tp0, tp0, tp0};
#endif
    const int lane = threadIdx.x & (kWave - 1);
    const uint64_t t0 = tile * kTile;
    const uint64_t r = t0 + (uint64_t)lane;
    const bool valid = r < a.n;
    const uint64_t last = t0 + kTile < a.n ? t0 + kTile : a.n;
    const uint64_t T0 = uniform64(a.rec_off[t0]);
    const uint64_t end = (uniform64(a.rec_off[last]) + 15) & ~15ull;
    const uint64_t rc = r < a.n ? r : a.n - 1;
    const uint64_t rs = a.rec_off[rc];
    const uint64_t rl = valid ? a.rec_off[rc + 1] - rs : 0;

    Desc d;
    d.clear();
    bool done = !valid;
    if (valid && rl > 0xffffffffull) {
        dec_oversize<kMode>(d);
        done = true;
    }
    // first window: the whole tile when its records are at most 256 B on average
    uint64_t wb = T0 & ~15ull;
    uint64_t we = wb + kWin < end ? wb + kWin : (end > wb ? end : wb);
    // the served path classifies the staged chunks in parallel (one chunk a lane for a small
    // batch) instead of a per-lane payload scan, whose dependent steps a lone wave cannot hide
    // (1.4 µs of a one-record request, profiles/r04_serve_probe.log)
    const bool wide = kServe || __ballot(valid && rl > kSeqLaneRec) != 0;
    uint4 I[dec_regs<kWin>()];
    SBE_SVP(5, tp0);  // offsets read
    dec_issue<kWin>(a, wb, we, lane, I);
    uint32_t sm = dec_commit<kMode, kWin>(win, wb, we, wide, lane, I);
    SBE_SVP(6, tp0);  // first window in LDS
    // The second window starts at the first record the first one cannot hold, which the record
    // offsets already tell: its loads go out before the first window is parsed (tiles of records
    // over 256 B on average take two windows; each would otherwise wait one more HBM round trip).
    bool pre = false;
    uint64_t wb2 = 0, we2 = 0;
    {
        const uint64_t m = __ballot(!(done || (rs >= wb && rs + rl <= we)));
        if (m) {
            const int f = __builtin_ctzll(m);
            const uint64_t rsf = uniform64(__shfl(rs, f, kWave));
            const uint64_t rlf = uniform64(__shfl(rl, f, kWave));
            if ((rsf & 15) + rlf <= kWin && rsf + rlf <= end && rsf >= (T0 & ~15ull)) {
                wb2 = rsf & ~15ull;
                we2 = wb2 + kWin < end ? wb2 + kWin : end;
                pre = true;
                dec_issue<kWin>(a, wb2, we2, lane, I);
            }
        }
    }
    wsync();
    dec_window<kMode>(win, wb, we, rs, rl, wide, sm, done, d, lane);
    if (pre) {
        wsync();
        sm = dec_commit<kMode, kWin>(win, wb2, we2, wide, lane, I);
        wsync();
        dec_window<kMode>(win, wb2, we2, rs, rl, wide, sm, done, d, lane);
    }
    if (__ballot(!done)) dec_rest<kMode, kWin>(a, win, T0, end, rs, rl, wide, done, d, lane, I);
    SBE_SVP(7, tp0);  // parsed
    dec_outputs<kMode, kServe>(a, r, valid, rs, d);
    SBE_SVP(8, tp0);  // descriptor stores issued
#ifdef SBE_SERVE_PROF
    if (kServe && lane == 0)
        for (int k = 0; k < 4; ++k) g_serve_prof[5 + k] += tpk[k] - tp0;
#endif
}

#ifndef SBE_DEC_MINW_WIDE  // A/B builds: waves per SIMD the kWinWide kernel is compiled for
#define SBE_DEC_MINW_WIDE SBE_DEC_MINW
#endif
template <uint32_t kMode, uint32_t kWin>
// the 20 KiB window's LDS allows 8 workgroups per CU, 2 waves per SIMD: its registers are sized for that
__global__ __launch_bounds__(kWave, kWin == kWinWide && kWinWide > 16384 ? 2 : ((kWin == kWinWide || kWin == kWinLarge) ? SBE_DEC_MINW_WIDE : SBE_DEC_MINW)) void sbe_decode_kernel(DecArgs a) {
    __shared__ uint32_t win[kWin / 4];
    dec_tile<kMode, kWin>(a, blockIdx.x, win);
}

// Decode of mixed batches with waves specialised by record kind (verdict r5 item 3).  In a tile of
// config 3's mix (69 % TopicMessages, 30 % Acks) a wave runs both parse paths one after the other:
// the TopicMessage lanes' payload scan with the Ack lanes idle, then the Ack lanes' printable-run
// scan with the TopicMessage lanes idle.  A workgroup of kG waves stages the kG tiles' bytes into
// one shared window, counts the TopicMessages and the Acks, and deals the records to the waves by
// kind (TopicMessages first, in record order, then Acks): at most one wave of the group holds
// both kinds.  Each lane parses its record from the shared window, and the descriptors go back to
// record order through LDS before the stores, so each wave stores contiguous rows.  A record that
// does not lie in the window (the group's bytes past kGW, or rec_off not increasing) is parsed
// from HBM by its lane (dec_record_glb), as the one-wave kernel does with a record no window can
// hold.  (A fallback to the one-wave path inside this kernel gave the parse functions a second
// call site, so the compiler outlined them and passed each descriptor through scratch: 30 scratch
// stores a wave, twice the decode time.)
// The workgroups are persistent (occupancy x CUs) and take groups g, g + G, ...; the next group's
// bytes are loaded into registers while the current one is parsed, and the offsets of the one
// after it a step earlier still, so a group's two dependent HBM round trips (offsets, then bytes)
// hide behind the previous group's work.  Every load of the loop is issued unconditionally (at a
// clamped group index on the last step), so the compiler's waits count them exactly.
struct GroupOffs {
    uint64_t g0, wb, we;  // first record; staged window [wb, we) (uniform)
    uint64_t rs, rl;      // this thread's record
    bool valid;
};
template <uint32_t kT, uint32_t kGW>
__device__ __forceinline__ GroupOffs group_offs(const DecArgs& a, uint64_t g, uint32_t tid) {
    GroupOffs o;
    o.g0 = g * kT;
    const uint64_t r = o.g0 + tid;
    o.valid = r < a.n;
    const uint64_t last = o.g0 + kT < a.n ? o.g0 + kT : a.n;
    const uint64_t T0 = uniform64(a.rec_off[o.g0]);
    const uint64_t end = (uniform64(a.rec_off[last]) + 15) & ~15ull;
    o.wb = T0 & ~15ull;
    o.we = end <= o.wb ? o.wb : (end - o.wb <= kGW ? end : o.wb + kGW);
    const uint64_t rc = o.valid ? r : a.n - 1;
    o.rs = a.rec_off[rc];
    o.rl = a.rec_off[rc + 1] - o.rs;
    return o;
}
template <uint32_t kT, uint32_t kPerThr>
__device__ __forceinline__ void group_issue(const DecArgs& a, const GroupOffs& o, uint32_t tid, uint4 (&I)[kPerThr]) {
    const uint32_t nch = (uint32_t)((o.we - o.wb) >> 4);
    const uintptr_t src = reinterpret_cast<uintptr_t>(a.in) + o.wb;
#pragma unroll
    for (uint32_t k = 0; k < kPerThr; ++k) {
        const uint32_t ch = tid + kT * k;
        I[k] = ch < nch ? gload128_nt(src + 16ull * ch) : make_uint4(0, 0, 0, 0);
    }
}

template <uint32_t kMode, uint32_t kG, uint32_t kGW>
__device__ __forceinline__ void dec_group(const DecArgs& a, uint32_t* win) {
    constexpr uint32_t kT = kG * kWave;  // records of the group
    constexpr uint32_t kPerThr = kGW / 16 / kT;  // staged chunks per thread
    static_assert(kGW % (16 * kT) == 0, "group window shape");
    __shared__ uint32_t rsA[kT], rlA[kT];
    __shared__ uint16_t slot_rec[kT];
    __shared__ uint32_t kcount[2 * kG];
    const uint32_t tid = threadIdx.x, w = tid / kWave, lane = tid & (kWave - 1);
    const uint64_t ngroups = (a.n + kT - 1) / kT, G = gridDim.x;
    uint64_t g = blockIdx.x;
    if (g >= ngroups) return;
    auto clampg = [&](uint64_t x) { return x < ngroups ? x : ngroups - 1; };
    GroupOffs o = group_offs<kT, kGW>(a, g, tid);
    uint4 I[kPerThr];
    group_issue<kT, kPerThr>(a, o, tid, I);
    GroupOffs on = group_offs<kT, kGW>(a, clampg(g + G), tid);
    for (;;) {
        const bool has_next = g + G < ngroups;  // uniform
        const uint64_t r = o.g0 + tid;
        const bool inw = o.valid && o.rs >= o.wb && o.rs + o.rl <= o.we;  // parsed from the window
        {
            const uint32_t nch = (uint32_t)((o.we - o.wb) >> 4);
#pragma unroll
            for (uint32_t k = 0; k < kPerThr; ++k) {
                const uint32_t ch = tid + kT * k;
                if (ch < nch) lds_write_chunk(win, ch, I[k]);
            }
        }
        rsA[tid] = inw ? (uint32_t)(o.rs - o.wb) : ~0u;
        rlA[tid] = (uint32_t)(o.rl < 0xffffffffull ? o.rl : 0xffffffffull);
        __syncthreads();
        // the next group's bytes and the offsets of the one after it, in flight from here on
        group_issue<kT, kPerThr>(a, on, tid, I);
        const GroupOffs onn = group_offs<kT, kGW>(a, clampg(g + 2 * G), tid);
        // kind of the record: an Ack (template 2, schema 1: the printable-run path) or anything else
        uint32_t ack = 0;
        if (inw && o.rl >= 8) {
            const LdsRec R{win, (uint32_t)(o.rs - o.wb)};
            const uint32_t h0 = R.u32(0), h1 = R.u32(4);
            ack = (h0 >> 16) == 2u && (h1 & 0xffffu) == 1u;
        }
        const uint64_t below = (1ull << lane) - 1ull;
        const uint64_t bt = __ballot(o.valid && !ack), ba = __ballot(o.valid && ack);
        if (lane == 0) {
            kcount[w] = (uint32_t)__builtin_popcountll(bt);
            kcount[kG + w] = (uint32_t)__builtin_popcountll(ba);
        }
        __syncthreads();
        uint32_t ntm = 0, pre_t = 0, pre_a = 0, nval = 0;
#pragma unroll
        for (uint32_t k = 0; k < kG; ++k) {
            ntm += kcount[k];
            nval += kcount[k] + kcount[kG + k];
            pre_t += k < w ? kcount[k] : 0u;
            pre_a += k < w ? kcount[kG + k] : 0u;
        }
        // invalid threads (the batch's last group) keep their own index, past the valid ones
        const uint32_t slot = !o.valid ? tid
                            : ack      ? ntm + pre_a + (uint32_t)__builtin_popcountll(ba & below)
                                       : pre_t + (uint32_t)__builtin_popcountll(bt & below);
        slot_rec[slot] = (uint16_t)tid;
        __syncthreads();
        // this lane's record: the tid-th of the dealt order
        const uint32_t j = slot_rec[tid];
        const bool jv = tid < nval;
        Desc d;
        d.clear();
        const uint32_t jb = rsA[j], jl = rlA[j];
        if (jv) {
            if (jb != ~0u) {
                dec_record<kMode>(LdsRec{win, jb}, jl, d);
                if (kMode == SBE_DEC_PARSE_MESSAGE && (d.flags & kFlSeqPending))
                    d.flags = (d.flags & ~kFlSeqPending) | has_seq_key_lane(LdsRec{win, jb}, d.off[3], d.len[3]);
            } else {  // not in the window: from HBM
                const uint64_t rj = o.g0 + j, sj = a.rec_off[rj], lj = a.rec_off[rj + 1] - sj;
                if (lj > 0xffffffffull) dec_oversize<kMode>(d);
                else d = dec_record_glb<kMode>(a.in, sj, (uint32_t)lj);
            }
        }
        // the descriptors back in record order through LDS (the window is free once every lane
        // has parsed), so each wave's stores cover contiguous rows as in the one-wave kernel
        constexpr uint32_t kDs = 17;  // dwords per staged descriptor (odd: no bank conflicts)
        static_assert(kDs * kT * 4 <= kGW, "descriptor staging fits the window");
        __syncthreads();
        if (jv) {
            uint32_t* q = win + kDs * j;
            q[0] = d.status | (d.flags << 8);
            q[1] = (uint32_t)d.hdr[0] | ((uint32_t)d.hdr[1] << 16);
            q[2] = (uint32_t)d.hdr[2] | ((uint32_t)d.hdr[3] << 16);
            q[3] = (uint32_t)d.ts;
            q[4] = (uint32_t)(d.ts >> 32);
#pragma unroll
            for (int k = 0; k < 5; ++k) {
                q[5 + k] = d.off[k];
                q[10 + k] = d.len[k];
            }
        }
        __syncthreads();
        Desc e;
        e.clear();
        if (o.valid) {
            const uint32_t* q = win + kDs * tid;
            e.status = q[0] & 0xffu;
            e.flags = q[0] >> 8;
            e.hdr[0] = (uint16_t)q[1];
            e.hdr[1] = (uint16_t)(q[1] >> 16);
            e.hdr[2] = (uint16_t)q[2];
            e.hdr[3] = (uint16_t)(q[2] >> 16);
            e.ts = (uint64_t)q[3] | ((uint64_t)q[4] << 32);
#pragma unroll
            for (int k = 0; k < 5; ++k) {
                e.off[k] = q[5 + k];
                e.len[k] = q[10 + k];
            }
        }
        dec_outputs<kMode, false>(a, r, o.valid, o.rs, e);
        if (!has_next) break;
        __syncthreads();  // every thread is past its descriptor read before the window is rewritten
        g += G;
        o = on;
        on = onn;
    }
}

#ifndef SBE_DEC_GROUP  // A/B builds: tiles per workgroup of the group decode kernel (0: the one-wave mid kernel)
#define SBE_DEC_GROUP 0
#endif
constexpr uint32_t kDecG = SBE_DEC_GROUP > 0 ? SBE_DEC_GROUP : 1;
template <uint32_t kMode>
__global__ __launch_bounds__(kDecG * kWave, kDecG >= 3 ? 2 : 3) void sbe_decode_group_kernel(DecArgs a) {
    __shared__ uint32_t win[kDecG * kWinMid / 4];
    dec_group<kMode, kDecG, kDecG * kWinMid>(a, win);
}

thread_local char g_last_error[256] = "";

int record_hip(hipError_t e) {
    if (e == hipSuccess) return SBE_OK;
    std::strncpy(g_last_error, hipGetErrorString(e), sizeof(g_last_error) - 1);
    return SBE_EHIP;
}

constexpr uint64_t kMaxTiles = 0xffffffffull;

// Persistent grid of the pack kernel: every workgroup resident at once (occupancy x CUs).
uint64_t pack_grid(const void* kernel, uint64_t tiles) {
    struct Entry {
        const void* k;
        int dev;
        uint64_t g;
    };
    static thread_local Entry cache[32] = {};
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess) dev = 0;
    uint64_t g = 0;
    for (const Entry& e : cache)
        if (e.k == kernel && e.dev == dev) g = e.g;
    if (g == 0) {
        int per_cu = 0, cus = 0;
        if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, kernel, kWave, 0) != hipSuccess || per_cu < 1)
            per_cu = 1;
        if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus < 1)
            cus = 256;
        g = (uint64_t)per_cu * (uint64_t)cus;
        for (Entry& e : cache)
            if (e.k == nullptr) {
                e = Entry{kernel, dev, g};
                break;
            }
    }
    // the pack kernel's tile_load adds at most one superblock total per lane per tile step:
    // G/128 + 1 <= 64
    if (g > (uint64_t)(kWave - 1) * kTilesPerSb) g = (uint64_t)(kWave - 1) * kTilesPerSb;
    return tiles < g ? tiles : g;
}

// Persistent grid of the group decode kernel (kDecG waves a workgroup): occupancy x CUs, at most
// one workgroup per group.
uint64_t group_grid(const void* kernel, uint64_t groups) {
    static thread_local const void* ck[4] = {};
    static thread_local int cdev[4] = {};
    static thread_local uint64_t cg[4] = {};
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess) dev = 0;
    uint64_t g = 0;
    for (int i = 0; i < 4; ++i)
        if (ck[i] == kernel && cdev[i] == dev) g = cg[i];
    if (g == 0) {
        int per_cu = 0, cus = 0;
        if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, kernel, kDecG * kWave, 0) != hipSuccess || per_cu < 1)
            per_cu = 1;
        if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus < 1)
            cus = 256;
        g = (uint64_t)per_cu * (uint64_t)cus;
        for (int i = 0; i < 4; ++i)
            if (ck[i] == nullptr) {
                ck[i] = kernel;
                cdev[i] = dev;
                cg[i] = g;
                break;
            }
    }
    return groups < g ? groups : g;
}

// Optional launch profiling: every `g_prof_every`-th launch of the pack kernel and of the decode
// kernel carries a pair of HIP events, kept in a ring per kernel (read by sbe_profile_read).
struct ProfRing {
    static constexpr int kCap = 256;
    hipEvent_t ev[kCap][2];
    int head = 0, count = 0;
    uint64_t launches = 0;
    bool ready = false;
};
thread_local int g_prof_every = 0;
thread_local ProfRing g_prof[2];

// The ring slot's (start, stop) events for this launch of `which`, or nulls when it is not
// sampled.  They are handed to hipExtLaunchKernel, which timestamps the kernel's own dispatch.
// The ring's events, created once (by sbe_profile_enable, outside any timed region); the error of
// the failing creation otherwise.
hipError_t prof_ready(ProfRing& R) {
    if (!R.ready) {
        for (int i = 0; i < ProfRing::kCap; ++i)
            for (int j = 0; j < 2; ++j) {
                const hipError_t e = hipEventCreate(&R.ev[i][j]);
                if (e != hipSuccess) return e;
            }
        R.ready = true;
    }
    return hipSuccess;
}

void prof_slot(int which, hipEvent_t* start, hipEvent_t* stop) {
    *start = *stop = nullptr;
    if (g_prof_every <= 0) return;
    ProfRing& R = g_prof[which];
    if (R.launches++ % (uint64_t)g_prof_every != 0) return;
    if (!R.ready) return;  // sbe_profile_enable creates the events; never inside a launch
    *start = R.ev[R.head][0];
    *stop = R.ev[R.head][1];
}
void prof_commit(int which, hipEvent_t start) {
    if (!start) return;
    ProfRing& R = g_prof[which];
    R.head = (R.head + 1) % ProfRing::kCap;
    if (R.count < ProfRing::kCap) ++R.count;
}


// ------------------------------------------------------------------------------------------
// Aeron fragment reassembly (LocalFragmentReassembler::onFragment, src/cluster_client.cpp:39-82)
//   1-3. the inclusive scan of one element per fragment (delivery-point count, last BEGIN, last
//      END, singles, the accumulator as an affine map) in three launches (frag_reduce,
//      frag_scan_blocks, frag_scan: the elements are classified on the fly, never stored)
//   4. frag_messages: every delivery point (a BEGIN|END single, or an END) writes its message's
//      offset and size from the accumulator map, and the first / last fragment of its group (the
//      non-single fragments since the last BEGIN or END before it); the open group at the end of
//      the batch is the carry
//   5. frag_copy: one wave per 64 messages, runs of back-to-back messages copied as one block
//      (fragment by fragment only when a single sits inside a group)
// ------------------------------------------------------------------------------------------
// The accumulator of onFragment as an affine map on (p = pending bytes, d = delivered bytes):
// (p, d) -> (A p + B, d + C p + E), A, C in {0, 1}:
//   single (BEGIN|END) A = 1, E = len;  BEGIN  A = 0, B = len;  middle  A = 1, B = len;
//   END    A = 0, C = 1, E = len.
// Maps compose associatively (g after f: A = Ag Af, B = Ag Bf + Bg, C = Cf + Cg Af, E = Ef + Cg Bf
// + Eg; C stays 0 or 1: Cf = 1 implies Af = 0), so the inclusive scan gives, from (0, 0), the
// pending and delivered bytes after every fragment: a message delivered at fragment i starts at
// E(i - 1) in the output and has E(i) - E(i - 1) bytes, and the carry is B(n - 1).
struct FragScan {  // 32 bytes (batches of up to 2^31 fragments, so bit 31 of dp / sg is free)
    uint32_t dp;   // delivery points (singles + ENDs) so far; bit 31: C
    uint32_t sg;   // singles so far; bit 31: A
    int32_t lb;    // last BEGIN (non-single) index so far, -1 none
    int32_t le;    // last END (non-single) index so far, -1 none
    uint64_t B, E; // the accumulator map (above)
};
constexpr uint32_t kFsCount = 0x7fffffffu;
__host__ __device__ __forceinline__ uint32_t fs_dp(const FragScan& e) { return e.dp & kFsCount; }
__host__ __device__ __forceinline__ uint32_t fs_sg(const FragScan& e) { return e.sg & kFsCount; }
struct FragScanOp {  // a before b
    __host__ __device__ FragScan operator()(const FragScan& a, const FragScan& b) const {
        const bool Aa = (a.sg >> 31) != 0, Ab = (b.sg >> 31) != 0, Ca = (a.dp >> 31) != 0, Cb = (b.dp >> 31) != 0;
        const uint32_t C = (Ca || (Cb && Aa)) ? 0x80000000u : 0u, A = (Aa && Ab) ? 0x80000000u : 0u;
        return FragScan{((fs_dp(a) + fs_dp(b)) & kFsCount) | C, ((fs_sg(a) + fs_sg(b)) & kFsCount) | A,
                        a.lb > b.lb ? a.lb : b.lb, a.le > b.le ? a.le : b.le,
                        (Ab ? a.B : 0ull) + b.B, a.E + (Cb ? a.B : 0ull) + b.E};
    }
};

struct FragArgs {
    const uint8_t* in;
    const uint64_t* frag_off;
    const uint8_t* flags;
    uint64_t n;
    uint8_t* out;
    uint64_t* msg_off;
    uint64_t* counts;
    FragScan* el;      // [n] scan elements
    FragScan* sc;      // [n] their inclusive scan
    uint64_t* msize;   // [n + 1]
    uint64_t* mfirst;  // [n + 1] first fragment of message j
    uint64_t* mlast;   // [n + 1] last fragment (bit 63: a single sits inside the group)
    uint64_t* big;     // big[0]: count, big[1..]: messages of >= kFcBig bytes without a single inside
                       // (copied by every wave of frag_copy together); nullptr: none singled out
};
// A message (or the carry) this large is not copied by the one wave that holds its table entry:
// frag_scan_msgs lists it, and frag_copy's waves copy the listed messages together in 64 KiB
// pieces after their own groups.  One wave copies a few GB/s, so one 32 MB message took 12 ms
// alone while a 1 M-fragment batch of short messages takes 0.1 ms (tests/test_reassembly.py).
constexpr uint64_t kFcBig = 64 * 1024, kFcPiece = 64 * 1024;

__device__ __forceinline__ bool frag_single(uint8_t f) {
    return (f & (SBE_FRAG_BEGIN | SBE_FRAG_END)) == (SBE_FRAG_BEGIN | SBE_FRAG_END);
}

// The scan of the per-fragment elements in three launches of our own (it replaced a classify
// kernel + a generic device scan over the 24-B tuple, which ran at 0.6 TB/s): frag_reduce classifies each
// 1024-fragment block on the fly and writes the block's aggregate; frag_scan_blocks turns the
// aggregates into exclusive block prefixes (one workgroup, 1024 at a time with a carry);
// frag_scan re-classifies and writes the inclusive scan.  Elements are never materialised.
#ifndef SBE_FS_PER  // A/B builds: fragments per thread of the scan launches
#define SBE_FS_PER 4
#endif
constexpr int kFsPer = SBE_FS_PER, kFsThreads = 256, kFsBlk = kFsPer * kFsThreads;
__device__ __forceinline__ FragScan fs_identity() { return FragScan{0u, 0x80000000u, -1, -1, 0ull, 0ull}; }
__device__ __forceinline__ FragScan fs_elem(const FragArgs& a, uint64_t i) {
    if (i >= a.n) return fs_identity();
    const uint8_t f = a.flags[i];
    const bool single = frag_single(f);
    const bool begin = (f & SBE_FRAG_BEGIN) != 0, endf = (f & SBE_FRAG_END) != 0;
    const uint64_t len = a.frag_off[i + 1] - a.frag_off[i];
    FragScan e;
    e.dp = ((single || endf) ? 1u : 0u) | ((!single && endf) ? 0x80000000u : 0u);      // C: END
    e.sg = (single ? 1u : 0u) | ((single || (!begin && !endf)) ? 0x80000000u : 0u);  // A: single / middle
    e.lb = (!single && begin) ? (int32_t)i : -1;
    e.le = (!single && endf) ? (int32_t)i : -1;
    e.B = (!single && !endf) ? len : 0ull;  // BEGIN / middle
    e.E = (single || endf) ? len : 0ull;    // single / END
    return e;
}
__device__ __forceinline__ FragScan fs_shfl_up(const FragScan& v, int d) {
    FragScan t;
    t.dp = __shfl_up(v.dp, d, kWave);
    t.sg = __shfl_up(v.sg, d, kWave);
    t.lb = __shfl_up(v.lb, d, kWave);
    t.le = __shfl_up(v.le, d, kWave);
    t.B = __shfl_up(v.B, d, kWave);
    t.E = __shfl_up(v.E, d, kWave);
    return t;
}
// inclusive scan across the wave (Hillis-Steele on shuffles: this is a small share of the work)
__device__ __forceinline__ FragScan fs_wave_scan(FragScan v, int lane) {
#pragma unroll
    for (int d = 1; d < kWave; d <<= 1) {
        const FragScan t = fs_shfl_up(v, d);
        if (lane >= d) v = FragScanOp{}(t, v);
    }
    return v;
}
// the block's kFsBlk elements, kFsPer consecutive ones per thread, scanned: thread-inclusive values
// in e[], the block total returned (LDS wt[] holds the wave totals)
__device__ __forceinline__ FragScan fs_block(const FragArgs& a, uint64_t b, FragScan (&e)[kFsPer], FragScan* wt,
                                             FragScan& before) {
    const int tid = threadIdx.x, lane = tid & (kWave - 1), w = tid / kWave;
    const uint64_t i0 = b * kFsBlk + (uint64_t)tid * kFsPer;
#pragma unroll
    for (int k = 0; k < kFsPer; ++k) e[k] = fs_elem(a, i0 + k);
#pragma unroll
    for (int k = 1; k < kFsPer; ++k) e[k] = FragScanOp{}(e[k - 1], e[k]);
    const FragScan inc = fs_wave_scan(e[kFsPer - 1], lane);
    const FragScan up = fs_shfl_up(inc, 1);
    const FragScan ex = lane ? up : fs_identity();  // the thread's exclusive prefix inside the wave
    if (lane == kWave - 1) wt[w] = inc;
    __syncthreads();
    FragScan wpre = fs_identity(), tot = fs_identity();
#pragma unroll
    for (int k = 0; k < kFsThreads / kWave; ++k) {
        if (k < w) wpre = FragScanOp{}(wpre, wt[k]);
        tot = FragScanOp{}(tot, wt[k]);
    }
    before = FragScanOp{}(wpre, ex);
    return tot;
}
__global__ __launch_bounds__(kFsThreads) void frag_reduce(FragArgs a, FragScan* agg) {
    __shared__ FragScan wt[kFsThreads / kWave];
    const uint64_t b = blockIdx.x;
    FragScan e[kFsPer], before;
    const FragScan tot = fs_block(a, b, e, wt, before);
    if (threadIdx.x == 0) agg[b] = tot;
}
// exclusive prefixes of the nb block aggregates, in place: one workgroup of kFsThreads threads,
// kFsPer consecutive aggregates a thread (a million fragments' 977 aggregates in one pass; at 1024
// threads a pass the scan's registers spilled: 21 us instead of a few)
constexpr int kFsbThreads = kFsThreads;
__global__ __launch_bounds__(kFsbThreads) void frag_scan_blocks(FragScan* agg, uint64_t nb, uint64_t* big) {
    __shared__ FragScan wt[kFsbThreads / kWave];
    const int tid = threadIdx.x, lane = tid & (kWave - 1), w = tid / kWave;
    if (big && tid == 0) big[0] = 0;  // the big-message list of frag_scan_msgs (next launch)
    FragScan carry = fs_identity();
    for (uint64_t c0 = 0; c0 < nb; c0 += kFsBlk) {
        const uint64_t j0 = c0 + (uint64_t)tid * kFsPer;
        FragScan e[kFsPer];
#pragma unroll
        for (int k = 0; k < kFsPer; ++k) e[k] = j0 + k < nb ? agg[j0 + k] : fs_identity();
        FragScan r[kFsPer];  // thread-inclusive
        r[0] = e[0];
#pragma unroll
        for (int k = 1; k < kFsPer; ++k) r[k] = FragScanOp{}(r[k - 1], e[k]);
        const FragScan inc = fs_wave_scan(r[kFsPer - 1], lane);
        const FragScan up = fs_shfl_up(inc, 1);
        const FragScan ex = lane ? up : fs_identity();
        __syncthreads();
        if (lane == kWave - 1) wt[w] = inc;
        __syncthreads();
        FragScan wpre = fs_identity(), tot = fs_identity();
#pragma unroll
        for (int k = 0; k < kFsbThreads / kWave; ++k) {
            if (k < w) wpre = FragScanOp{}(wpre, wt[k]);
            tot = FragScanOp{}(tot, wt[k]);
        }
        const FragScan P = FragScanOp{}(carry, FragScanOp{}(wpre, ex));  // before this thread's first
#pragma unroll
        for (int k = 0; k < kFsPer; ++k)
            if (j0 + k < nb) agg[j0 + k] = k ? FragScanOp{}(P, r[k - 1]) : P;
        carry = FragScanOp{}(carry, tot);
    }
}
__global__ __launch_bounds__(kFsThreads) void frag_scan(FragArgs a, const FragScan* pre) {
    __shared__ FragScan wt[kFsThreads / kWave];
    const uint64_t b = blockIdx.x;
    FragScan e[kFsPer], before;
    (void)fs_block(a, b, e, wt, before);
    const FragScan base = FragScanOp{}(pre[b], before);
    const uint64_t i0 = b * kFsBlk + (uint64_t)threadIdx.x * kFsPer;
#pragma unroll
    for (int k = 0; k < kFsPer; ++k)
        if (i0 + k < a.n) a.sc[i0 + k] = FragScanOp{}(base, e[k]);
}

// group of non-single fragments ending at i (inclusive): from the later of the last BEGIN at or
// before i and the fragment after the last END before i
// (its bytes come from the accumulator map: FragScan)
__device__ __forceinline__ void frag_group(const FragArgs& a, uint64_t i, int64_t le_before, uint64_t& s, bool& gap) {
    const FragScan& e = a.sc[i];
    int64_t st = (int64_t)e.lb > le_before + 1 ? (int64_t)e.lb : le_before + 1;
    if (st < 0) st = 0;
    s = (uint64_t)st;
    const uint32_t sg0 = s ? fs_sg(a.sc[s - 1]) : 0u;
    gap = fs_sg(e) != sg0;
}

__global__ __launch_bounds__(256) void frag_messages(FragArgs a) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= a.n) return;
    const uint8_t f = a.flags[i];
    const FragScan e = a.sc[i];
    const uint64_t E0 = i ? a.sc[i - 1].E : 0ull;  // delivered bytes before fragment i
    const bool single = frag_single(f);
    const uint32_t dp = fs_dp(e);
    if ((single || (f & SBE_FRAG_END)) && dp >= 1 && dp <= a.n) {
        const uint64_t j = dp - 1;
        a.msize[j] = e.E - E0;
        a.msg_off[j] = E0;
        if (single) {
            a.mfirst[j] = i;
            a.mlast[j] = i;
        } else {
            uint64_t s;
            bool gap;
            frag_group(a, i, i ? a.sc[i - 1].le : -1, s, gap);
            a.mfirst[j] = s;
            a.mlast[j] = i | (gap ? (1ull << 63) : 0ull);
        }
    }
    if (i == a.n - 1) {  // the open accumulator after the last fragment: the carry
        const uint64_t m = dp <= a.n ? dp : a.n;
        uint64_t s;
        bool gap;
        frag_group(a, i, e.le, s, gap);
        const uint64_t bytes = e.B;  // pending bytes after the last fragment
        const bool open = (int64_t)s <= (int64_t)i && bytes > 0;
        a.msize[m] = open ? bytes : 0u;
        a.msg_off[m] = e.E;
        a.mfirst[m] = s;
        a.mlast[m] = i | (gap ? (1ull << 63) : 0ull);
        a.counts[0] = m;
        a.counts[1] = open ? bytes : 0u;
    }
}

// frag_scan and frag_messages in one launch (the default): the block's inclusive scan stays in
// registers (and the singles counts in LDS) instead of a 32-B element per fragment written to HBM
// and read back.  A group that starts before the block finds the singles before its start from
// the block's exclusive prefix minus the singles between its start and the block (few fragments:
// groups are short).
#ifndef SBE_FRAG_FUSED  // A/B builds: 0 = frag_scan + frag_messages
#define SBE_FRAG_FUSED 1
#endif
// The block's messages are the consecutive indices [dp before the block, dp after it): their four
// table entries go through LDS, one array at a time, and leave as contiguous 8-B stores per lane
// (stored straight from each fragment's lane, a wave's 64 stores land 32 B apart and the table
// cost 56.6 MB of HBM writes for 32 MB of entries, profiles/r05_reasm2_summary.txt).
#ifndef SBE_FRAG_STAGE
#define SBE_FRAG_STAGE 1
#endif
// Singles among fragments [0, x] for an x in an earlier block than b (rare: the start of a group
// that crosses into block b; out of line, so its registers stay out of frag_scan_msgs): from the
// nearer block boundary, counting the singles between it and x from 16-byte aligned flag loads (at
// most kFsBlk / 32 + 1 independent loads; an aligned 16-B block holding a flag byte never crosses
// a page): x's own block's exclusive prefix plus the singles in [its start, x], or the prefix of
// the block after x's minus the singles in (x, that block's start).  Walking one flag at a time
// from x up to block b cost thousands of loads for a group of thousands of fragments;
// always counting from x's block start made every short group across a block boundary read its
// whole block (reassembly row 146 -> 172 us, profiles/r06_ab_reasm_big.log).
__device__ __noinline__ uint32_t frag_singles_before(const FragArgs& a, const FragScan* pre, uint64_t x, uint64_t b) {
    const uint64_t bx = x / kFsBlk, s = bx * kFsBlk;
    const bool fwd = x - s < s + kFsBlk - 1 - x;
    const uint32_t c = fs_sg(fwd ? pre[bx] : pre[bx + 1]);  // bx + 1 <= b: pre[b] is the block's own prefix
    const uintptr_t lo = reinterpret_cast<uintptr_t>(a.flags + (fwd ? s : x + 1)),
                    hi = reinterpret_cast<uintptr_t>(a.flags + (fwd ? x : s + kFsBlk - 1));
    uint32_t cnt = 0;
    for (uintptr_t q = lo & ~(uintptr_t)15; q <= hi && lo <= hi; q += 16) {
        const uint4 w4 = gload128(q);
        const uint32_t w0 = w4.x, w1 = w4.y, w2 = w4.z, w3 = w4.w;
#pragma unroll
        for (int t = 0; t < 4; ++t) {
            const uint32_t w = t == 0 ? w0 : t == 1 ? w1 : t == 2 ? w2 : w3;
            const uintptr_t b0 = q + 4 * t;  // address of byte 0 of this dword
            uint32_t m = (w >> 1) & w & 0x40404040u;  // bit 6 of a byte: BEGIN and END both set
            if (b0 < lo) m &= lo - b0 >= 4 ? 0u : ~0u << (8 * (lo - b0));
            if (b0 + 3 > hi) m &= b0 > hi ? 0u : byte_mask_bits((uint32_t)(hi - b0 + 1));
            cnt += __builtin_popcount(m);
        }
    }
    (void)b;
    return fwd ? c + cnt : c - cnt;
}

__global__ __launch_bounds__(kFsThreads) void frag_scan_msgs(FragArgs a, const FragScan* pre) {
    __shared__ FragScan wt[kFsThreads / kWave];
    __shared__ uint32_t sgl[kFsBlk];  // inclusive singles count at every fragment of the block
#if SBE_FRAG_STAGE
    __shared__ uint64_t stg[kFsBlk];  // one table array of the block's messages
    uint64_t tv[kFsPer][4];
    uint32_t tj[kFsPer];              // message index - j0, or ~0u (no message at this fragment)
#endif
    const uint64_t b = blockIdx.x;
    FragScan e[kFsPer], before;
    const FragScan tot = fs_block(a, b, e, wt, before);
    const FragScan P = pre[b];  // the scan at the fragment before the block
    const FragScan base = FragScanOp{}(P, before);
    const int tid = threadIdx.x;
    const uint64_t blk0 = b * kFsBlk, i0 = blk0 + (uint64_t)tid * kFsPer;
    FragScan v[kFsPer];
#pragma unroll
    for (int k = 0; k < kFsPer; ++k) {
        v[k] = FragScanOp{}(base, e[k]);
        sgl[tid * kFsPer + k] = fs_sg(v[k]);
    }
    __syncthreads();
    auto sg_at = [&](uint64_t x) -> uint32_t {  // singles among fragments [0, x]
        return x >= blk0 ? sgl[x - blk0] : frag_singles_before(a, pre, x, b);
    };
    auto group = [&](const FragScan& x, int64_t le_before, uint64_t& s0, bool& gap) {  // frag_group
        int64_t st = (int64_t)x.lb > le_before + 1 ? (int64_t)x.lb : le_before + 1;
        if (st < 0) st = 0;
        s0 = (uint64_t)st;
        const uint32_t sg0 = s0 ? sg_at(s0 - 1) : 0u;
        gap = fs_sg(x) != sg0;
    };
#if SBE_FRAG_STAGE
    const uint32_t j0 = fs_dp(P), nj = fs_dp(tot);  // the block's messages: [j0, j0 + nj)
#pragma unroll
    for (int k = 0; k < kFsPer; ++k) tj[k] = ~0u;
#endif
#pragma unroll
    for (int k = 0; k < kFsPer; ++k) {
        const uint64_t i = i0 + k;
        if (i >= a.n) break;
        const FragScan& x = v[k];
        const FragScan& prev = k ? v[k - 1] : base;  // the scan at fragment i - 1 (identity before 0)
        const uint8_t f = a.flags[i];
        const uint64_t E0 = i ? prev.E : 0ull;
        const bool single = frag_single(f);
        const uint32_t dp = fs_dp(x);
        if ((single || (f & SBE_FRAG_END)) && dp >= 1 && dp <= a.n) {
            const uint64_t j = dp - 1;
            uint64_t first = i, last = i;
            if (!single) {
                uint64_t s0;
                bool gap;
                group(x, i ? (int64_t)prev.le : -1, s0, gap);
                first = s0;
                last = i | (gap ? (1ull << 63) : 0ull);
            }
            if (a.big && !(last >> 63) && x.E - E0 >= kFcBig)  // rare: a few per batch at most
                a.big[1 + atomicAdd(reinterpret_cast<unsigned long long*>(a.big), 1ull)] = j;
#if SBE_FRAG_STAGE
            tj[k] = (uint32_t)(j - j0);
            tv[k][0] = x.E - E0;
            tv[k][1] = E0;
            tv[k][2] = first;
            tv[k][3] = last;
#else
            a.msize[j] = x.E - E0;
            a.msg_off[j] = E0;
            a.mfirst[j] = first;
            a.mlast[j] = last;
#endif
        }
        if (i == a.n - 1) {  // the open accumulator after the last fragment: the carry
            const uint64_t m = dp <= a.n ? dp : a.n;
            uint64_t s0;
            bool gap;
            group(x, x.le, s0, gap);
            const uint64_t bytes = x.B;
            const bool open = (int64_t)s0 <= (int64_t)i && bytes > 0;
            a.msize[m] = open ? bytes : 0u;
            a.msg_off[m] = x.E;
            a.mfirst[m] = s0;
            a.mlast[m] = i | (gap ? (1ull << 63) : 0ull);
            a.counts[0] = m;
            a.counts[1] = open ? bytes : 0u;
            if (a.big && open && !gap && bytes >= kFcBig)
                a.big[1 + atomicAdd(reinterpret_cast<unsigned long long*>(a.big), 1ull)] = m;
        }
    }
#if SBE_FRAG_STAGE
#pragma unroll
    for (int r = 0; r < 4; ++r) {
#pragma unroll
        for (int k = 0; k < kFsPer; ++k)
            if (tj[k] != ~0u) stg[tj[k]] = tv[k][r];
        __syncthreads();
        uint64_t* dst = (r == 0 ? a.msize : r == 1 ? a.msg_off : r == 2 ? a.mfirst : a.mlast) + j0;
        for (uint32_t t = tid; t < nj; t += kFsThreads) dst[t] = stg[t];
        __syncthreads();
    }
#endif
}

// the 16 bytes at src + 16c + sh from the aligned blocks b0 (at 16c) and b1 (the next one)
__device__ __forceinline__ uint4 join16(uint4 b0, uint4 b1, uint32_t sh) {
    const uint32_t w[8] = {b0.x, b0.y, b0.z, b0.w, b1.x, b1.y, b1.z, b1.w};
    const uint32_t ds = sh >> 2, bs = sh & 3u;
    uint32_t v[5];
#pragma unroll
    for (int t = 0; t < 5; ++t)  // v[t] = w[t + ds] (selects keep w in registers)
        v[t] = ds == 0 ? w[t] : ds == 1 ? w[t + 1] : ds == 2 ? w[t + 2] : w[t + 3 < 8 ? t + 3 : 7];
    return make_uint4(__builtin_amdgcn_alignbyte(v[1], v[0], bs), __builtin_amdgcn_alignbyte(v[2], v[1], bs),
                      __builtin_amdgcn_alignbyte(v[3], v[2], bs), __builtin_amdgcn_alignbyte(v[4], v[3], bs));
}

// wave copy of src[0, len) to dst with 16-byte stores once dst is aligned; each output chunk
// joins the two aligned 16-byte source blocks it spans (never past the source's last block);
// four chunks per lane per step, all eight loads issued before the first join
#ifndef SBE_FC_U  // A/B builds: chunks per lane per copy step
#define SBE_FC_U 4
#endif
constexpr int kFcU = SBE_FC_U;
// One unaligned 16-byte load per output chunk (a single global_load_dwordx4 at any byte address)
// instead of the two aligned blocks it spans joined with v_alignbyte: reassembly row 188.4 ->
// 185.3 us (profiles/r05_ab_fragcopy.log); SBE_FC_UA=0 builds the joined form.
#ifndef SBE_FC_UA
#define SBE_FC_UA 1
#endif
#ifndef SBE_FC_NT
#define SBE_FC_NT 1
#endif
typedef u32x4 u32x4_a1 __attribute__((aligned(1)));
typedef __attribute__((address_space(1))) const u32x4_a1 g_u32x4_a1;
// The copy's source loads are nontemporal (each fragment is read once): on rotated inputs the row
// read 157.0 / 157.0 / 156.9 -> 154.9 / 155.8 / 154.2 us over three alternations
// (profiles/r06_ab_fc_rot.log; round 5, re-reading one batch every step, had them slower, 149.7 ->
// 163.4 us); 2 / 8 chunks a lane a step 160.4-161.1 / 157.7-159.4 us.
#ifndef SBE_FC_NTL  // A/B builds: 0 = default-policy source loads
#define SBE_FC_NTL 1
#endif
__device__ __forceinline__ uint4 gload128_ua(uintptr_t addr) {  // any byte address (one global_load_dwordx4)
#if SBE_FC_NTL
    const u32x4 v = __builtin_nontemporal_load(reinterpret_cast<g_u32x4_a1*>(addr));
#else
    const u32x4 v = *reinterpret_cast<g_u32x4_a1*>(addr);
#endif
    return make_uint4(v.x, v.y, v.z, v.w);
}
__device__ __forceinline__ void wave_copy16(uint8_t* dst, const uint8_t* src, uint64_t len, int lane) {
    if (len == 0) return;
    uint64_t head = (16u - ((uintptr_t)dst & 15u)) & 15u;
    head = head < len ? head : len;
    if ((uint64_t)lane < head) dst[lane] = src[lane];
    const uint64_t nc = (len - head) >> 4;
    const uintptr_t p0 = reinterpret_cast<uintptr_t>(src) + head;
    uint4* d16 = reinterpret_cast<uint4*>(dst + head);
#if SBE_FC_UA
    // the chunk's 16 source bytes in one load at their own (unaligned) address: no join, half the
    // loads (every byte read lies inside the source)
    for (uint64_t c0 = 0; c0 < nc; c0 += kFcU * kWave) {
        uint4 x[kFcU];
#pragma unroll
        for (int u = 0; u < kFcU; ++u) {
            const uint64_t c = c0 + (uint64_t)lane + (uint64_t)kWave * u;
            x[u] = gload128_ua(p0 + 16 * (c < nc ? c : nc - 1));
        }
#pragma unroll
        for (int u = 0; u < kFcU; ++u) {
            const uint64_t c = c0 + (uint64_t)lane + (uint64_t)kWave * u;
#if SBE_FC_NT  // nontemporal (streamed) stores, as the pack and decode kernels' outputs
            if (c < nc) {
                u32x4 v;
                v.x = x[u].x, v.y = x[u].y, v.z = x[u].z, v.w = x[u].w;
                __builtin_nontemporal_store(v, reinterpret_cast<u32x4*>(d16 + c));
            }
#else
            if (c < nc) d16[c] = x[u];
#endif
        }
    }
#else
    const uint32_t sh = (uint32_t)(p0 & 15u);
    const uintptr_t q0 = p0 & ~(uintptr_t)15;
    for (uint64_t c0 = 0; c0 < nc; c0 += kFcU * kWave) {
        uint4 x[kFcU], y[kFcU];
#pragma unroll
        for (int u = 0; u < kFcU; ++u) {
            const uint64_t c = c0 + (uint64_t)lane + (uint64_t)kWave * u;
            const uintptr_t q = q0 + 16 * (c < nc ? c : nc - 1);
            x[u] = gload128(q);
            y[u] = gload128(q + (sh ? 16 : 0));
        }
#pragma unroll
        for (int u = 0; u < kFcU; ++u) {
            const uint64_t c = c0 + (uint64_t)lane + (uint64_t)kWave * u;
            if (c < nc) d16[c] = sh ? join16(x[u], y[u], sh) : x[u];
        }
    }
#endif
    const uint64_t t0 = head + 16 * nc;
    if ((uint64_t)lane < len - t0) dst[t0 + lane] = src[t0 + lane];
}

// One wave per kFragGroup consecutive messages: lane l loads message (base + l)'s size, source
// and destination (coalesced; small groups keep each wave's copy short, many waves in flight).  Consecutive messages whose sources are back to back (singles and
// complete groups: the common case) form runs, each copied as one block; a message with a single
// inside its group is copied fragment by fragment.
constexpr int kFragGroup = 64;
#ifndef SBE_FC_PF  // A/B builds: prefetch the next group's message metadata during the copy
#define SBE_FC_PF 0
#endif
__global__ __launch_bounds__(256) void frag_copy(FragArgs a) {
    const int lane = threadIdx.x & (kWave - 1);
    const uint64_t waves = (uint64_t)gridDim.x * (blockDim.x / kWave);
    const uint64_t m = a.counts[0];
    const uint64_t base0 = ((uint64_t)blockIdx.x * (blockDim.x / kWave) + threadIdx.x / kWave) * kFragGroup;
    const uint64_t step = waves * kFragGroup;
#if SBE_FC_PF
    // the next group's metadata is loaded while this group is copied (clamped index, loaded
    // unconditionally: no wait on it before the copy)
    auto meta = [&](uint64_t b, uint64_t& len_, uint64_t& first_, uint64_t& mlast_, uint64_t& dst_) {
        uint64_t jj = b + (uint64_t)lane;
        jj = jj <= m ? jj : m;
        len_ = a.msize[jj];
        first_ = a.mfirst[jj];
        mlast_ = a.mlast[jj];
        dst_ = a.msg_off[jj];
    };
    uint64_t nlen, nfirst, nmlast, ndst;
    meta(base0, nlen, nfirst, nmlast, ndst);
#endif
    for (uint64_t base = base0; base <= m; base += step) {
        const uint64_t j = base + (uint64_t)lane;
        const bool valid = lane < kFragGroup && j <= m;
#if SBE_FC_PF
        uint64_t len = nlen, first = nfirst, mlast = nmlast, dst = ndst;
        uint64_t src = a.frag_off[first];
        if (!valid) len = src = dst = mlast = first = 0;
        meta(base + step, nlen, nfirst, nmlast, ndst);
#else
        uint64_t len = 0, src = 0, dst = 0, mlast = 0, first = 0;
        if (valid) {
            len = a.msize[j];
            first = a.mfirst[j];
            mlast = a.mlast[j];
            dst = a.msg_off[j];
            src = a.frag_off[first];
        }
#endif
        const bool gap = valid && (mlast >> 63);
        // a listed big message (frag_scan_msgs) is copied by all waves after the loop: it takes no
        // part in a run here, as a gapped message does not
        const bool brk = gap || (a.big && valid && len >= kFcBig);
        // run membership: this message's source follows the previous one's (and neither is gapped)
        const uint64_t pend = __shfl_up(src + len, 1, kWave);
        const bool pgap = __shfl_up(brk ? 1 : 0, 1, kWave) != 0;
        const bool cont = lane > 0 && valid && !brk && !pgap && src == pend;
        const uint64_t starts = __ballot(valid && !brk && !cont);
        const uint64_t vmask = __ballot(valid);
        for (uint64_t mk = starts; mk; mk &= mk - 1) {
            const int k = __builtin_ctzll(mk);
            // the run ends before the next start, gapped message or invalid lane
            const uint64_t stop = (starts | __ballot(brk) | ~vmask) & ~((2ull << k) - 1);
            const int e = stop ? __builtin_ctzll(stop) : kWave;  // first lane after the run
            const uint64_t D = uniform64(__shfl(dst, k, kWave));
            const uint64_t De = uniform64(__shfl(dst + len, e - 1, kWave));
            wave_copy16(a.out + D, a.in + uniform64(__shfl(src, k, kWave)), De - D, lane);
        }
        for (uint64_t mk = __ballot(gap && len > 0); mk; mk &= mk - 1) {
            const int k = __builtin_ctzll(mk);
            const uint64_t D = uniform64(__shfl(dst, (int)k, kWave));
            const uint64_t ML = uniform64(__shfl(mlast, (int)k, kWave));
            // a single inside the group: the group's fragments 64 at a time, one a lane (flags and
            // offsets loaded at once, not one dependent round trip per fragment), singles skipped,
            // consecutive kept fragments (back to back in the input) copied as one run
            const uint64_t F = uniform64(__shfl(first, (int)k, kWave)), last = ML & ~(1ull << 63);
            uint64_t at = 0;
            for (uint64_t f0 = F; f0 <= last; f0 += kWave) {
                const uint64_t f = f0 + (uint64_t)lane;
                bool take = false;
                uint64_t fo = 0, fl = 0;
                if (f <= last) {
                    take = !frag_single(a.flags[f]);
                    fo = a.frag_off[f];
                    fl = take ? a.frag_off[f + 1] - fo : 0;
                }
                const uint64_t incl = wave_incl_scan64(fl, lane), excl = incl - fl;  // bytes before it
                const bool prev = __shfl_up(take ? 1 : 0, 1, kWave) != 0;
                const uint64_t kept = __ballot(take);
                for (uint64_t rm = __ballot(take && (lane == 0 || !prev)); rm; rm &= rm - 1) {
                    const int r0 = __builtin_ctzll(rm);
                    const uint64_t after = ~kept & ~((2ull << r0) - 1);  // first lane past the run
                    const int r1 = after ? __builtin_ctzll(after) : kWave;
                    const uint64_t d0 = uniform64(__shfl(excl, r0, kWave));
                    const uint64_t d1 = uniform64(__shfl(incl, r1 - 1, kWave));
                    wave_copy16(a.out + D + at + d0, a.in + uniform64(__shfl(fo, r0, kWave)), d1 - d0, lane);
                }
                at += lane_u64(incl, kWave - 1);
            }
        }
    }
    // the listed big messages, in kFcPiece pieces dealt round robin over every wave of the grid
    // (the list's order is the atomics' order: each message's pieces are disjoint whatever it is)
    const uint64_t nbig = a.big ? uniform64(a.big[0]) : 0ull;
    const uint64_t me = (uint64_t)blockIdx.x * (blockDim.x / kWave) + threadIdx.x / kWave;
    uint64_t pbase = 0;  // pieces of the listed messages before message q
    for (uint64_t q = 0; q < nbig; ++q) {
        const uint64_t j = uniform64(a.big[1 + q]);
        const uint64_t len = uniform64(a.msize[j]);
        const uint64_t np = (len + kFcPiece - 1) / kFcPiece;
        const uint64_t src = uniform64(a.frag_off[uniform64(a.mfirst[j])]), dst = uniform64(a.msg_off[j]);
        for (uint64_t p = (me + waves - pbase % waves) % waves; p < np; p += waves) {
            const uint64_t o = p * kFcPiece;
            wave_copy16(a.out + dst + o, a.in + src + o, len - o < kFcPiece ? len - o : kFcPiece, lane);
        }
        pbase += np;
    }
}

// ------------------------------------------------------------------------------------------
// MATERIALIZE (sbe_materialize_views): the decoded views copied into an arena.  Three launches:
// mat_sums (view bytes per 64-record tile and per 1024-record block), mat_scan_blocks (one
// workgroup: the exclusive scan of the block sums, the arena total into arena_off[5 n]) and
// mat_copy, one wave per tile.  A tile's views are one contiguous range of the arena (its base: the
// block prefix plus the sums of the block's earlier tiles plus a wave scan).  Each lane stages its
// record's views into an LDS window as 16-byte chunks, the record's chunks dealt in batches of
// kMatBatch loads in flight at once (a view's last chunk is the 16 bytes ending at the view's end,
// overlapping the chunk before it with the same bytes; a view under 16 bytes is written bytewise
// from one 16-byte load that stays inside the record), then the wave stores the window with 16-byte
// coalesced nontemporal stores and moves it on to the first record not yet written.  A record
// larger than the window is copied by its own lane straight to the arena.  Measured (1 M fixed-256
// records, all three launches; profiles/r06_ab_mat*.log): one thread a record copying straight to
// the arena 0.823 ms (every store instruction wrote 64 scattered 16-byte pieces); the LDS window
// with one dependent load a chunk 0.184 ms; batches of 1 / 4 / 8 chunk loads 0.221 / 0.169 / 0.170
// ms (and 0.20 while the large-record path was out of line: its arrays went to scratch); 8 or 12
// KiB windows, or registers for 4 waves per SIMD, 0.168-0.190 ms; the tile's input staged in a
// second 16 KiB of LDS by coalesced loads first, 0.207 ms (5 workgroups per CU instead of 10).
// ------------------------------------------------------------------------------------------
constexpr int kMatBlk = 1024;
constexpr int kMatTile = kWave;                       // records per copy wave
constexpr int kMatTpb = kMatBlk / kMatTile;           // tiles per block
#ifndef SBE_MAT_WIN  // A/B builds
#define SBE_MAT_WIN 16384
#endif
#ifndef SBE_MAT_MINW  // A/B builds: waves per SIMD the copy's registers must allow
#define SBE_MAT_MINW 1
#endif
constexpr int32_t kMatWin = SBE_MAT_WIN;              // LDS window bytes of a copy wave
#ifndef SBE_MAT_BATCH
#define SBE_MAT_BATCH 4
#endif
constexpr int kMatBatch = SBE_MAT_BATCH;              // chunk loads of a lane in flight at once
struct MatArgs {
    const uint8_t* in;
    const uint64_t* rec_off;
    uint64_t n;
    const uint8_t* status;
    const uint32_t* view_off;
    const uint32_t* view_len;
    uint8_t* arena;
    uint64_t cap;
    uint64_t* arena_off;
    uint64_t* bsum;  // per block: view bytes, then (in place) their exclusive scan
    uint64_t* tsum;  // per tile: view bytes
};
__device__ __forceinline__ uint64_t mat_rec_bytes(const MatArgs& a, uint64_t i) {
    if (i >= a.n) return 0;
    uint64_t t = 0;
#pragma unroll
    for (int k = 0; k < 5; ++k) t += a.view_len[5 * i + k];
    return t;
}
// exclusive scan of v over the 1024-thread block; total = the block's sum
__device__ __forceinline__ uint64_t mat_block_scan(uint64_t v, uint64_t& total) {
    __shared__ uint64_t wt[kMatBlk / kWave];
    const int tid = threadIdx.x, lane = tid & (kWave - 1), w = tid / kWave;
    const uint64_t inc = wave_incl_scan64(v, lane);
    if (lane == kWave - 1) wt[w] = inc;
    __syncthreads();
    uint64_t pre = 0, tot = 0;
#pragma unroll
    for (int k = 0; k < kMatBlk / kWave; ++k) {
        pre += k < w ? wt[k] : 0ull;
        tot += wt[k];
    }
    total = tot;
    return pre + inc - v;
}
__global__ __launch_bounds__(kMatBlk) void mat_sums(MatArgs a) {
    const uint64_t i = (uint64_t)blockIdx.x * kMatBlk + threadIdx.x;
    const uint64_t v = mat_rec_bytes(a, i);
    const uint64_t t = wave_sum64(v);
    if ((threadIdx.x & (kWave - 1)) == 0 && i < a.n) a.tsum[i / kMatTile] = t;
    uint64_t tot;
    (void)mat_block_scan(v, tot);
    if (threadIdx.x == 0) a.bsum[blockIdx.x] = tot;
}
__global__ __launch_bounds__(kMatBlk) void mat_scan_blocks(MatArgs a, uint64_t nb) {
    uint64_t carry = 0;
    for (uint64_t c0 = 0; c0 < nb; c0 += kMatBlk) {
        const uint64_t j = c0 + threadIdx.x;
        uint64_t tot;
        const uint64_t v = j < nb ? a.bsum[j] : 0ull;
        const uint64_t ex = mat_block_scan(v, tot);
        __syncthreads();
        if (j < nb) a.bsum[j] = carry + ex;
        carry += tot;
        __syncthreads();
    }
    if (threadIdx.x == 0) a.arena_off[5 * a.n] = carry;
}
typedef uint32_t u32x4_ua __attribute__((ext_vector_type(4), aligned(1)));
typedef __attribute__((address_space(3))) u32x4_ua lds_u32x4_ua;
typedef __attribute__((address_space(3))) uint8_t mat_lds8;
// Views [0, k_end) of a record (arena offsets at[], lengths L[], record-relative sources O[]) from
// rec straight to the arena at dst (= arena byte at[0]), one lane: whole 16-byte chunks, a view's
// last chunk running into the next view (written afterwards) when the source stays inside the
// record (rl bytes) and the destination before lim; the last view's tail bytewise.  The path of
// records larger than an LDS window.
__device__ __forceinline__ void mat_views_direct(uint8_t* dst, const uint8_t* rec, uint64_t rl, const uint64_t (&at)[6],
                                                 const uint32_t (&L)[5], const uint32_t (&O)[5], int k_end, uint64_t lim) {
#pragma unroll
    for (int k = 0; k < 5; ++k) {
        if (k >= k_end || L[k] == 0) continue;
        const uint8_t* src = rec + O[k];
        uint8_t* d = dst + (at[k] - at[0]);
        uint32_t c = 0;
        for (; c + 16 <= L[k] || (c < L[k] && at[k] + c + 16 <= lim && O[k] + c + 16 <= rl); c += 16) {
            const u32x4_ua v = *reinterpret_cast<const u32x4_ua*>(src + c);
            __builtin_nontemporal_store(v, reinterpret_cast<u32x4_ua*>(d + c));
        }
        for (; c < L[k]; ++c) d[c] = src[c];
    }
}
// byte o (0..15) of a 16-byte block, by 64-bit shifts (no private array)
__device__ __forceinline__ uint8_t mat_byte(const u32x4_ua& v, uint32_t o) {
    const uint64_t h = (o & 8) ? ((uint64_t)v.w << 32 | v.z) : ((uint64_t)v.y << 32 | v.x);
    return (uint8_t)(h >> (8 * (o & 7)));
}
__device__ __forceinline__ uint64_t mat_wave_min(uint64_t v) {
#pragma unroll
    for (int d = 32; d >= 1; d >>= 1) {
        const uint64_t t = __shfl_xor(v, d, kWave);
        v = t < v ? t : v;
    }
    return v;
}
__device__ __forceinline__ uint64_t mat_wave_max(uint64_t v) {
#pragma unroll
    for (int d = 32; d >= 1; d >>= 1) {
        const uint64_t t = __shfl_xor(v, d, kWave);
        v = t > v ? t : v;
    }
    return v;
}
// Views [0, k_end) of a record into the LDS window at w (= arena byte at[0]): chunk q of the record
// (views in order, ceil(L / 16) chunks a view, chunk j of a view at min(16 j, L - 16)), kMatBatch
// loads issued before their LDS stores.  A view under 16 bytes: one 16-byte load inside the record
// (from the view's start, or ending at its end) and its bytes stored one by one.
// (nontemporal view loads: 0.165 -> 0.244 ms, profiles/r06_ab_matntl.log: a record's later chunks
// re-read the lines its first loads brought in)
#ifndef SBE_MAT_NTL  // A/B builds: 1 = the views' loads nontemporal
#define SBE_MAT_NTL 0
#endif
__device__ __forceinline__ void mat_views_lds(mat_lds8* w, const uint8_t* rec, uint64_t rl, const uint64_t (&at)[6],
                                              const uint32_t (&L)[5], const uint32_t (&O)[5], int k_end) {
    uint32_t cc[6];  // first chunk of each view
    cc[0] = 0;
#pragma unroll
    for (int k = 0; k < 5; ++k) cc[k + 1] = cc[k] + (k < k_end ? (L[k] + 15) >> 4 : 0u);
    const uint32_t nq = cc[5];
    for (uint32_t q0 = 0; q0 < nq; q0 += kMatBatch) {
        u32x4_ua v[kMatBatch];
        uint32_t dof[kMatBatch], bo[kMatBatch], bm[kMatBatch];
#pragma unroll
        for (int b = 0; b < kMatBatch; ++b) {
            const uint32_t q = q0 + b;
            // the view holding chunk q (views past k_end have no chunks)
            uint32_t Lk = L[0], Ok = O[0], ck = 0;
            uint64_t ak = at[0];
#pragma unroll
            for (int k = 1; k < 5; ++k)
                if (q >= cc[k]) {
                    Lk = L[k];
                    Ok = O[k];
                    ck = cc[k];
                    ak = at[k];
                }
            const uint32_t j = q - ck;
            uint32_t s;   // source offset in the record of the 16 loaded bytes
            uint32_t d;   // window offset of the first byte stored
            bo[b] = 0;    // first loaded byte stored
            bm[b] = 16;   // bytes stored (16: one 16-byte store)
            if (Lk >= 16) {
                const uint32_t p = 16 * j < Lk - 16 ? 16 * j : Lk - 16;
                s = Ok + p;
                d = (uint32_t)(ak - at[0]) + p;
            } else {  // a short view: its bytes from one load inside the record
                const bool fwd = (uint64_t)Ok + 16 <= rl;
                s = fwd ? Ok : (Ok + Lk >= 16 ? Ok + Lk - 16 : 0u);
                bo[b] = fwd ? 0u : (Ok + Lk >= 16 ? 16u - Lk : Ok);
                bm[b] = Lk;
                d = (uint32_t)(ak - at[0]);
                if (rl < 16) {  // a record under 16 bytes: no load fits inside it; bytewise below
                    bm[b] = 0x100u | Lk;
                    bo[b] = Ok;
                }
            }
            dof[b] = d;
            if (q < nq && bm[b] <= 16)
                v[b] = SBE_MAT_NTL ? __builtin_nontemporal_load(reinterpret_cast<const u32x4_ua*>(rec + s))
                                   : *reinterpret_cast<const u32x4_ua*>(rec + s);
        }
#pragma unroll
        for (int b = 0; b < kMatBatch; ++b) {
            if (q0 + b >= nq) break;
            if (bm[b] == 16) {
                *reinterpret_cast<lds_u32x4_ua*>(w + dof[b]) = v[b];
            } else if (bm[b] < 16) {
                for (uint32_t t = 0; t < bm[b]; ++t) w[dof[b] + t] = mat_byte(v[b], bo[b] + t);
            } else {
                for (uint32_t t = 0; t < (bm[b] & 0xffu); ++t) w[dof[b] + t] = rec[bo[b] + t];
            }
        }
    }
}
// A tile's descriptors, loaded one tile ahead (unconditional loads at clamped indices, so the
// compiler's waits count them exactly and the next tile's loads stay in flight during this copy)
struct MatDesc {
    uint32_t L[5], O[5];
    uint64_t r0, r1, pre, bs;
};
__device__ __forceinline__ void mat_desc_load(const MatArgs& a, uint64_t t, uint64_t nt, int lane, MatDesc& d) {
    const uint64_t tc = t < nt ? t : nt - 1;
    uint64_t i = tc * kMatTile + (uint64_t)lane;
    i = i < a.n ? i : a.n - 1;
#pragma unroll
    for (int k = 0; k < 5; ++k) {
        d.L[k] = a.view_len[5 * i + k];
        d.O[k] = a.view_off[5 * i + k];
    }
    d.r0 = a.rec_off[i];
    d.r1 = a.rec_off[i + 1];
    const uint64_t b = tc / kMatTpb;
    uint64_t j = b * kMatTpb + (uint64_t)lane;
    j = j < nt ? j : nt - 1;
    d.pre = a.tsum[j];  // used by lanes < the tile's index in its block
    d.bs = a.bsum[b];
}
__device__ __forceinline__ void mat_tile(const MatArgs& a, uint64_t t, const MatDesc& d, int lane, uint8_t* win) {
    const uint64_t i = t * kMatTile + (uint64_t)lane;
    const bool live = i < a.n;
    uint32_t L[5], O[5];
    uint64_t bytes = 0;
#pragma unroll
    for (int k = 0; k < 5; ++k) {
        L[k] = live ? d.L[k] : 0u;
        O[k] = live ? d.O[k] : 0u;
        bytes += L[k];
    }
    const uint64_t r0 = live ? d.r0 : 0ull, r1 = live ? d.r1 : 0ull;
    // base: the block's prefix, the block's tiles before this one, the wave's scan
    const uint64_t t0 = t / kMatTpb * kMatTpb;
    const uint64_t pre = (uint64_t)lane < t - t0 ? d.pre : 0ull;
    const uint64_t o = d.bs + wave_sum64(pre) + wave_incl_scan64(bytes, lane) - bytes;
    uint64_t at[6];
    at[0] = o;
#pragma unroll
    for (int k = 0; k < 5; ++k) at[k + 1] = at[k] + L[k];
    if (live) {
#pragma unroll
        for (int k = 0; k < 5; ++k) a.arena_off[5 * i + k] = at[k];
    }
    // views written: those ending within the capacity (a prefix: at[] is non-decreasing)
    int k_end = 0;
#pragma unroll
    for (int k = 0; k < 5; ++k) k_end += (live && at[k + 1] <= a.cap) ? 1 : 0;
    uint64_t fit = o;  // end of this record's written bytes
#pragma unroll
    for (int k = 0; k < 5; ++k)
        if (k < k_end) fit = at[k + 1];
    const uint8_t* rec = a.in + r0;
    const uint64_t rl = r1 - r0;
    bool done = fit == o;
    if (!done && fit - o > (uint64_t)(kMatWin - 16)) {  // larger than any window: straight to the arena
        mat_views_direct(a.arena + o, rec, rl, at, L, O, k_end, fit);
        done = true;
    }
    uint64_t start = mat_wave_min(done ? ~0ull : o);
    while (start != ~0ull) {  // uniform
        const uint64_t wbase = start - (uint64_t)((reinterpret_cast<uintptr_t>(a.arena) + start) & 15u);
        uint64_t my_end = 0;
        if (!done && fit - wbase <= (uint64_t)kMatWin) {
            mat_views_lds((mat_lds8*)win + (o - wbase), rec, rl, at, L, O, k_end);
            done = true;
            my_end = fit;
        }
        const uint64_t cend = mat_wave_max(my_end);
        __syncthreads();
        const uint64_t nch = (cend - wbase + 15) / 16;
        for (uint64_t c = (uint64_t)lane; c < nch; c += kWave) {
            const uint64_t x0 = wbase + 16 * c;  // arena + x0 is 16-byte aligned
            if (x0 >= start && x0 + 16 <= cend) {
                const u32x4 v = *(const __attribute__((address_space(3))) u32x4*)(win + 16 * c);
                __builtin_nontemporal_store(v, reinterpret_cast<u32x4*>(a.arena + x0));
            } else {
                for (uint64_t x = x0 < start ? start : x0; x < x0 + 16 && x < cend; ++x) a.arena[x] = win[x - wbase];
            }
        }
        __syncthreads();
        start = mat_wave_min(done ? ~0ull : o);
    }
}
// SBE_MAT_PERSIST (A/B builds): 1 = a persistent grid (occupancy x CUs) whose waves loop over the
// tiles with the next tile's descriptors in flight: 0.201 ms against 0.164 for one workgroup per
// tile (profiles/r06_ab_mat6.log; a tile's loads then wait behind the previous tile's stores)
#ifndef SBE_MAT_PERSIST
#define SBE_MAT_PERSIST 0
#endif
__global__ __launch_bounds__(kWave, SBE_MAT_MINW) void mat_copy(MatArgs a, uint64_t nt) {
    __shared__ __attribute__((aligned(16))) uint8_t win[kMatWin];
    const int lane = threadIdx.x;
    MatDesc d;
    mat_desc_load(a, blockIdx.x, nt, lane, d);
    if (!SBE_MAT_PERSIST) {
        mat_tile(a, blockIdx.x, d, lane, win);
        return;
    }
    for (uint64_t t = blockIdx.x; t < nt; t += gridDim.x) {
        MatDesc dn;
        mat_desc_load(a, t + gridDim.x, nt, lane, dn);
        mat_tile(a, t, d, lane, win);
        d = dn;
    }
}

// ------------------------------------------------------------------------------------------
// Gather of encoded shards to one rank: the {bytes, n} of every rank go round in
// one ncclAllGather, then the shards move in one group of ncclSend / ncclRecv at the prefix
// offsets, and the root rebases each received offset array by its shard's byte prefix.
// ------------------------------------------------------------------------------------------
__global__ void shard_size_put(uint64_t* dst, const uint64_t* out_off, uint64_t n, uint64_t cap, uint64_t off_cap) {
    if (threadIdx.x == 0) {
        dst[0] = out_off[n];
        dst[1] = n;
        dst[2] = cap;      // the root's receive capacity in bytes (0 elsewhere)
        dst[3] = off_cap;  // the root's dst_off entries (0 elsewhere)
    }
}

__global__ void u64_put(uint64_t* dst, uint64_t v) {
    if (threadIdx.x == 0) *dst = v;
}

__global__ __launch_bounds__(256) void offsets_rebase(uint64_t* dst, const uint64_t* src, uint64_t count, uint64_t base) {
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < count; i += stride) dst[i] = src[i] + base;
}


// One encode request, whatever the layout (the C entry points fill it).
struct EncReq {
    const uint8_t* arena;
    const uint32_t* str_off;
    const uint32_t* str_len;
    const uint64_t* ts;   // timestamp / sequence
    const uint32_t* tid;  // Lite topicId
    uint32_t tmpl;
    int64_t term_id, sess_id;
};

size_t enc_workspace_size(uint64_t n) {  // the smallest tile shape's (the most tiles)
    const uint64_t sbs = (n + kSbRecMin - 1) / kSbRecMin;
    const uint64_t tiles = sbs * kTilesPerSb;
    return (size_t)(16 * (tiles + sbs) + kSinkBytes + 16);
}

template <class LY, bool kPacked, int kLen>
void enc_launch_k(const EncArgs& a, uint64_t sbs, uint64_t tiles, hipStream_t s) {
    const uint64_t grid = pack_grid(reinterpret_cast<const void*>(&sbe_enc_pack<LY, kPacked, kLen>), tiles);
    hipLaunchKernelGGL((sbe_enc_sums<LY, kPacked, kLen>), dim3((uint32_t)sbs), dim3(kSbThreads), 0, s, a);
    hipEvent_t e0, e1;
    prof_slot(0, &e0, &e1);
    hipExtLaunchKernelGGL((sbe_enc_pack<LY, kPacked, kLen>), dim3((uint32_t)grid), dim3(kWave), 0, s, e0, e1, 0, a);
    prof_commit(0, e0);
}

// Argument checks shared by the batch and serve entry points (the workspace aside).
template <class LY>
int enc_check(const EncReq& q, uint64_t n, uint32_t flags, const uint8_t* out, const uint64_t* out_off) {
    if (!out_off) return SBE_EINVAL;
    if (flags & ~(SBE_ENC_REF_TRUNCATE8 | SBE_ENC_PUBLISH_TOPIC)) return SBE_EINVAL;
    if (!LY::kTM && flags) return SBE_EINVAL;
    if ((flags & SBE_ENC_PUBLISH_TOPIC) && ((flags & SBE_ENC_REF_TRUNCATE8) || LY::kPre)) return SBE_EINVAL;
    if (n == 0) return SBE_OK;
    if (!q.str_len || !q.ts || !q.arena || !out) return SBE_EINVAL;
    if ((reinterpret_cast<uintptr_t>(out) & 15u) || (reinterpret_cast<uintptr_t>(out_off) & 7u)) return SBE_EINVAL;
    if ((n + LY::kRpt - 1) / LY::kRpt > kMaxTiles) return SBE_EINVAL;
    return SBE_OK;
}

inline int enc_len_mode(uint32_t flags) {
    return (flags & SBE_ENC_REF_TRUNCATE8) ? kLenRef : (flags & SBE_ENC_PUBLISH_TOPIC) ? kLenPub : kLenWire;
}

// Argument checks, workspace carving and the two launches (sums, pack) of one encode call.
template <class LY>
int enc_launch(const EncReq& q, uint64_t n, uint64_t ts_default, uint32_t flags, uint8_t* out, uint64_t out_capacity,
               uint64_t* out_off, uint8_t* status, void* workspace, size_t workspace_bytes, void* stream) {
    if (const int rc = enc_check<LY>(q, n, flags, out, out_off)) return rc;
    hipStream_t s = reinterpret_cast<hipStream_t>(stream);
    if (n == 0) return record_hip(hipMemsetAsync(out_off, 0, sizeof(uint64_t), s));
    const uint64_t sbs = (n + LY::kSbRec - 1) / LY::kSbRec;
    const uint64_t tiles = (n + LY::kRpt - 1) / LY::kRpt;
    if (!workspace || workspace_bytes < enc_workspace_size(n)) return SBE_ENOSPC;
    if (reinterpret_cast<uintptr_t>(workspace) & 15u) return SBE_EINVAL;
    uint64_t* ws = static_cast<uint64_t*>(workspace);
    EncArgs a{q.arena, q.str_off, q.str_len, q.ts, q.tid, q.tmpl, q.term_id, q.sess_id, n, ts_default,
              out,     out_capacity, out_off, status, ws, ws + 2 * sbs * kTilesPerSb,
              reinterpret_cast<uint8_t*>(ws + 2 * sbs * (kTilesPerSb + 1))};
    const bool packed = q.str_off == nullptr;
    const int len = enc_len_mode(flags);
    if constexpr (LY::kTM) {
        if (packed) {
            if (len == kLenWire) enc_launch_k<LY, true, kLenWire>(a, sbs, tiles, s);
            else if (len == kLenRef) enc_launch_k<LY, true, kLenRef>(a, sbs, tiles, s);
            else if constexpr (LY::kPre == 0) enc_launch_k<LY, true, kLenPub>(a, sbs, tiles, s);
        } else {
            if (len == kLenWire) enc_launch_k<LY, false, kLenWire>(a, sbs, tiles, s);
            else if (len == kLenRef) enc_launch_k<LY, false, kLenRef>(a, sbs, tiles, s);
            else if constexpr (LY::kPre == 0) enc_launch_k<LY, false, kLenPub>(a, sbs, tiles, s);
        }
    } else {
        if (packed) enc_launch_k<LY, true, kLenWire>(a, sbs, tiles, s);
        else enc_launch_k<LY, false, kLenWire>(a, sbs, tiles, s);
    }
    return record_hip(hipGetLastError());
}

// Argument checks of a decode call (batch and serve entry points).
int dec_check(const uint8_t* in, const uint64_t* rec_off, uint64_t n, uint32_t mode, const sbe_decoded* out) {
    if (mode != SBE_DEC_PARSE_MESSAGE && mode != SBE_DEC_ON_EGRESS && mode != SBE_DEC_LITE) return SBE_EINVAL;
    if (n == 0) return SBE_OK;
    if (!in || !rec_off || !out || !out->status || !out->flags || !out->hdr || !out->ts || !out->view_off ||
        !out->view_len)
        return SBE_EINVAL;
    if ((reinterpret_cast<uintptr_t>(in) & 15u) || (reinterpret_cast<uintptr_t>(rec_off) & 7u) ||
        (reinterpret_cast<uintptr_t>(out->hdr) & 7u) || (reinterpret_cast<uintptr_t>(out->ts) & 7u) ||
        (reinterpret_cast<uintptr_t>(out->view_off) & 3u) || (reinterpret_cast<uintptr_t>(out->view_len) & 3u))
        return SBE_EINVAL;
    if ((n + kTile - 1) / kTile > kMaxTiles) return SBE_EINVAL;
    if (mode == SBE_DEC_PARSE_MESSAGE && out->seq && (reinterpret_cast<uintptr_t>(out->seq) & 7u)) return SBE_EINVAL;
    return SBE_OK;
}

// ------------------------------------------------------------------------------------------
// Serve kernel: one resident wave that polls a page-locked request slot (sbecodec.h, "small-batch
// serve kernel").  A request is one EncArgs or DecArgs; the wave runs the same device code as the
// batch kernels over the whole batch (decode: dec_tile over its tiles; encode: the pack loop as
// workgroup 0 of 1 over one chunk, whose running offsets make the tile sums unnecessary), then
// publishes done_seq.
// ------------------------------------------------------------------------------------------
enum : uint32_t {
    kSvShutdown = 1,
    kSvDecParse, kSvDecEgress, kSvDecLite,
    kSvTmWire, kSvTmRef, kSvTmPub, kSvTmsWire, kSvTmsRef, kSvLite2, kSvLite3
};

// op | kSvPlanned: an encode whose tile sums the host supplied (e.tsum / e.bsum as sbe_enc_sums
// writes them), run by the tile loop over the request's workgroups
constexpr uint32_t kSvPlanned = 0x100u;
struct ServeReq {
    uint32_t op;
    uint32_t inl;  // bytes of the slot's inline area to copy to the device scratch before running
    uint32_t nwg;  // workgroups that take part (1: the leader alone)
    uint32_t tag;  // the request's sequence number (a follower checks its copy against the header)
    EncArgs e;
    DecArgs d;
};
constexpr int kReqWords = (int)(sizeof(ServeReq) / 4);
static_assert(sizeof(ServeReq) % 4 == 0 && kReqWords <= kWave, "a request is read one dword per lane");

// Host-written words and device-written words on separate 64-B lines.
// Inline inputs (sbe_serve_*_host): the host copies a request's inputs into the slot, the wave
// copies them to device scratch (the first KiB in the same round trip as the request) and runs
// from there, so the kernel's dependent reads (offsets, then records; lengths, then strings) hit
// the L2 instead of crossing PCIe.
constexpr uint32_t kServeInline = SBE_SERVE_INLINE_BYTES;
static_assert(kServeInline % 1024 == 0, "inline area: whole 1 KiB wave loads");
struct ServeSlot {
    alignas(64) uint32_t req_seq;  // host → device: sequence number of the posted request
    alignas(64) uint32_t done_seq; // device → host: the last request completed
    uint32_t alive;                // 1 from the host's launch until the kernel's exit
    alignas(64) ServeReq req;
    alignas(64) uint8_t inl[kServeInline];
};

// Device-memory side of a multi-workgroup server: the leader (workgroup 0) polls the host slot and
// republishes a request for the followers here (an L2 poll instead of a PCIe one); arrive counts
// the workgroups done with the current request, exited the workgroups gone at an idle exit.
// hdr packs seq (bits 0-31), nwg (32-47) and op (48-63) in one word, so a follower learns with one
// atomic load whether it takes part; only those that do read req, which cannot change before they
// have counted themselves in arrive.
struct ServeDev {
    alignas(64) uint64_t hdr;
    uint32_t quit;  // the launch epoch whose leader went idle (its followers exit)
    alignas(64) uint32_t arrive;
    uint32_t exited;
    alignas(64) ServeReq req;
};

union ServeLds {
    PackLds<LayTM, true> tm;
    PackLds<LayTMS, true> tms;
    PackLds<LayL2, true> l2;
    PackLds<LayL3, true> l3;
    uint32_t win[kWin / 4];
};

__device__ __forceinline__ uint32_t sys_acquire(const uint32_t* p) {
    return __hip_atomic_load(p, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_SYSTEM);
}
// Polls are relaxed loads that bypass the non-coherent caches; the acquire (its cache
// invalidation) is paid once, when the value has changed: an acquiring load on every poll
// invalidates the L2 each time, which a resident server must not do to the kernels around it.
__device__ __forceinline__ uint32_t sys_poll(const uint32_t* p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}
__device__ __forceinline__ void sys_release(uint32_t* p, uint32_t v) {
    __hip_atomic_store(p, v, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}

template <uint32_t kMode>
__device__ __forceinline__ void serve_decode(const DecArgs& a, uint32_t* win, uint32_t first, uint32_t G) {
    for (uint64_t t = first; t * kTile < a.n; t += G) {
        dec_tile<kMode, kWin, true>(a, t, win);
        wsync();
    }
}

template <class LY, int kLen>
__device__ __forceinline__ void serve_encode(const EncArgs& a, PackLds<LY, true>& L, bool planned, uint32_t first,
                                             uint32_t G) {
    if (a.n == 0) {
        if (threadIdx.x == 0 && first == 0) a.out_off[0] = 0;
        return;
    }
    if (planned) {  // the host's tile sums: the batch kernel's tile loop over the request's workgroups
        enc_pack_run<LY, true, kLen>(a, first, G, L);
        return;
    }
    // one chunk (the zero prefix of tile 0 is the only base), chunks spread over the wave
    enc_pack_run_vt<LY, true, kLen>(a, 0, 1, L, 0, true);
}

#ifdef SBE_SERVE_PROF
// Debug builds only: per-request phase times of the serve kernel, s_memrealtime ticks (10 ns)
// summed over requests: [0] request seen → request words in registers, [1] → inline inputs in
// scratch, [2] → body issued, [3] → done_seq stored (the release waits for every store), [4] count;
// inside a served decode tile, from its start: [5] offsets read, [6] window in LDS, [7] parsed,
// [8] descriptor stores issued (read with sbe_debug_serve_prof)
#define SBE_SV_T(x) const uint64_t x = __builtin_amdgcn_s_memrealtime()
#else
#define SBE_SV_T(x)
#endif

// idle_ticks: s_memrealtime ticks (100 MHz) without a request before the leader exits; scratch:
// the device copy of the inline area; dev / epoch: the followers' mailbox and this launch's number.
// Workgroup 0 (the leader) polls the host slot.  A request for more than one workgroup is
// republished in dev; every taking part workgroup runs its share (decode: tiles first, first + G,
// ...; planned encode: the tile loop), makes its stores visible system-wide and counts itself in
// dev->arrive; the last one resets the count and publishes done_seq.  On an idle exit the leader
// posts its epoch in dev->quit, and the last workgroup to leave clears the host's alive flag.
__global__ __launch_bounds__(kWave, 1) void sbe_serve_kernel(ServeSlot* slot, uint64_t idle_ticks, uint8_t* scratch,
                                                             ServeDev* dev, uint32_t epoch) {
    __shared__ ServeLds lds;
    const int lane = threadIdx.x;
    const uint32_t wg = blockIdx.x;
    const bool leader = wg == 0;
    auto dev_hdr = [&]() -> uint64_t {  // relaxed: the caller fences once it sees a change
        const uint64_t h = __hip_atomic_load(&dev->hdr, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        return uniform64(h);
    };
    uint32_t last = leader ? __builtin_amdgcn_readfirstlane(sys_acquire(&slot->done_seq)) : (uint32_t)dev_hdr();
    uint64_t t_idle = __builtin_amdgcn_s_memrealtime();
    for (;;) {
        uint32_t seq;
        uint64_t h = 0;
        if (leader) {
            seq = __builtin_amdgcn_readfirstlane(sys_poll(&slot->req_seq));
            if (seq == last) {
                if (__builtin_amdgcn_s_memrealtime() - t_idle > idle_ticks) {
                    if (lane == 0) __hip_atomic_store(&dev->quit, epoch, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
                    break;
                }
                __builtin_amdgcn_s_sleep(2);
                continue;
            }
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");  // the request and inputs, fresh
        } else {
            h = dev_hdr();
            seq = (uint32_t)h;
            if (seq == last) {
                if (__builtin_amdgcn_readfirstlane(
                        __hip_atomic_load(&dev->quit, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) == epoch)
                    break;
                __builtin_amdgcn_s_sleep(16);
                continue;
            }
            // system scope: the inputs may have come from the host or a copy engine since
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
        }
        SBE_SV_T(t0);
        union {
            ServeReq r;
            uint32_t u[kReqWords];
        } q;
        if (leader) {
            // the request, one dword per lane (after the acquire: fresh from host memory)
            const uint32_t* w = reinterpret_cast<const uint32_t*>(&slot->req);
            const uint32_t v = lane < kReqWords ? __builtin_nontemporal_load(w + lane) : 0u;
            typedef __attribute__((address_space(1))) u32x4 g_v4;
            const g_v4* inl = reinterpret_cast<const g_v4*>(reinterpret_cast<uintptr_t>(slot->inl));
            const u32x4 i0 = inl[lane];  // the first KiB of inline input, with the request (unused if none)
#pragma unroll
            for (int i = 0; i < kReqWords; ++i) q.u[i] = __builtin_amdgcn_readlane(v, i);
            if (q.r.inl) {
                g_v4* dst = reinterpret_cast<g_v4*>(reinterpret_cast<uintptr_t>(scratch));
                if (16u * (uint32_t)lane < q.r.inl) dst[lane] = i0;
                for (uint32_t o = 1024u + 16u * (uint32_t)lane; o < q.r.inl; o += 1024u) dst[o >> 4] = inl[o >> 4];
                // the wave's stores complete (this XCD's L2 holds them) and no line of an earlier
                // request stays in the CU's vector L1, before its reads of the scratch
                __builtin_amdgcn_s_waitcnt(0);
                __asm__ volatile("buffer_inv sc0" ::: "memory");
            }
            if (q.r.nwg > 1) {  // republish for the followers (agent-scope release: other XCDs' L2s)
                uint32_t* dw = reinterpret_cast<uint32_t*>(&dev->req);
                if (lane < kReqWords) dw[lane] = v;
                const uint64_t hv = (uint64_t)seq | ((uint64_t)(q.r.nwg & 0xffffu) << 32) | ((uint64_t)(q.r.op & 0xffffu) << 48);
                if (lane == 0) __hip_atomic_store(&dev->hdr, hv, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
            }
        } else {
            const uint32_t hn = (uint32_t)(h >> 32) & 0xffffu, hop = (uint32_t)(h >> 48);
            if (wg < hn) {  // taking part: the request stays put until this workgroup has arrived
                const uint32_t* w = reinterpret_cast<const uint32_t*>(&dev->req);
                const uint32_t v = lane < kReqWords ? w[lane] : 0u;
#pragma unroll
                for (int i = 0; i < kReqWords; ++i) q.u[i] = __builtin_amdgcn_readlane(v, i);
                if (q.r.tag != seq) {  // not the request the header names: take no part
                    q.r.op = hop;
                    q.r.nwg = 0;
                }
            } else {
                q.r.op = hop;
                q.r.nwg = hn;
            }
        }
        last = seq;
        SBE_SV_T(t1);
        SBE_SV_T(t2);
        const uint32_t G = leader && q.r.nwg == 0 ? 1u : q.r.nwg;
        const uint32_t op = q.r.op & ~kSvPlanned;
        const bool planned = (q.r.op & kSvPlanned) != 0;
        if (wg < G) {
            switch (op) {
                case kSvDecParse: serve_decode<SBE_DEC_PARSE_MESSAGE>(q.r.d, lds.win, wg, G); break;
                case kSvDecEgress: serve_decode<SBE_DEC_ON_EGRESS>(q.r.d, lds.win, wg, G); break;
                case kSvDecLite: serve_decode<SBE_DEC_LITE>(q.r.d, lds.win, wg, G); break;
                case kSvTmWire: serve_encode<LayTM, kLenWire>(q.r.e, lds.tm, planned, wg, G); break;
                case kSvTmRef: serve_encode<LayTM, kLenRef>(q.r.e, lds.tm, planned, wg, G); break;
                case kSvTmPub: serve_encode<LayTM, kLenPub>(q.r.e, lds.tm, planned, wg, G); break;
                case kSvTmsWire: serve_encode<LayTMS, kLenWire>(q.r.e, lds.tms, planned, wg, G); break;
                case kSvTmsRef: serve_encode<LayTMS, kLenRef>(q.r.e, lds.tms, planned, wg, G); break;
                case kSvLite2: serve_encode<LayL2, kLenWire>(q.r.e, lds.l2, planned, wg, G); break;
                case kSvLite3: serve_encode<LayL3, kLenWire>(q.r.e, lds.l3, planned, wg, G); break;
                default: break;
            }
            wsync();
            SBE_SV_T(t3);
            if (G == 1) {
                // lane 0's system-scope release (an L2 write-back and a wait for every outstanding
                // store of the wave) orders all lanes' result stores before done_seq
                if (lane == 0) sys_release(&slot->done_seq, seq);
            } else {
                // this workgroup's results visible system-wide, then counted; the last one publishes
                __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
                if (lane == 0) {
                    const uint32_t old = __hip_atomic_fetch_add(&dev->arrive, 1u, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT);
                    if (old == G - 1) {
                        __hip_atomic_store(&dev->arrive, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                        sys_release(&slot->done_seq, seq);
                    }
                }
            }
#ifdef SBE_SERVE_PROF
            SBE_SV_T(t4);
            if (leader && lane == 0) {
                g_serve_prof[0] += t1 - t0;
                g_serve_prof[1] += t2 - t1;
                g_serve_prof[2] += t3 - t2;
                g_serve_prof[3] += t4 - t3;
                g_serve_prof[4] += 1;
            }
#endif
        }
        if (op == kSvShutdown) break;
        t_idle = __builtin_amdgcn_s_memrealtime();
    }
    __threadfence_system();
    if (lane == 0) {
        const uint32_t n = gridDim.x;
        const uint32_t old = n > 1 ? __hip_atomic_fetch_add(&dev->exited, 1u, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT)
                                   : 0u;
        if (old == n - 1) sys_release(&slot->alive, 0u);
    }
}

}  // namespace

struct sbe_server {
    ServeSlot* h = nullptr;  // page-locked slot, host address
    ServeSlot* d = nullptr;  // its device address
    uint64_t* ws = nullptr;  // device: zero tile sums (2 u64, never written) + the pack's sink
    ServeDev* dev = nullptr; // device: the followers' mailbox and counters
    hipStream_t stream = nullptr;
    uint32_t seq = 0;
    uint32_t nwg = 1;        // workgroups per launch
    uint64_t idle_ticks = 0;
    uint64_t requests = 0, launches = 0;
    bool failed = false;     // a request timed out or the stream failed: the slot may still hold it
};

namespace {

// device workspace: zero tile sums (16 B), the pack's sink, then the inline scratch
constexpr size_t kServeScratchOff = 16 + kSinkBytes + 16;
constexpr size_t kServeWsBytes = kServeScratchOff + kServeInline;

int serve_launch(sbe_server* s) {
    __atomic_store_n(&s->h->alive, 1u, __ATOMIC_RELEASE);
    // the exit count of the previous launch back to 0 (stream order: before the kernel starts)
    if (const int rc = record_hip(hipMemsetAsync(&s->dev->exited, 0, sizeof(uint32_t), s->stream))) return rc;
    ++s->launches;
    hipLaunchKernelGGL(sbe_serve_kernel, dim3(s->nwg), dim3(kWave), 0, s->stream, s->d, s->idle_ticks,
                       reinterpret_cast<uint8_t*>(s->ws) + kServeScratchOff, s->dev, (uint32_t)s->launches);
    return record_hip(hipGetLastError());
}

// Post one request and wait for its completion (relaunching the kernel whenever it is not running).
int serve_call(sbe_server* s, const ServeReq& r) {
    if (!s || !s->h) return SBE_EINVAL;
    if (s->failed) {
        // a request this server gave up on may still run: no new one is posted over it
        std::snprintf(g_last_error, sizeof g_last_error, "serve: an earlier request failed; destroy this server");
        return SBE_EHIP;
    }
    ServeSlot* h = s->h;
    std::memcpy(&h->req, &r, sizeof r);
    if (h->req.nwg == 0) h->req.nwg = 1;
    const uint32_t seq = ++s->seq;
    h->req.tag = seq;
    __atomic_store_n(&h->req_seq, seq, __ATOMIC_RELEASE);
    ++s->requests;
    const auto t0 = std::chrono::steady_clock::now();
    for (uint64_t spin = 0;; ++spin) {
        if (__atomic_load_n(&h->done_seq, __ATOMIC_ACQUIRE) == seq) return SBE_OK;
        if (__atomic_load_n(&h->alive, __ATOMIC_ACQUIRE) == 0) {
            // exited (idle): it may have answered just before, else start one
            if (__atomic_load_n(&h->done_seq, __ATOMIC_ACQUIRE) == seq) return SBE_OK;
            if (const int rc = serve_launch(s)) return rc;
        }
        if ((spin & 4095) == 4095) {
            const hipError_t e = hipStreamQuery(s->stream);
            if (e != hipSuccess && e != hipErrorNotReady) {
                s->failed = true;
                return record_hip(e);
            }
            if (std::chrono::steady_clock::now() - t0 > std::chrono::seconds(10)) {
                s->failed = true;
                std::snprintf(g_last_error, sizeof g_last_error, "serve request %u timed out", seq);
                return SBE_EHIP;
            }
        }
        __builtin_ia32_pause();
    }
}

template <class LY>
int serve_encode_req(sbe_server* s, const EncReq& q, uint64_t n, uint64_t ts_default, uint32_t flags, uint8_t* out,
                     uint64_t out_capacity, uint64_t* out_off, uint8_t* status, uint32_t op) {
    if (!s) return SBE_EINVAL;
    if (const int rc = enc_check<LY>(q, n, flags, out, out_off)) return rc;
    if (n > SBE_SERVE_MAX_RECORDS || (n && q.str_off)) return SBE_EINVAL;
    ServeReq r{};
    r.op = op;
    r.e = EncArgs{q.arena, nullptr, q.str_len, q.ts, q.tid, q.tmpl, q.term_id, q.sess_id, n, ts_default,
                  out, out_capacity, out_off, status, s->ws, s->ws, reinterpret_cast<uint8_t*>(s->ws + 2)};
    return serve_call(s, r);
}

// Planned encode: device-visible inputs plus the tile sums the caller computed (the layout
// sbe_enc_sums writes), run by the tile loop over up to the server's workgroups.
template <class LY>
int serve_encode_planned(sbe_server* s, const EncReq& q, uint64_t n, uint64_t ts_default, uint32_t flags,
                         uint8_t* out, uint64_t out_capacity, uint64_t* out_off, uint8_t* status,
                         const uint64_t* tile_sums, const uint64_t* sb_sums, uint32_t op) {
    if (!s) return SBE_EINVAL;
    if (const int rc = enc_check<LY>(q, n, flags, out, out_off)) return rc;
    if (n > SBE_SERVE_MAX_RECORDS || (n && (q.str_off || !tile_sums || !sb_sums))) return SBE_EINVAL;
    const uint64_t tiles = (n + LY::kRpt - 1) / LY::kRpt;
    ServeReq r{};
    r.op = op | kSvPlanned;
    r.nwg = (uint32_t)(tiles < s->nwg ? (tiles ? tiles : 1) : s->nwg);
    r.e = EncArgs{q.arena, nullptr, q.str_len, q.ts, q.tid, q.tmpl, q.term_id, q.sess_id, n, ts_default,
                  out, out_capacity, out_off, status, const_cast<uint64_t*>(tile_sums), const_cast<uint64_t*>(sb_sums),
                  reinterpret_cast<uint8_t*>(s->ws + 2)};
    return serve_call(s, r);
}

// Inline inputs: place `bytes` from host memory at offset `at` of the slot's inline area and
// return the device address they will have in the scratch.
struct Inline {
    sbe_server* s;
    uint32_t at = 0;
    bool ok = true;
    template <class T>
    const T* put(const T* src, size_t count) {
        const size_t bytes = count * sizeof(T);
        const uint32_t o = at;
        if (bytes > kServeInline || o + bytes > kServeInline) {
            ok = false;
            return nullptr;
        }
        if (bytes) std::memcpy(s->h->inl + o, src, bytes);
        at = (uint32_t)((o + bytes + 15) & ~(size_t)15);
        return reinterpret_cast<const T*>(reinterpret_cast<const uint8_t*>(s->ws) + kServeScratchOff + o);
    }
};

uint32_t serve_tm_op(bool session, uint32_t flags) {
    const int len = enc_len_mode(flags);
    if (session) return len == kLenRef ? kSvTmsRef : kSvTmsWire;
    return len == kLenRef ? kSvTmRef : len == kLenPub ? kSvTmPub : kSvTmWire;
}

// host-input encode: the packed strings, lengths, timestamps / sequences (and Lite topicIds) into
// the inline area, then the device-pointer request on the scratch copies
template <class LY>
int serve_encode_host(sbe_server* s, const EncReq& q, uint64_t n, uint64_t ts_default, uint32_t flags, uint8_t* out,
                      uint64_t out_capacity, uint64_t* out_off, uint8_t* status, uint32_t op) {
    if (!s || !s->h) return SBE_EINVAL;
    if (n > SBE_SERVE_MAX_RECORDS || (n && q.str_off)) return SBE_EINVAL;
    if (n && (!q.str_len || !q.ts)) return SBE_EINVAL;
    uint64_t sum = 0;
    for (uint64_t i = 0; i < (uint64_t)LY::kNF * n; ++i) sum += q.str_len[i];
    if (sum > kServeInline) return SBE_EINVAL;
    Inline I{s};
    EncReq d = q;
    if (n) {
        d.arena = I.put(q.arena, (size_t)sum);
        d.str_len = I.put(q.str_len, (size_t)(LY::kNF * n));
        d.ts = I.put(q.ts, (size_t)n);
        if (!LY::kTM) d.tid = I.put(q.tid, (size_t)n);
        if (!I.ok) return SBE_EINVAL;
        if (!d.arena) d.arena = reinterpret_cast<const uint8_t*>(s->ws) + kServeScratchOff;  // Σlen = 0
    }
    if (const int rc = enc_check<LY>(d, n, flags, out, out_off)) return rc;
    ServeReq r{};
    r.op = op;
    r.inl = I.at;
    r.e = EncArgs{d.arena, nullptr, d.str_len, d.ts, d.tid, d.tmpl, d.term_id, d.sess_id, n, ts_default,
                  out, out_capacity, out_off, status, s->ws, s->ws, reinterpret_cast<uint8_t*>(s->ws + 2)};
    return serve_call(s, r);
}

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

size_t sbe_encode_workspace_size(uint64_t n) { return enc_workspace_size(n); }

uint64_t sbe_encode_output_bound(uint64_t n, uint64_t string_bytes, uint32_t flags) {
    (void)flags;  // the wire length bounds the truncated one; session framing adds 32 B a record
    return string_bytes + (uint64_t)(SBE_TM_WIRE_OVERHEAD + SBE_SESSION_HDR_LEN) * n;
}

int sbe_encode_workspace_init(void* workspace, size_t workspace_bytes, void* stream) {
    if (!workspace) return SBE_EINVAL;
    return record_hip(hipMemsetAsync(workspace, 0, workspace_bytes, reinterpret_cast<hipStream_t>(stream)));
}

int sbe_encode_topic_batch(const sbe_tm_batch* in, uint64_t n, uint64_t ts_default, uint32_t flags,
                           uint8_t* out, uint64_t out_capacity, uint64_t* out_off, uint8_t* status,
                           void* workspace, size_t workspace_bytes, void* stream) {
    if (!in) return SBE_EINVAL;
    EncReq q{in->arena, in->str_off, in->str_len, in->timestamp, nullptr, 0, 0, 0};
    return enc_launch<LayTM>(q, n, ts_default, flags, out, out_capacity, out_off, status, workspace,
                             workspace_bytes, stream);
}

int sbe_encode_session_batch(const sbe_tm_batch* in, uint64_t n, uint64_t ts_default, uint32_t flags,
                             int64_t leadership_term_id, int64_t cluster_session_id, uint8_t* out,
                             uint64_t out_capacity, uint64_t* out_off, uint8_t* status, void* workspace,
                             size_t workspace_bytes, void* stream) {
    if (!in) return SBE_EINVAL;
    EncReq q{in->arena, in->str_off, in->str_len, in->timestamp, nullptr, 0, leadership_term_id, cluster_session_id};
    return enc_launch<LayTMS>(q, n, ts_default, flags, out, out_capacity, out_off, status, workspace,
                              workspace_bytes, stream);
}

uint32_t sbe_lite_fields(uint32_t template_id) {
    switch (template_id) {
        case SBE_COMMIT_OFFSET_LITE_TEMPLATE_ID: return 2;
        case SBE_ORDER_REQUEST_LITE_TEMPLATE_ID:
        case SBE_ORDER_NOTIFICATION_LITE_TEMPLATE_ID: return 3;
        default: return 0;
    }
}

uint64_t sbe_lite_output_bound(uint64_t n, uint64_t string_bytes, uint32_t template_id) {
    const uint32_t nf = sbe_lite_fields(template_id);
    return string_bytes + (uint64_t)SBE_LITE_OVERHEAD(nf ? nf : 3) * n;
}

int sbe_encode_lite_batch(const sbe_lite_batch* in, uint64_t n, uint32_t template_id, uint8_t* out,
                          uint64_t out_capacity, uint64_t* out_off, uint8_t* status, void* workspace,
                          size_t workspace_bytes, void* stream) {
    const uint32_t nf = sbe_lite_fields(template_id);
    if (!in || nf == 0) return SBE_EINVAL;
    if (n && !in->topic_id) return SBE_EINVAL;
    EncReq q{in->arena, in->str_off, in->str_len, in->sequence, in->topic_id, template_id, 0, 0};
    if (nf == 2)
        return enc_launch<LayL2>(q, n, 0, 0, out, out_capacity, out_off, status, workspace, workspace_bytes, stream);
    return enc_launch<LayL3>(q, n, 0, 0, out, out_capacity, out_off, status, workspace, workspace_bytes, stream);
}

int sbe_decode_batch_sized(const uint8_t* in, const uint64_t* rec_off, uint64_t n, uint64_t in_bytes, uint32_t mode,
                           const sbe_decoded* out, void* stream) {
    if (const int rc = dec_check(in, rec_off, n, mode, out)) return rc;
    if (n == 0) return SBE_OK;
    const uint64_t tiles = (n + kTile - 1) / kTile;
    DecArgs a{in,           rec_off,       n,
              out->status,  out->flags,    out->hdr,
              out->ts,      out->view_off, out->view_len,
              mode == SBE_DEC_PARSE_MESSAGE ? out->seq : nullptr};
    hipStream_t s = reinterpret_cast<hipStream_t>(stream);
    const dim3 grid((uint32_t)tiles), block(kWave);
    hipEvent_t e0, e1;
    prof_slot(1, &e0, &e1);
    // kernel shape by the average record size (in_bytes = 0: unknown, the 16 KiB window)
    const int shape = in_bytes > (uint64_t)kLargeAvg * n  ? 4
                      : in_bytes > (uint64_t)kWideAvg * n   ? 1
                      : in_bytes == 0                     ? 0
                      : in_bytes <= (uint64_t)kSmallAvg * n ? 3
                      : in_bytes <= (uint64_t)kMidAvg * n   ? 2
                                                          : 0;
#define SBE_DEC_LAUNCH(M)                                                                                  \
    do {                                                                                                   \
        if (shape == 4)                                                                                    \
            hipExtLaunchKernelGGL((sbe_decode_kernel<M, kWinLarge>), grid, block, 0, s, e0, e1, 0, a);     \
        else if (shape == 1)                                                                               \
            hipExtLaunchKernelGGL((sbe_decode_kernel<M, kWinWide>), grid, block, 0, s, e0, e1, 0, a);      \
        else if (shape == 2 && SBE_DEC_GROUP > 0)                                                          \
            hipExtLaunchKernelGGL((sbe_decode_group_kernel<M>),                                             \
                                  dim3((uint32_t)group_grid((const void*)sbe_decode_group_kernel<M>,       \
                                                            (n + kDecG * kTile - 1) / (kDecG * kTile))),    \
                                  dim3(kDecG * kWave), 0, s, e0, e1, 0, a);                                \
        else if (shape == 2)                                                                               \
            hipExtLaunchKernelGGL((sbe_decode_kernel<M, kWinMid>), grid, block, 0, s, e0, e1, 0, a);       \
        else if (shape == 3)                                                                               \
            hipExtLaunchKernelGGL((sbe_decode_kernel<M, kWinSmall>), grid, block, 0, s, e0, e1, 0, a);     \
        else                                                                                               \
            hipExtLaunchKernelGGL((sbe_decode_kernel<M, kWin>), grid, block, 0, s, e0, e1, 0, a);          \
    } while (0)
    if (mode == SBE_DEC_ON_EGRESS)
        SBE_DEC_LAUNCH(SBE_DEC_ON_EGRESS);
    else if (mode == SBE_DEC_LITE)
        SBE_DEC_LAUNCH(SBE_DEC_LITE);
    else
        SBE_DEC_LAUNCH(SBE_DEC_PARSE_MESSAGE);
#undef SBE_DEC_LAUNCH
    prof_commit(1, e0);
    return record_hip(hipGetLastError());
}

int sbe_decode_batch(const uint8_t* in, const uint64_t* rec_off, uint64_t n, uint32_t mode,
                     const sbe_decoded* out, void* stream) {
    return sbe_decode_batch_sized(in, rec_off, n, 0, mode, out, stream);
}

int sbe_server_create(sbe_server** srv, uint32_t idle_us) { return sbe_server_create_wide(srv, idle_us, 1); }

int sbe_server_create_wide(sbe_server** srv, uint32_t idle_us, uint32_t workgroups) {
    if (!srv) return SBE_EINVAL;
    *srv = nullptr;
    if (workgroups == 0 || workgroups > SBE_SERVE_MAX_WORKGROUPS) return SBE_EINVAL;
    sbe_server* s = new (std::nothrow) sbe_server;
    if (!s) return SBE_EINVAL;
    s->nwg = workgroups;
    s->idle_ticks = 100ull * (idle_us ? idle_us : 1000u);
    void* h = nullptr;
    void* d = nullptr;
    hipError_t e = hipHostMalloc(&h, sizeof(ServeSlot), hipHostMallocCoherent | hipHostMallocMapped);
    if (e == hipSuccess) {
        std::memset(h, 0, sizeof(ServeSlot));
        e = hipHostGetDevicePointer(&d, h, 0);
    }
    if (e == hipSuccess) e = hipMalloc(reinterpret_cast<void**>(&s->ws), kServeWsBytes);
    // the followers' mailbox uncached: their polls and the request copy bypass the XCDs' L2s, which
    // do not see each other's lines inside a kernel
    if (e == hipSuccess) e = hipExtMallocWithFlags(reinterpret_cast<void**>(&s->dev), sizeof(ServeDev), hipDeviceMallocUncached);
    if (e == hipSuccess) e = hipStreamCreateWithFlags(&s->stream, hipStreamNonBlocking);
    if (e == hipSuccess) e = hipMemsetAsync(s->ws, 0, kServeWsBytes, s->stream);
    if (e == hipSuccess) e = hipMemsetAsync(s->dev, 0, sizeof(ServeDev), s->stream);
    if (e == hipSuccess) e = hipStreamSynchronize(s->stream);
    s->h = static_cast<ServeSlot*>(h);
    s->d = static_cast<ServeSlot*>(d);
    if (e != hipSuccess) {
        const int rc = record_hip(e);
        sbe_server_destroy(s);
        return rc;
    }
    *srv = s;
    return SBE_OK;
}

int sbe_server_quiesce(sbe_server* s) {
    if (!s) return SBE_EINVAL;
    if (s->failed) {
        std::snprintf(g_last_error, sizeof g_last_error, "serve: an earlier request failed; destroy this server");
        return SBE_EHIP;
    }
    if (!s->h || !s->stream || !__atomic_load_n(&s->h->alive, __ATOMIC_ACQUIRE)) return SBE_OK;
    ServeReq r{};
    r.op = kSvShutdown;
    r.nwg = s->nwg;  // every workgroup sees it
    int rc = serve_call(s, r);
    const hipError_t e = hipStreamSynchronize(s->stream);  // the kernel has left
    if (rc == SBE_OK && e != hipSuccess) {
        s->failed = true;
        rc = record_hip(e);
    }
    return rc;
}

int sbe_server_destroy(sbe_server* s) {
    if (!s) return SBE_OK;
    int rc = SBE_OK;
    if (s->h && s->stream && !s->failed && __atomic_load_n(&s->h->alive, __ATOMIC_ACQUIRE)) {
        ServeReq r{};
        r.op = kSvShutdown;
        r.nwg = s->nwg;  // every workgroup sees it
        rc = serve_call(s, r);
    }
    if (s->stream) {
        // a bounded wait: a server that failed may hold a kernel that never leaves;
        // after idle time + 10 s its buffers are left allocated (the kernel may still touch them)
        // and the call fails instead of hanging the caller
        const auto t0 = std::chrono::steady_clock::now();
        const auto limit = std::chrono::microseconds(s->idle_ticks / 100) + std::chrono::seconds(10);
        hipError_t e;
        while ((e = hipStreamQuery(s->stream)) == hipErrorNotReady) {
            if (std::chrono::steady_clock::now() - t0 > limit) {
                std::snprintf(g_last_error, sizeof g_last_error,
                              "serve kernel still running %lld us after shutdown: its buffers are left allocated",
                              (long long)std::chrono::duration_cast<std::chrono::microseconds>(limit).count());
                delete s;
                return SBE_EHIP;
            }
            std::this_thread::sleep_for(std::chrono::microseconds(50));
        }
        if (rc == SBE_OK && e != hipSuccess) rc = record_hip(e);
        (void)hipStreamDestroy(s->stream);
    }
    if (s->ws) (void)hipFree(s->ws);
    if (s->dev) (void)hipFree(s->dev);
    if (s->h) (void)hipHostFree(s->h);
    delete s;
    return rc;
}

#ifdef SBE_SERVE_PROF
int sbe_debug_serve_prof(uint64_t* out16) {
    hipError_t e = hipMemcpyFromSymbol(out16, HIP_SYMBOL(g_serve_prof), 16 * sizeof(uint64_t));
    if (e == hipSuccess) {
        const uint64_t z[16] = {};
        e = hipMemcpyToSymbol(HIP_SYMBOL(g_serve_prof), z, sizeof z);
    }
    return record_hip(e);
}
#endif

#ifdef SBE_VT_GUARD
// debug builds: the virtual-tile guard record (16 u64; [0] = 0 when nothing was caught), then cleared
int sbe_debug_vt_guard(uint64_t* out16) {
    hipError_t e = hipMemcpyFromSymbol(out16, HIP_SYMBOL(g_vt_guard), 16 * sizeof(uint64_t));
    if (e == hipSuccess) {
        const uint64_t z[16] = {};
        e = hipMemcpyToSymbol(HIP_SYMBOL(g_vt_guard), z, sizeof z);
    }
    return record_hip(e);
}
#endif

int sbe_server_stats(const sbe_server* s, uint64_t* requests, uint64_t* launches) {
    if (!s) return SBE_EINVAL;
    if (requests) *requests = s->requests;
    if (launches) *launches = s->launches;
    return SBE_OK;
}

int sbe_serve_encode_topic(sbe_server* srv, const sbe_tm_batch* in, uint64_t n, uint64_t ts_default, uint32_t flags,
                           uint8_t* out, uint64_t out_capacity, uint64_t* out_off, uint8_t* status) {
    if (!in) return SBE_EINVAL;
    EncReq q{in->arena, in->str_off, in->str_len, in->timestamp, nullptr, 0, 0, 0};
    return serve_encode_req<LayTM>(srv, q, n, ts_default, flags, out, out_capacity, out_off, status,
                                   serve_tm_op(false, flags));
}

int sbe_serve_encode_session(sbe_server* srv, const sbe_tm_batch* in, uint64_t n, uint64_t ts_default,
                             uint32_t flags, int64_t leadership_term_id, int64_t cluster_session_id, uint8_t* out,
                             uint64_t out_capacity, uint64_t* out_off, uint8_t* status) {
    if (!in) return SBE_EINVAL;
    EncReq q{in->arena, in->str_off, in->str_len, in->timestamp, nullptr, 0, leadership_term_id, cluster_session_id};
    return serve_encode_req<LayTMS>(srv, q, n, ts_default, flags, out, out_capacity, out_off, status,
                                    serve_tm_op(true, flags));
}

int sbe_serve_encode_lite(sbe_server* srv, const sbe_lite_batch* in, uint64_t n, uint32_t template_id, uint8_t* out,
                          uint64_t out_capacity, uint64_t* out_off, uint8_t* status) {
    const uint32_t nf = sbe_lite_fields(template_id);
    if (!in || nf == 0) return SBE_EINVAL;
    if (n && !in->topic_id) return SBE_EINVAL;
    EncReq q{in->arena, in->str_off, in->str_len, in->sequence, in->topic_id, template_id, 0, 0};
    if (nf == 2)
        return serve_encode_req<LayL2>(srv, q, n, 0, 0, out, out_capacity, out_off, status, kSvLite2);
    return serve_encode_req<LayL3>(srv, q, n, 0, 0, out, out_capacity, out_off, status, kSvLite3);
}


int sbe_serve_encode_topic_host(sbe_server* srv, const sbe_tm_batch* in, uint64_t n, uint64_t ts_default,
                                uint32_t flags, uint8_t* out, uint64_t out_capacity, uint64_t* out_off,
                                uint8_t* status) {
    if (!in) return SBE_EINVAL;
    EncReq q{in->arena, in->str_off, in->str_len, in->timestamp, nullptr, 0, 0, 0};
    return serve_encode_host<LayTM>(srv, q, n, ts_default, flags, out, out_capacity, out_off, status,
                                    serve_tm_op(false, flags));
}

int sbe_serve_encode_session_host(sbe_server* srv, const sbe_tm_batch* in, uint64_t n, uint64_t ts_default,
                                  uint32_t flags, int64_t leadership_term_id, int64_t cluster_session_id,
                                  uint8_t* out, uint64_t out_capacity, uint64_t* out_off, uint8_t* status) {
    if (!in) return SBE_EINVAL;
    EncReq q{in->arena, in->str_off, in->str_len, in->timestamp, nullptr, 0, leadership_term_id, cluster_session_id};
    return serve_encode_host<LayTMS>(srv, q, n, ts_default, flags, out, out_capacity, out_off, status,
                                     serve_tm_op(true, flags));
}

int sbe_serve_encode_lite_host(sbe_server* srv, const sbe_lite_batch* in, uint64_t n, uint32_t template_id,
                               uint8_t* out, uint64_t out_capacity, uint64_t* out_off, uint8_t* status) {
    const uint32_t nf = sbe_lite_fields(template_id);
    if (!in || nf == 0) return SBE_EINVAL;
    if (n && !in->topic_id) return SBE_EINVAL;
    EncReq q{in->arena, in->str_off, in->str_len, in->sequence, in->topic_id, template_id, 0, 0};
    if (nf == 2) return serve_encode_host<LayL2>(srv, q, n, 0, 0, out, out_capacity, out_off, status, kSvLite2);
    return serve_encode_host<LayL3>(srv, q, n, 0, 0, out, out_capacity, out_off, status, kSvLite3);
}

int sbe_serve_encode_topic_planned(sbe_server* srv, const sbe_tm_batch* in, uint64_t n, uint64_t ts_default,
                                   uint32_t flags, uint8_t* out, uint64_t out_capacity, uint64_t* out_off,
                                   uint8_t* status, const uint64_t* tile_sums, const uint64_t* sb_sums) {
    if (!in) return SBE_EINVAL;
    EncReq q{in->arena, in->str_off, in->str_len, in->timestamp, nullptr, 0, 0, 0};
    return serve_encode_planned<LayTM>(srv, q, n, ts_default, flags, out, out_capacity, out_off, status, tile_sums,
                                       sb_sums, serve_tm_op(false, flags));
}

int sbe_serve_encode_session_planned(sbe_server* srv, const sbe_tm_batch* in, uint64_t n, uint64_t ts_default,
                                     uint32_t flags, int64_t leadership_term_id, int64_t cluster_session_id,
                                     uint8_t* out, uint64_t out_capacity, uint64_t* out_off, uint8_t* status,
                                     const uint64_t* tile_sums, const uint64_t* sb_sums) {
    if (!in) return SBE_EINVAL;
    EncReq q{in->arena, in->str_off, in->str_len, in->timestamp, nullptr, 0, leadership_term_id, cluster_session_id};
    return serve_encode_planned<LayTMS>(srv, q, n, ts_default, flags, out, out_capacity, out_off, status, tile_sums,
                                        sb_sums, serve_tm_op(true, flags));
}

int sbe_serve_encode_lite_planned(sbe_server* srv, const sbe_lite_batch* in, uint64_t n, uint32_t template_id,
                                  uint8_t* out, uint64_t out_capacity, uint64_t* out_off, uint8_t* status,
                                  const uint64_t* tile_sums, const uint64_t* sb_sums) {
    const uint32_t nf = sbe_lite_fields(template_id);
    if (!in || nf == 0) return SBE_EINVAL;
    if (n && !in->topic_id) return SBE_EINVAL;
    EncReq q{in->arena, in->str_off, in->str_len, in->sequence, in->topic_id, template_id, 0, 0};
    if (nf == 2)
        return serve_encode_planned<LayL2>(srv, q, n, 0, 0, out, out_capacity, out_off, status, tile_sums, sb_sums,
                                           kSvLite2);
    return serve_encode_planned<LayL3>(srv, q, n, 0, 0, out, out_capacity, out_off, status, tile_sums, sb_sums,
                                       kSvLite3);
}

uint32_t sbe_encode_tile_records(uint32_t layout) {
    switch (layout) {
        case SBE_LAYOUT_TOPIC: return LayTM::kRpt;
        case SBE_LAYOUT_SESSION: return LayTMS::kRpt;
        case SBE_LAYOUT_LITE: return LayL2::kRpt;
        default: return 0;
    }
}

int sbe_serve_decode_host(sbe_server* srv, const uint8_t* in, const uint64_t* rec_off, uint64_t n, uint32_t mode,
                          const sbe_decoded* out) {
    if (!srv || !srv->h) return SBE_EINVAL;
    if (n > SBE_SERVE_MAX_RECORDS) return SBE_EINVAL;
    if (n == 0) return mode <= SBE_DEC_LITE ? SBE_OK : SBE_EINVAL;
    if (!in || !rec_off) return SBE_EINVAL;
    const uint64_t lo = rec_off[0], bytes = rec_off[n] - lo;
    const uint64_t o_data = (8 * (n + 1) + 15) & ~15ull;
    if (rec_off[n] < lo || o_data + bytes > kServeInline) return SBE_EINVAL;
    uint64_t* ro = reinterpret_cast<uint64_t*>(srv->h->inl);
    for (uint64_t i = 0; i <= n; ++i) ro[i] = rec_off[i] - lo;
    if (bytes) std::memcpy(srv->h->inl + o_data, in + lo, (size_t)bytes);
    const uint8_t* scr = reinterpret_cast<const uint8_t*>(srv->ws) + kServeScratchOff;
    if (const int rc = dec_check(scr + o_data, reinterpret_cast<const uint64_t*>(scr), n, mode, out)) return rc;
    ServeReq r{};
    r.op = mode == SBE_DEC_ON_EGRESS ? kSvDecEgress : mode == SBE_DEC_LITE ? kSvDecLite : kSvDecParse;
    r.inl = (uint32_t)(o_data + bytes);
    r.nwg = (uint32_t)std::min<uint64_t>(srv->nwg, (n + kTile - 1) / kTile);
    r.d = DecArgs{scr + o_data, reinterpret_cast<const uint64_t*>(scr), n, out->status, out->flags, out->hdr,
                  out->ts, out->view_off, out->view_len, mode == SBE_DEC_PARSE_MESSAGE ? out->seq : nullptr};
    return serve_call(srv, r);
}

int sbe_serve_decode(sbe_server* srv, const uint8_t* in, const uint64_t* rec_off, uint64_t n, uint32_t mode,
                     const sbe_decoded* out) {
    if (!srv) return SBE_EINVAL;
    if (const int rc = dec_check(in, rec_off, n, mode, out)) return rc;
    if (n > SBE_SERVE_MAX_RECORDS) return SBE_EINVAL;
    if (n == 0) return SBE_OK;
    ServeReq r{};
    r.op = mode == SBE_DEC_ON_EGRESS ? kSvDecEgress : mode == SBE_DEC_LITE ? kSvDecLite : kSvDecParse;
    r.nwg = (uint32_t)std::min<uint64_t>(srv->nwg, (n + kTile - 1) / kTile);
    r.d = DecArgs{in,          rec_off,      n,           out->status,
                  out->flags,  out->hdr,     out->ts,     out->view_off,
                  out->view_len, mode == SBE_DEC_PARSE_MESSAGE ? out->seq : nullptr};
    return serve_call(srv, r);
}

int sbe_eval_sequence_numbers(const uint8_t* in, const uint64_t* rec_off, uint64_t n, const sbe_decoded* dec,
                              uint64_t* seq, void* stream) {
    if (n == 0) return SBE_OK;
    if (!in || !rec_off || !dec || !dec->status || !dec->flags || !dec->view_off || !dec->view_len || !seq)
        return SBE_EINVAL;
    if ((reinterpret_cast<uintptr_t>(rec_off) & 7u) || (reinterpret_cast<uintptr_t>(seq) & 7u) ||
        (reinterpret_cast<uintptr_t>(dec->view_off) & 3u) || (reinterpret_cast<uintptr_t>(dec->view_len) & 3u))
        return SBE_EINVAL;
    SeqArgs a{in, rec_off, n, dec->status, dec->flags, dec->view_off, dec->view_len, seq};
    const uint64_t blocks = ((n + 15) / 16 + 255) / 256;  // 16 records per thread
    hipLaunchKernelGGL(sbe_seqnum_kernel, dim3((uint32_t)(blocks < 65536 ? blocks : 65536)), dim3(256), 0,
                       reinterpret_cast<hipStream_t>(stream), a);
    return record_hip(hipGetLastError());
}

size_t sbe_materialize_workspace_size(uint64_t n) {
    return (size_t)(8 * ((n + kMatBlk - 1) / kMatBlk) + 8 * ((n + kMatTile - 1) / kMatTile) + 32);
}

int sbe_materialize_views(const uint8_t* in, const uint64_t* rec_off, uint64_t n, const sbe_decoded* dec,
                          uint8_t* arena, uint64_t arena_capacity, uint64_t* arena_off, void* workspace,
                          size_t workspace_bytes, void* stream) {
    hipStream_t s = reinterpret_cast<hipStream_t>(stream);
    if (!arena_off) return SBE_EINVAL;
    if (n == 0) return record_hip(hipMemsetAsync(arena_off, 0, 8, s));
    if (!in || !rec_off || !dec || !dec->status || !dec->view_off || !dec->view_len || !workspace) return SBE_EINVAL;
    if (!arena && arena_capacity) return SBE_EINVAL;
    if (workspace_bytes < sbe_materialize_workspace_size(n)) return SBE_ENOSPC;
    const uint64_t nb = (n + kMatBlk - 1) / kMatBlk;      // mat_sums blocks
    const uint64_t nt = (n + kMatTile - 1) / kMatTile;    // copy waves
    if (nt > 0xffffffffull) return SBE_EINVAL;
    uint64_t* bsum = reinterpret_cast<uint64_t*>((reinterpret_cast<uintptr_t>(workspace) + 15) & ~(uintptr_t)15);
    MatArgs a{in, rec_off, n, dec->status, dec->view_off, dec->view_len, arena, arena_capacity, arena_off, bsum, bsum + nb};
    hipLaunchKernelGGL(mat_sums, dim3((uint32_t)nb), dim3(kMatBlk), 0, s, a);
    hipLaunchKernelGGL(mat_scan_blocks, dim3(1), dim3(kMatBlk), 0, s, a, nb);
    const uint64_t g = SBE_MAT_PERSIST ? pack_grid(reinterpret_cast<const void*>(&mat_copy), nt) : nt;
    hipLaunchKernelGGL(mat_copy, dim3((uint32_t)g), dim3(kWave), 0, s, a, nt);
    return record_hip(hipGetLastError());
}

size_t sbe_reassemble_workspace_size(uint64_t n) {
    // block aggregates / scan elements, sizes, first / last fragment per message
    return (size_t)(2 * n * sizeof(FragScan) + 3 * 8 * (n + 1) + 5 * 16);
}

int sbe_reassemble_fragments(const uint8_t* in, const uint64_t* frag_off, const uint8_t* flags, uint64_t n,
                             uint8_t* out, uint64_t* msg_off, uint64_t* counts, void* workspace,
                             size_t workspace_bytes, void* stream) {
    hipStream_t s = reinterpret_cast<hipStream_t>(stream);
    if (!msg_off || !counts) return SBE_EINVAL;
    if (n == 0) {
        hipError_t e = hipMemsetAsync(counts, 0, 16, s);
        if (e == hipSuccess) e = hipMemsetAsync(msg_off, 0, 8, s);
        return record_hip(e);
    }
    if (!in || !frag_off || !flags || !out || !workspace) return SBE_EINVAL;
    if (n >= (1ull << 31)) return SBE_EINVAL;
    if (workspace_bytes < sbe_reassemble_workspace_size(n)) return SBE_ENOSPC;
    auto al = [](uintptr_t x) { return (x + 15) & ~(uintptr_t)15; };
    uintptr_t w = al(reinterpret_cast<uintptr_t>(workspace));
    FragScan* el = reinterpret_cast<FragScan*>(w);
    w = al(w + n * sizeof(FragScan));
    FragScan* sc = reinterpret_cast<FragScan*>(w);
    w = al(w + n * sizeof(FragScan));
    uint64_t* msize = reinterpret_cast<uint64_t*>(w);
    w = al(w + 8 * (n + 1));
    uint64_t* mfirst = reinterpret_cast<uint64_t*>(w);
    w = al(w + 8 * (n + 1));
    uint64_t* mlast = reinterpret_cast<uint64_t*>(w);
    // the big-message list lives in sc[], which the fused scan does not use (n + 2 <= 4n words)
#ifndef SBE_FRAG_BIG  // A/B builds: 0 = no big-message list (every message copied by its own wave)
#define SBE_FRAG_BIG 1
#endif
    FragArgs a{in, frag_off, flags, n, out, msg_off, counts, el, sc, msize, mfirst, mlast,
               SBE_FRAG_FUSED && SBE_FRAG_BIG ? reinterpret_cast<uint64_t*>(sc) : nullptr};
    const uint32_t blocks = (uint32_t)((n + 1 + 255) / 256);
    const uint64_t nb = (n + kFsBlk - 1) / kFsBlk;
    hipLaunchKernelGGL(frag_reduce, dim3((uint32_t)nb), dim3(kFsThreads), 0, s, a, el);
    hipLaunchKernelGGL(frag_scan_blocks, dim3(1), dim3(kFsbThreads), 0, s, el, nb, a.big);
    hipError_t e = hipSuccess;
    if (SBE_FRAG_FUSED) {
        hipLaunchKernelGGL(frag_scan_msgs, dim3((uint32_t)nb), dim3(kFsThreads), 0, s, a, static_cast<const FragScan*>(el));
        e = hipGetLastError();
        if (e != hipSuccess) return record_hip(e);
    } else {
        hipLaunchKernelGGL(frag_scan, dim3((uint32_t)nb), dim3(kFsThreads), 0, s, a, static_cast<const FragScan*>(el));
        e = hipGetLastError();
        if (e != hipSuccess) return record_hip(e);
        hipLaunchKernelGGL(frag_messages, dim3(blocks), dim3(256), 0, s, a);
        e = hipGetLastError();
        if (e != hipSuccess) return record_hip(e);
    }
    const uint64_t cb = (n + 1 + 4 * kFragGroup - 1) / (4 * kFragGroup);  // four waves per block
#ifndef SBE_FC_MAXB  // A/B builds: the copy's grid cap (blocks of four waves; they loop over the groups)
#define SBE_FC_MAXB 4096
#endif
    hipLaunchKernelGGL(frag_copy, dim3((uint32_t)(cb < SBE_FC_MAXB ? cb : SBE_FC_MAXB)), dim3(256), 0, s, a);
    return record_hip(hipGetLastError());
}

size_t sbe_order_json_workspace_size(uint64_t n) {
    // text sizes and string bases (n each), two block-sum arrays, alignment
    const uint64_t nblk = (n + oj::kBlock - 1) / oj::kBlock;
    return (size_t)(16 * n + 16 * nblk + 4 * 16);
}

int sbe_order_to_json_batch(const sbe_order_batch* in, uint64_t n, uint32_t what, uint8_t* out,
                            uint64_t out_capacity, uint64_t* out_off, uint8_t* status, void* workspace,
                            size_t workspace_bytes, void* stream) {
    hipStream_t s = reinterpret_cast<hipStream_t>(stream);
    if (!in || !out_off || what > SBE_JSON_PUBLISH_HEADERS) return SBE_EINVAL;
    if (n == 0) return record_hip(hipMemsetAsync(out_off, 0, 8, s));
    if (!in->arena || !in->str_len || !in->customer_id || !in->timestamp || !in->quantity || !workspace)
        return SBE_EINVAL;
    if (n >= (1ull << 40)) return SBE_EINVAL;
    if (workspace_bytes < sbe_order_json_workspace_size(n)) return SBE_ENOSPC;
    if (!out && out_capacity) return SBE_EINVAL;
    const uint64_t nblk = (n + oj::kBlock - 1) / oj::kBlock;
    auto al = [](uintptr_t x) { return (x + 15) & ~(uintptr_t)15; };
    uintptr_t w = al(reinterpret_cast<uintptr_t>(workspace));
    uint64_t* sz = reinterpret_cast<uint64_t*>(w);
    w = al(w + 8 * n);
    uint64_t* base = reinterpret_cast<uint64_t*>(w);
    w = al(w + 8 * n);
    uint64_t* blk_str = reinterpret_cast<uint64_t*>(w);
    w = al(w + 8 * nblk);
    uint64_t* blk_txt = reinterpret_cast<uint64_t*>(w);
    oj::JsonArgs a{in->arena, in->str_off, in->str_len, in->customer_id, in->timestamp, in->quantity, n, what,
                   out,       out_capacity, out_off,  status,  sz,  base,  blk_str,  blk_txt};
    // sizing (per-block sums), one small scan of the block sums per chain, writing
    const uint32_t blocks = (uint32_t)nblk;
    if (!in->str_off) {
        hipLaunchKernelGGL(oj::order_json_totals, dim3(blocks), dim3(oj::kBlock), 0, s, a);
        hipLaunchKernelGGL(oj::order_json_scan_blocks, dim3(1), dim3(oj::kScanThreads), 0, s, blk_str, nblk);
    }
    if (what == SBE_JSON_PUBLISH_HEADERS)
        hipLaunchKernelGGL(oj::order_json_measure<SBE_JSON_PUBLISH_HEADERS>, dim3(blocks), dim3(oj::kBlock), 0, s, a);
    else
        hipLaunchKernelGGL(oj::order_json_measure<SBE_JSON_ORDER_PAYLOAD>, dim3(blocks), dim3(oj::kBlock), 0, s, a);
    hipLaunchKernelGGL(oj::order_json_scan_blocks, dim3(1), dim3(oj::kScanThreads), 0, s, blk_txt, nblk);
    if (what == SBE_JSON_PUBLISH_HEADERS) {
        constexpr uint64_t t = oj::WShape<SBE_JSON_PUBLISH_HEADERS>::kOpw;
        hipLaunchKernelGGL(oj::order_json_write<SBE_JSON_PUBLISH_HEADERS>, dim3((uint32_t)((n + t - 1) / t)),
                           dim3(oj::kWWave), 0, s, a);
    } else {
        constexpr uint64_t t = oj::WShape<SBE_JSON_ORDER_PAYLOAD>::kOpw;
        hipLaunchKernelGGL(oj::order_json_write<SBE_JSON_ORDER_PAYLOAD>, dim3((uint32_t)((n + t - 1) / t)),
                           dim3(oj::kWWave), 0, s, a);
    }
    return record_hip(hipGetLastError());
}

// RCCL is loaded on the first communicator call (dlopen), so the codec itself needs no RCCL to
// load.  In a process that already holds an RCCL (torch's), that same library is used.
struct RcclApi {
    bool loaded = false;
    char err[160] = "";
    ncclResult_t (*GetUniqueId)(ncclUniqueId*) = nullptr;
    ncclResult_t (*CommInitRank)(ncclComm_t*, int, ncclUniqueId, int) = nullptr;
    ncclResult_t (*CommDestroy)(ncclComm_t) = nullptr;
    ncclResult_t (*AllGather)(const void*, void*, size_t, ncclDataType_t, ncclComm_t, hipStream_t) = nullptr;
    ncclResult_t (*Send)(const void*, size_t, ncclDataType_t, int, ncclComm_t, hipStream_t) = nullptr;
    ncclResult_t (*Recv)(void*, size_t, ncclDataType_t, int, ncclComm_t, hipStream_t) = nullptr;
    ncclResult_t (*GroupStart)() = nullptr;
    ncclResult_t (*GroupEnd)() = nullptr;
    const char* (*GetErrorString)(ncclResult_t) = nullptr;
};

static RcclApi& rccl_api() {
    static RcclApi api;
    static std::once_flag once;
    std::call_once(once, [] {
        void* h = nullptr;
        // test only: SBE_RCCL_LIB names a stand-in with RCCL's symbols (tests/mock_rccl: the ranks
        // of a communicator as threads of one process), so the multi-rank gather runs on one GPU
        if (const char* alt = std::getenv("SBE_RCCL_LIB"); alt && *alt) {
            h = dlopen(alt, RTLD_NOW | RTLD_LOCAL);
            if (!h) {
                std::snprintf(api.err, sizeof(api.err), "SBE_RCCL_LIB not loadable: %s", dlerror());
                return;
            }
        }
        for (const char* name : {"librccl.so.1", "librccl.so"})
            if (!h) h = dlopen(name, RTLD_NOW | RTLD_NOLOAD);  // the process's own RCCL first
        for (const char* name : {"librccl.so.1", "/opt/rocm/lib/librccl.so.1", "librccl.so"})
            if (!h) h = dlopen(name, RTLD_NOW | RTLD_GLOBAL);
        if (!h) {
            std::snprintf(api.err, sizeof(api.err), "RCCL not loadable: %s", dlerror());
            return;
        }
        bool ok = true;
        auto sym = [&](auto& fn, const char* name) {
            fn = reinterpret_cast<std::remove_reference_t<decltype(fn)>>(dlsym(h, name));
            ok = ok && fn != nullptr;
        };
        sym(api.GetUniqueId, "ncclGetUniqueId");
        sym(api.CommInitRank, "ncclCommInitRank");
        sym(api.CommDestroy, "ncclCommDestroy");
        sym(api.AllGather, "ncclAllGather");
        sym(api.Send, "ncclSend");
        sym(api.Recv, "ncclRecv");
        sym(api.GroupStart, "ncclGroupStart");
        sym(api.GroupEnd, "ncclGroupEnd");
        sym(api.GetErrorString, "ncclGetErrorString");
        if (!ok) std::snprintf(api.err, sizeof(api.err), "RCCL lacks a required symbol");
        api.loaded = ok;
    });
    return api;
}

static int rccl_ready() {
    RcclApi& r = rccl_api();
    if (r.loaded) return SBE_OK;
    std::snprintf(g_last_error, sizeof(g_last_error), "%s", r.err);
    return SBE_ECOMM;
}

struct sbe_comm {
    ncclComm_t nc = nullptr;
    int world = 0, rank = 0;
    uint64_t* d_mine = nullptr;   // {bytes, n, root byte capacity, root offset capacity} (device, 32 B)
    uint64_t* d_all = nullptr;    // the same of every rank (device, 32 B per rank)
    uint64_t* h_all = nullptr;    // pinned host copy of d_all
    uint64_t* plan = nullptr;       // host [world][4]: {bytes, records, root capacity, root offset capacity}
    uint64_t* byte_base = nullptr;  // host [world + 1]: the gather plan
    uint64_t* rec_base = nullptr;
};

static int record_nccl(ncclResult_t r, const char* what) {
    if (r == ncclSuccess) return SBE_OK;
    std::snprintf(g_last_error, sizeof(g_last_error), "%s: %s", what, rccl_api().GetErrorString(r));
    return SBE_ECOMM;
}

int sbe_gather_plan(const uint64_t* ranks, int world, int root, uint64_t* byte_base, uint64_t* rec_base,
                    uint64_t* totals) {
    if (!ranks || world < 1 || root < 0 || root >= world || !byte_base || !rec_base) return SBE_EINVAL;
    uint64_t b = 0, m = 0;
    for (int r = 0; r < world; ++r) {
        byte_base[r] = b;
        rec_base[r] = m;
        b += ranks[4 * r];
        m += ranks[4 * r + 1];
    }
    byte_base[world] = b;
    rec_base[world] = m;
    if (totals) {
        totals[0] = b;
        totals[1] = m;
    }
    // every rank decides from the root's capacities: a short root buffer stops all of them before
    // any transfer is posted
    const uint64_t cap = ranks[4 * root + 2], off_cap = ranks[4 * root + 3];
    if (b > cap) {
        std::snprintf(g_last_error, sizeof(g_last_error), "gather: root buffer holds %llu of %llu bytes",
                      (unsigned long long)cap, (unsigned long long)b);
        return SBE_ENOSPC;
    }
    if (m + 1 > off_cap) {
        std::snprintf(g_last_error, sizeof(g_last_error), "gather: root offsets hold %llu of %llu entries",
                      (unsigned long long)off_cap, (unsigned long long)(m + 1));
        return SBE_ENOSPC;
    }
    return SBE_OK;
}

int sbe_comm_unique_id(uint8_t id[SBE_COMM_ID_BYTES]) {
    static_assert(sizeof(ncclUniqueId) == SBE_COMM_ID_BYTES, "RCCL unique id size");
    if (!id) return SBE_EINVAL;
    int rc = rccl_ready();
    if (rc != SBE_OK) return rc;
    ncclUniqueId u;
    rc = record_nccl(rccl_api().GetUniqueId(&u), "ncclGetUniqueId");
    if (rc == SBE_OK) std::memcpy(id, &u, sizeof(u));
    return rc;
}

int sbe_comm_init(sbe_comm** comm, int world, int rank, const uint8_t id[SBE_COMM_ID_BYTES]) {
    if (!comm || !id || world < 1 || rank < 0 || rank >= world) return SBE_EINVAL;
    *comm = nullptr;
    int rc = rccl_ready();
    if (rc != SBE_OK) return rc;
    sbe_comm* c = new sbe_comm;
    c->world = world;
    c->rank = rank;
    c->plan = new uint64_t[4 * (size_t)world];
    c->byte_base = new uint64_t[world + 1];
    c->rec_base = new uint64_t[world + 1];
    rc = record_hip(hipMalloc(reinterpret_cast<void**>(&c->d_mine), 32));
    if (rc == SBE_OK) rc = record_hip(hipMalloc(reinterpret_cast<void**>(&c->d_all), 32 * (size_t)world));
    if (rc == SBE_OK) rc = record_hip(hipHostMalloc(reinterpret_cast<void**>(&c->h_all), 32 * (size_t)world, 0));
    if (rc == SBE_OK) {
        ncclUniqueId u;
        std::memcpy(&u, id, sizeof(u));
        rc = record_nccl(rccl_api().CommInitRank(&c->nc, world, u, rank), "ncclCommInitRank");
    }
    if (rc != SBE_OK) {
        sbe_comm_destroy(c);
        return rc;
    }
    *comm = c;
    return SBE_OK;
}

int sbe_comm_destroy(sbe_comm* c) {
    if (!c) return SBE_OK;
    int rc = SBE_OK;
    if (c->nc) rc = record_nccl(rccl_api().CommDestroy(c->nc), "ncclCommDestroy");
    if (c->d_mine) (void)hipFree(c->d_mine);
    if (c->d_all) (void)hipFree(c->d_all);
    if (c->h_all) (void)hipHostFree(c->h_all);
    delete[] c->plan;
    delete[] c->byte_base;
    delete[] c->rec_base;
    delete c;
    return rc;
}

// Steps 2-3 of both gathers: from the plan in c->plan ({bytes, records, ...} per rank, 4 words a
// rank) and c->byte_base / c->rec_base, one group of sends / receives, then the root's own shard,
// the rebase and the closing offset.  Everything is enqueued on s; nothing waits on the host.
static int gather_transfer(sbe_comm* c, int root, const uint8_t* out, const uint64_t* out_off, uint8_t* dst,
                           uint64_t* dst_off, const uint64_t tot[2], hipStream_t s) {
    const RcclApi& R = rccl_api();
    const bool am_root = c->rank == root;
    const uint64_t* plan = c->plan;
    int rc = record_nccl(R.GroupStart(), "ncclGroupStart");
    if (rc != SBE_OK) return rc;
    for (int r = 0; r < c->world && rc == SBE_OK; ++r) {
        const uint64_t b = plan[4 * r], m = plan[4 * r + 1];
        if (r == c->rank && !am_root) {
            if (b) rc = record_nccl(R.Send(out, b, ncclUint8, root, c->nc, s), "ncclSend");
            if (m && rc == SBE_OK) rc = record_nccl(R.Send(out_off, m, ncclUint64, root, c->nc, s), "ncclSend");
        } else if (am_root && r != root) {
            if (b) rc = record_nccl(R.Recv(dst + c->byte_base[r], b, ncclUint8, r, c->nc, s), "ncclRecv");
            if (m && rc == SBE_OK)
                rc = record_nccl(R.Recv(dst_off + c->rec_base[r], m, ncclUint64, r, c->nc, s), "ncclRecv");
        }
    }
    const int rc_end = record_nccl(R.GroupEnd(), "ncclGroupEnd");
    if (rc != SBE_OK) return rc;
    if (rc_end != SBE_OK) return rc_end;
    if (!am_root) return SBE_OK;
    // root: its own shard, the offset rebase, the closing offset
    for (int r = 0; r < c->world; ++r) {
        const uint64_t b = plan[4 * r], m = plan[4 * r + 1];
        if (r == root && b)
            rc = record_hip(hipMemcpyAsync(dst + c->byte_base[r], out, b, hipMemcpyDeviceToDevice, s));
        if (rc != SBE_OK) return rc;
        if (m) {
            const uint64_t blocks = (m + 255) / 256;
            uint64_t* d = dst_off + c->rec_base[r];
            hipLaunchKernelGGL(offsets_rebase, dim3((uint32_t)(blocks < 4096 ? blocks : 4096)), dim3(256), 0, s, d,
                               r == root ? out_off : d, m, c->byte_base[r]);
            rc = record_hip(hipGetLastError());
            if (rc != SBE_OK) return rc;
        }
    }
    hipLaunchKernelGGL(u64_put, dim3(1), dim3(64), 0, s, dst_off + tot[1], tot[0]);
    return record_hip(hipGetLastError());
}

int sbe_gather_encoded(sbe_comm* c, int root, const uint8_t* out, const uint64_t* out_off, uint64_t n,
                       uint8_t* dst, uint64_t dst_capacity, uint64_t* dst_off, uint64_t dst_off_capacity,
                       uint64_t* totals, void* stream) {
    if (!c || !out_off || root < 0 || root >= c->world) return SBE_EINVAL;
    const bool am_root = c->rank == root;
    if (am_root && !dst_off) return SBE_EINVAL;
    const RcclApi& R = rccl_api();
    hipStream_t s = reinterpret_cast<hipStream_t>(stream);
    // 1. every rank's {bytes, n} and the root's capacities
    hipLaunchKernelGGL(shard_size_put, dim3(1), dim3(64), 0, s, c->d_mine, out_off, n,
                       am_root && dst ? dst_capacity : 0ull, am_root ? dst_off_capacity : 0ull);
    int rc = record_hip(hipGetLastError());
    if (rc != SBE_OK) return rc;
    rc = record_nccl(R.AllGather(c->d_mine, c->d_all, 4, ncclUint64, c->nc, s), "ncclAllGather");
    if (rc != SBE_OK) return rc;
    rc = record_hip(hipMemcpyAsync(c->h_all, c->d_all, 32 * (size_t)c->world, hipMemcpyDeviceToHost, s));
    if (rc == SBE_OK) rc = record_hip(hipStreamSynchronize(s));
    if (rc != SBE_OK) return rc;
    std::memcpy(c->plan, c->h_all, 32 * (size_t)c->world);
    uint64_t tot[2];
    rc = sbe_gather_plan(c->plan, c->world, root, c->byte_base, c->rec_base, tot);
    if (totals) {
        totals[0] = tot[0];
        totals[1] = tot[1];
    }
    if (rc != SBE_OK) return rc;
    // 2. the shards and their offsets, in one group; 3. the root's rebase
    return gather_transfer(c, root, out, out_off, dst, dst_off, tot, s);
}

int sbe_gather_encoded_sized(sbe_comm* c, int root, const uint64_t* sizes, const uint8_t* out,
                             const uint64_t* out_off, uint8_t* dst, uint64_t dst_capacity, uint64_t* dst_off,
                             uint64_t dst_off_capacity, uint64_t* totals, void* stream) {
    if (!c || !sizes || !out_off || root < 0 || root >= c->world || dst_off_capacity == 0) return SBE_EINVAL;
    const bool am_root = c->rank == root;
    if (am_root && !dst_off) return SBE_EINVAL;
    // the plan from the caller's sizes, with the root's capacities every rank was given
    for (int r = 0; r < c->world; ++r) {
        c->plan[4 * r] = sizes[2 * r];
        c->plan[4 * r + 1] = sizes[2 * r + 1];
        c->plan[4 * r + 2] = r == root ? dst_capacity : 0;
        c->plan[4 * r + 3] = r == root ? dst_off_capacity : 0;
    }
    uint64_t tot[2];
    const int rc = sbe_gather_plan(c->plan, c->world, root, c->byte_base, c->rec_base, tot);
    if (totals) {
        totals[0] = tot[0];
        totals[1] = tot[1];
    }
    if (rc != SBE_OK) return rc;
    return gather_transfer(c, root, out, out_off, dst, dst_off, tot, reinterpret_cast<hipStream_t>(stream));
}

#ifdef SBE_PACK_PHASES
// diagnosis build: the pack kernel's per-wave phase clocks (8 per workgroup, first `nwg` workgroups)
int sbe_debug_phases(uint64_t* host, int nwg) {
    if (nwg > 16384) nwg = 16384;
    return hipMemcpyFromSymbol(host, HIP_SYMBOL(g_pack_phase), sizeof(uint64_t) * 8 * (size_t)nwg, 0,
                               hipMemcpyDeviceToHost) == hipSuccess ? 0 : -1;
}
int sbe_debug_phases_clear() {
    static uint64_t zero[16384 * 8];
    return hipMemcpyToSymbol(HIP_SYMBOL(g_pack_phase), zero, sizeof(zero), 0, hipMemcpyHostToDevice) == hipSuccess ? 0 : -1;
}
#endif

int sbe_profile_enable(int every) {
    if (every < 0) return SBE_EINVAL;
    // both rings' events first: profiling turns on only once they exist
    if (every > 0)
        for (auto& R : g_prof) {
            const hipError_t e = prof_ready(R);
            if (e != hipSuccess) {
                g_prof_every = 0;
                return record_hip(e);
            }
        }
    g_prof_every = every;
    for (auto& R : g_prof) R.head = R.count = 0, R.launches = 0;
    return SBE_OK;
}

int sbe_profile_read(int kernel, float* ms, int max) {
    if (kernel < 0 || kernel > 1 || (!ms && max > 0)) return SBE_EINVAL;
    ProfRing& R = g_prof[kernel];
    const int n = R.count < max ? R.count : max;
    const int first = (R.head - R.count + ProfRing::kCap) % ProfRing::kCap;
    for (int i = 0; i < n; ++i) {
        const int k = (first + R.count - n + i) % ProfRing::kCap;
        const hipError_t e = hipEventElapsedTime(&ms[i], R.ev[k][0], R.ev[k][1]);
        if (e != hipSuccess) return record_hip(e);
    }
    R.head = R.count = 0;
    return n;
}

}  // extern "C"
