// order_json.hpp — Order JSON text on the GPU (included by sbe_codec.hip).
//
// Replaces Order::to_json (src/order_types.cpp:122-181) and the headers JSON publish_order builds
// (src/cluster_client.cpp:308-323): jsoncpp StreamWriterBuilder with indentation "" (compact,
// colon ":", object members in std::map order), so the text is a fixed skeleton with eight
// variable slots — escaped strings, two decimal integers and the quantity printed twice, once by
// jsoncpp valueToString ("%.17g", ".0" appended when there is no '.' or 'e') and once by
// std::to_string ("%f").  Both number formats follow glibc printf on the EXACT binary value
// (round half to even on the exact decimal expansion), so the formatter below expands the double
// exactly: the integer part as base-1e9 limbs, the fraction F / 2^k as a multiword numerator that
// yields nine digits per multiply.  Values with short binary fractions (prices, quantities) touch
// one or two words; the full range (subnormals, 1e308) takes more words, never a different path.
//
// One lane per Order; per-block string totals (packed arena) and their one-block scan, a sizing
// launch (text lengths, string bases, per-block text totals) and its one-block scan, then the
// writing launch, which finds each text's offset from the block sums, stages each wave's texts in
// LDS and stores them coalesced.
#pragma once

namespace oj {

constexpr uint32_t kFields = SBE_ORDER_FIELDS;

// Address-space-typed pointers: the helpers are out of line, and a plain pointer argument would
// make every byte access a flat instruction (which waits on both the LDS and the vector-memory
// counters).  Strings are read from HBM (global), texts are written to LDS or HBM.
typedef const __attribute__((address_space(1))) uint8_t gu8;
typedef const __attribute__((address_space(3))) uint8_t lr8;  // strings staged in LDS (sizing launch)
typedef __attribute__((address_space(1))) uint8_t gw8;
typedef __attribute__((address_space(3))) uint8_t lw8;
constexpr uint32_t kBlock = 256;

struct JsonArgs {
    const uint8_t* arena;
    const uint32_t* str_off;
    const uint32_t* str_len;
    const int64_t* customer_id;
    const int64_t* timestamp;
    const double* quantity;
    uint64_t n;
    uint32_t what;
    uint8_t* out;
    uint64_t cap;
    uint64_t* out_off;   // n + 1 text offsets
    uint8_t* status;
    uint64_t* sz;        // n text lengths (sizing launch)
    uint64_t* str_base;  // n packed-arena string bases (sizing launch)
    uint64_t* blk_str;   // per block of kBlock Orders: packed-arena string bytes, then their exclusive scan
    uint64_t* blk_txt;   // per block: text bytes, then their exclusive scan
};

// ---- byte sinks: counting (sizing launch) and writing (8-byte buffered, byte-exact edges) ----
// Byte o of a 16-byte block and the block shifted down by o bytes, by 64-bit shifts: a select
// chain over the four words is turned by the compiler into a private array (a scratch store and
// a scratch load per byte).
__device__ inline uint32_t block_byte(const uint4& v, uint32_t o) {
    const uint64_t h = (o & 8) ? ((uint64_t)v.w << 32 | v.z) : ((uint64_t)v.y << 32 | v.x);
    return (uint32_t)(h >> (8 * (o & 7))) & 0xFF;
}
__device__ inline uint4 block_shift(const uint4& v, uint32_t o) {  // bytes [o, 16) of v, then zeros
    const uint64_t lo = (uint64_t)v.y << 32 | v.x, hi = (uint64_t)v.w << 32 | v.z;
    const uint32_t sh = 8 * (o & 7);
    const uint64_t a = (o & 8) ? hi : lo, b = (o & 8) ? 0ull : hi;
    const uint64_t rlo = sh ? (a >> sh) | (b << (64 - sh)) : a, rhi = b >> sh;
    return make_uint4((uint32_t)rlo, (uint32_t)(rlo >> 32), (uint32_t)rhi, (uint32_t)(rhi >> 32));
}

// put(b) appends one byte; run(v, o, m) appends bytes [o, o + m) of the loaded 16-byte block v
struct CountSink {
    uint64_t n = 0;
    __device__ void put(uint8_t) { ++n; }
    __device__ void run(const uint4&, uint32_t, uint32_t m) { n += m; }
};

// One byte store per put: into the wave's LDS window (ds_write_b8) or, for a record larger than
// the window, straight to HBM.
struct LdsSink {
    lw8* p;
    uint32_t n = 0;
    uint32_t lim;  // the text's length: bytes [0, lim) of p are this lane's
    __device__ LdsSink(lw8* q, uint32_t len) : p(q), lim(len) {}
    __device__ void put(uint8_t b) { p[n++] = b; }
    // a run of m plain bytes: one (unaligned) 16-byte LDS store of the block realigned to o; the
    // bytes past the run are this lane's own later text, which overwrites them (near the end of
    // the text, byte stores)
    __device__ void run(const uint4& v, uint32_t o, uint32_t m) {
        if (n + 16 <= lim) {
            typedef uint32_t u32x4u __attribute__((ext_vector_type(4), aligned(1)));
            typedef __attribute__((address_space(3))) u32x4u lw128u;
            const uint4 r = block_shift(v, o);
            u32x4u x;
            x.x = r.x;
            x.y = r.y;
            x.z = r.z;
            x.w = r.w;
            *reinterpret_cast<lw128u*>(p + n) = x;
            n += m;
        } else {
            for (uint32_t k = o; k < o + m; ++k) p[n++] = (uint8_t)block_byte(v, k);
        }
    }
};
struct HbmSink {
    gw8* p;
    uint64_t n = 0;
    __device__ explicit HbmSink(gw8* q) : p(q) {}
    __device__ void put(uint8_t b) { p[n++] = b; }
    __device__ void run(const uint4& v, uint32_t o, uint32_t m) {
        for (uint32_t k = o; k < o + m; ++k) p[n++] = (uint8_t)block_byte(v, k);
    }
};

// A literal run: the length is a compile-time constant, so the copy unrolls into immediate
// stores at constant offsets from one address (no scalar character loop).
template <class S, size_t N>
__device__ inline void lit(S& s, const char (&t)[N]) {
#pragma unroll
    for (size_t k = 0; k + 1 < N; ++k) s.put((uint8_t)t[k]);
}

// jsoncpp json_writer.cpp utf8ToCodepoint (lead byte decides the length; continuation bytes are
// not checked; truncated / overlong / surrogate → U+FFFD; a truncated sequence consumes 1 byte).
// b1..b3 are the bytes after the lead (0 past the end of the string).
__device__ inline uint32_t utf8_cp(uint32_t b, uint32_t b1, uint32_t b2, uint32_t b3, uint64_t left,
                                   uint32_t& used) {
    used = 1;
    if (b < 0x80) return b;
    if (b < 0xE0) {
        if (left < 2) return 0xFFFD;
        const uint32_t c = ((b & 0x1F) << 6) | (b1 & 0x3F);
        used = 2;
        return c < 0x80 ? 0xFFFD : c;
    }
    if (b < 0xF0) {
        if (left < 3) return 0xFFFD;
        const uint32_t c = ((b & 0x0F) << 12) | ((b1 & 0x3F) << 6) | (b2 & 0x3F);
        used = 3;
        if (c >= 0xD800 && c <= 0xDFFF) return 0xFFFD;
        return c < 0x800 ? 0xFFFD : c;
    }
    if (b < 0xF8) {
        if (left < 4) return 0xFFFD;
        const uint32_t c = ((b & 0x07) << 18) | ((b1 & 0x3F) << 12) | ((b2 & 0x3F) << 6) | (b3 & 0x3F);
        used = 4;
        return c < 0x10000 ? 0xFFFD : c;
    }
    return 0xFFFD;
}

// Reads a string through aligned 16-byte loads, so a lane's walk over its string issues one
// load per 16 bytes instead of one dependent load per byte.  A block holding a byte of the
// string lies inside the allocation's page, so the over-read is harmless.
template <class P>
struct W32;  // the dword pointer of the same address space
template <>
struct W32<gu8*> {
    typedef const __attribute__((address_space(1))) uint32_t* T;
};
template <>
struct W32<lr8*> {
    typedef const __attribute__((address_space(3))) uint32_t* T;
};

template <class P>  // P: gu8* (HBM) or lr8* (LDS)
struct BlockReader {
    uintptr_t blk = ~(uintptr_t)0;
    uint4 v;
    __device__ uint32_t at(P p) {
        const uintptr_t a = (uintptr_t)p, b = a & ~(uintptr_t)15;
        if (b != blk) {
            blk = b;
            const typename W32<P>::T q = (typename W32<P>::T)b;
            v.x = q[0];
            v.y = q[1];
            v.z = q[2];
            v.w = q[3];
        }
        return block_byte(v, (uint32_t)(a & 15));
    }
};

template <class S>
__device__ inline void hex4(S& s, uint32_t v) {
    const char* hx = "0123456789abcdef";
    s.put('\\');
    s.put('u');
    s.put((uint8_t)hx[(v >> 12) & 15]);
    s.put((uint8_t)hx[(v >> 8) & 15]);
    s.put((uint8_t)hx[(v >> 4) & 15]);
    s.put((uint8_t)hx[v & 15]);
}

// Bit k set iff byte k of the block needs more than a plain copy in valueToQuotedStringN: a
// control byte (< 0x20), a byte >= 0x80, '"' or '\\' (SWAR, four bytes per dword, exact per byte).
__device__ inline uint32_t zero_bytes(uint32_t x) {  // 0x80 in exactly the zero bytes of x
    return ~(((x & 0x7f7f7f7fu) + 0x7f7f7f7fu) | x) & 0x80808080u;
}
__device__ inline uint32_t special4(uint32_t w) {  // 4-bit mask of w's special bytes
    const uint32_t ctl = ~((w & 0x7f7f7f7fu) + 0x60606060u) & 0x80808080u;  // low 7 bits < 0x20
    const uint32_t m = (w & 0x80808080u) | ctl | zero_bytes(w ^ 0x22222222u) | zero_bytes(w ^ 0x5c5c5c5cu);
    return __builtin_amdgcn_udot4(m >> 7, 0x08040201u, 0u, false);  // flags as bits 0-3 (one v_dot4)
}
__device__ inline uint32_t special16(const uint4& v) {
    return special4(v.x) | (special4(v.y) << 4) | (special4(v.z) << 8) | (special4(v.w) << 12);
}
__device__ inline uint32_t nul4(uint32_t w) { return __builtin_amdgcn_udot4(zero_bytes(w) >> 7, 0x08040201u, 0u, false); }
__device__ inline uint32_t nul16(const uint4& v) {  // bit k set iff byte k of the block is 0
    return nul4(v.x) | (nul4(v.y) << 4) | (nul4(v.z) << 8) | (nul4(v.w) << 12);
}

#ifndef SBE_OJ_INLINE  // A/B builds: 1 = the string and number helpers inlined into the kernels
#define SBE_OJ_INLINE 0
#endif
#if SBE_OJ_INLINE
#define OJ_HELPER __forceinline__
#else
#define OJ_HELPER __noinline__
#endif

// jsoncpp valueToQuotedStringN(str, len, emitUTF8 = false)
// Out-of-line helpers take the sink by value and return it: a sink passed by reference lives in
// scratch and every put would load and store its count.
template <class S, class P>
__device__ OJ_HELPER S quoted(S s, P p, uint64_t len) {
    s.put('"');
    BlockReader<P> rd;
    uint64_t i = 0;
    while (i < len) {
        {  // the common case: a run of plain bytes inside the current 16-byte block, found with
           // one SWAR classification of the block (no per-byte tests)
            (void)rd.at(p + i);  // loads the block holding p + i
            const uint32_t o = (uint32_t)((uintptr_t)(p + i) & 15);
            const uint64_t left = len - i;
            const uint32_t stop = left < 16 - o ? o + (uint32_t)left : 16;
            const uint32_t stops = special16(rd.v) | (0xffffffffu << stop);
            const uint32_t m = (uint32_t)__builtin_ctz(stops >> o);  // plain bytes from o
            s.run(rd.v, o, m);
            i += m;
            if (i >= len) break;
            if (o + m == 16) continue;  // the rest of the block was plain: next block
        }
        const uint8_t c = (uint8_t)rd.at(p + i);
        if (c >= 0x20 && c < 0x80 && c != '"' && c != '\\') {
            s.put(c);
            ++i;
            continue;
        }
        switch (c) {
            case '"': s.put('\\'); s.put('"'); ++i; continue;
            case '\\': s.put('\\'); s.put('\\'); ++i; continue;
            case '\b': s.put('\\'); s.put('b'); ++i; continue;
            case '\f': s.put('\\'); s.put('f'); ++i; continue;
            case '\n': s.put('\\'); s.put('n'); ++i; continue;
            case '\r': s.put('\\'); s.put('r'); ++i; continue;
            case '\t': s.put('\\'); s.put('t'); ++i; continue;
            default: break;
        }
        uint32_t used;
        const uint64_t left = len - i;
        const uint32_t b1 = left > 1 ? rd.at(p + i + 1) : 0, b2 = left > 2 ? rd.at(p + i + 2) : 0,
                       b3 = left > 3 ? rd.at(p + i + 3) : 0;
        uint32_t cp = utf8_cp(c, b1, b2, b3, left, used);
        i += used;
        if (cp < 0x10000) {
            hex4(s, cp);
        } else {
            cp -= 0x10000;
            hex4(s, 0xD800 + ((cp >> 10) & 0x3FF));
            hex4(s, 0xDC00 + (cp & 0x3FF));
        }
    }
    s.put('"');
    return s;
}

// ---- decimal text in registers ----------------------------------------------------------------
// A private digit array indexed by a running count lives in scratch (every digit a scratch store
// and load); these helpers keep the digits as packed ASCII words and append them with the sink's
// run(), so the common path touches no scratch.

// The four ASCII digits of v < 10000, most significant in byte 0.
__device__ inline uint32_t asc4(uint32_t v) {
    const uint32_t a = v / 100u, b = v - 100u * a;
    const uint32_t a1 = a / 10u, b1 = b / 10u;
    return 0x30303030u | a1 | (a - 10u * a1) << 8 | b1 << 16 | (b - 10u * b1) << 24;
}

// Twenty ASCII digits of v, zero padded, most significant first: bytes 0-15 in a, 16-19 in b.
struct Dec20 {
    uint4 a;
    uint32_t b;
};
__device__ inline Dec20 dec20(uint64_t v) {
    constexpr uint64_t kE16 = 10000000000000000ull;
    const uint64_t hi = v / kE16;  // <= 1844
    const uint64_t r = v - hi * kE16;
    const uint32_t mid = (uint32_t)(r / 100000000u), lo = (uint32_t)(r - (uint64_t)mid * 100000000u);
    Dec20 d;
    d.a.x = asc4((uint32_t)hi);
    d.a.y = asc4(mid / 10000u);
    d.a.z = asc4(mid % 10000u);
    d.a.w = asc4(lo / 10000u);
    d.b = asc4(lo % 10000u);
    return d;
}

// Appends bytes [o, o + m) of the twenty digits.
template <class S>
__device__ inline void dec_run(S& s, const Dec20& d, uint32_t o, uint32_t m) {
    if (o < 16) {
        const uint32_t m1 = m < 16 - o ? m : 16 - o;
        s.run(d.a, o, m1);
        m -= m1;
        o = 16;
    }
    if (m) s.run(make_uint4(d.b, 0u, 0u, 0u), o - 16, m);
}

__device__ inline uint32_t ndig64(uint64_t v) {  // decimal digits of v (1 for 0)
    uint32_t d = 1;
    uint64_t p = 10;
#pragma unroll
    for (int k = 1; k < 20; ++k, p *= 10) d += v >= p ? 1u : 0u;
    return d;
}

template <class S>
__device__ inline void dec_u64(S& s, uint64_t v) {
    const uint32_t nd = ndig64(v);
    dec_run(s, dec20(v), 20 - nd, nd);
}

template <class S>
__device__ void dec_i64(S& s, int64_t v) {  // "%ld"
    if (v < 0) {
        s.put('-');
        dec_u64(s, 0ull - (uint64_t)v);
    } else {
        dec_u64(s, (uint64_t)v);
    }
}

// ------------------------------------------------------------------------------------------
// Exact decimal expansion of a finite, non-zero |v| = I + F / 2^k.
// ------------------------------------------------------------------------------------------
constexpr uint32_t kE9 = 1000000000u;

struct Exact {
    uint32_t lim[36];  // integer part, base-1e9 limbs, most significant first
    int nl;            // 0 when I == 0
    uint32_t fw[35];   // fraction numerator, little-endian words (k bits)
    int nfw, k;
    // Register mode for price-like values (k <= 64 and I < 1e17): I as u64 in two limbs l0 l1,
    // F as one u64, digits through a 128-bit product.  The arrays above are then never touched
    // (they live in scratch).
    bool small;
    uint64_t sI, sF;
    uint32_t l0, l1;

    __device__ void set_small_int(uint64_t ip) {
        sI = ip;
        nl = ip == 0 ? 0 : (ip >= kE9 ? 2 : 1);
        l0 = nl == 2 ? (uint32_t)(ip / kE9) : (uint32_t)ip;
        l1 = nl == 2 ? (uint32_t)(ip % kE9) : 0;
    }
    __device__ uint32_t limb(int j) const { return small ? (j == 0 ? l0 : l1) : lim[j]; }

    __device__ void init(double v) {
        const uint64_t bits = (uint64_t)__double_as_longlong(v) & ~(1ull << 63);
        const uint32_t ex = (uint32_t)(bits >> 52);
        uint64_t m = bits & ((1ull << 52) - 1);
        int e;
        if (ex == 0) e = -1074;
        else m |= 1ull << 52, e = (int)ex - 1075;
        const int t = __builtin_ctzll(m);
        m >>= t;
        e += t;
        nl = 0;
        nfw = 0;
        k = 0;
        small = false;
        if (e < 0 && e >= -64) {
            small = true;
            k = -e;
            sF = k >= 64 ? m : (m & ((1ull << k) - 1));
            set_small_int(k >= 64 ? 0 : (m >> k));
            return;
        }
        if (e >= 0 && e <= 10 && (m << e) < 100000000000000000ull) {
            small = true;
            sF = 0;
            set_small_int(m << e);
            return;
        }
        if (e < 0) {
            k = -e;
            const uint64_t ip = k >= 64 ? 0 : (m >> k);
            const uint64_t fp = k >= 64 ? m : (m & ((1ull << k) - 1));
            int_from_u64(ip);
            nfw = (k + 31) / 32;
            for (int j = 0; j < nfw; ++j) fw[j] = 0;
            fw[0] = (uint32_t)fp;
            if (nfw > 1) fw[1] = (uint32_t)(fp >> 32);
        } else if (e <= 10) {
            int_from_u64(m << e);  // m < 2^53
        } else {
            // I = m << e as a little-endian word array, then repeated division by 1e9
            uint32_t w[34];
            const int nw = (53 + e + 31) / 32;
            for (int j = 0; j < nw; ++j) w[j] = 0;
            const int ws = e / 32, bs = e % 32;
            const unsigned __int128 sh = (unsigned __int128)m << bs;
            w[ws] = (uint32_t)sh;
            if (ws + 1 < nw) w[ws + 1] = (uint32_t)(sh >> 32);
            if (ws + 2 < nw) w[ws + 2] = (uint32_t)(sh >> 64);
            int top = nw;
            uint32_t rev[36];
            int nr = 0;
            while (top > 0) {
                uint64_t r = 0;
                for (int j = top - 1; j >= 0; --j) {
                    const uint64_t cur = (r << 32) | w[j];
                    w[j] = (uint32_t)(cur / kE9);
                    r = cur % kE9;
                }
                rev[nr++] = (uint32_t)r;
                while (top > 0 && w[top - 1] == 0) --top;
            }
            nl = nr;
            for (int j = 0; j < nr; ++j) lim[j] = rev[nr - 1 - j];
        }
    }

    __device__ void int_from_u64(uint64_t ip) {
        nl = 0;
        if (ip == 0) return;
        uint32_t r[3];
        int c = 0;
        while (ip) {
            r[c++] = (uint32_t)(ip % kE9);
            ip /= kE9;
        }
        nl = c;
        for (int j = 0; j < c; ++j) lim[j] = r[c - 1 - j];
    }

    __device__ bool frac_nonzero() const {
        if (small) return sF != 0;
        uint32_t o = 0;
        for (int j = 0; j < nfw; ++j) o |= fw[j];
        return o != 0;
    }

    // The next nine fraction digits, as an integer < 1e9 (F ← F·1e9 mod 2^k).
    __device__ uint32_t frac_next9() {
        if (small) {
            if (k == 0) return 0;
            const unsigned __int128 t = (unsigned __int128)sF * kE9;
            sF = k == 64 ? (uint64_t)t : ((uint64_t)t & ((1ull << k) - 1));
            return (uint32_t)(t >> k);
        }
        if (nfw == 0) return 0;
        uint64_t carry = 0;
        for (int j = 0; j < nfw; ++j) {
            const uint64_t t = (uint64_t)fw[j] * kE9 + carry;
            fw[j] = (uint32_t)t;
            carry = t >> 32;
        }
        const int kb = k & 31;
        if (kb == 0) return (uint32_t)carry;
        const uint32_t top = fw[nfw - 1];
        fw[nfw - 1] = top & ((1u << kb) - 1);
        return (uint32_t)((carry << (32 - kb)) | (top >> kb));
    }
};

__device__ inline int ndig9(uint32_t v) {  // decimal digits of 0 < v < 1e9
    int d = 1;
    while (v >= 10) v /= 10, ++d;
    return d;
}

// The nine decimal digits of v < 1e9, most significant first (constant divisors: multiply-shift,
// no runtime division).
__device__ inline void split9(uint32_t v, uint8_t dg[9]) {
#pragma unroll
    for (int q = 8; q >= 0; --q) {
        dg[q] = (uint8_t)(v % 10u);
        v /= 10u;
    }
}

// The last w (<= 9) digits of v, zero padded.
template <class S>
__device__ inline void put_digits(S& s, uint32_t v, int w) {
    uint8_t dg[9];
    split9(v, dg);
#pragma unroll
    for (int q = 0; q < 9; ++q)
        if (q >= 9 - w) s.put((uint8_t)('0' + dg[q]));
}

// ---- the register path for price-like values ----
// |v| = I + F / 2^k with k <= 64 and I < 1e17 (what Exact's register mode covers): I, F, k.
__device__ inline bool small_parts(double v, uint64_t& I, uint64_t& F, uint32_t& k) {
    const uint64_t bits = (uint64_t)__double_as_longlong(v) & ~(1ull << 63);
    const uint32_t ex = (uint32_t)(bits >> 52);
    uint64_t m = bits & ((1ull << 52) - 1);
    int e;
    if (ex == 0) e = -1074;
    else m |= 1ull << 52, e = (int)ex - 1075;
    const int t = __builtin_ctzll(m);
    m >>= t;
    e += t;
    if (e < 0 && e >= -64) {
        k = (uint32_t)-e;
        F = k >= 64 ? m : (m & ((1ull << k) - 1));
        I = k >= 64 ? 0 : (m >> k);
        return true;
    }
    if (e >= 0 && e <= 10 && (m << e) < 100000000000000000ull) {
        k = 0;
        F = 0;
        I = m << e;
        return true;
    }
    return false;
}

typedef unsigned __int128 u128;
__device__ inline u128 low_bits(uint32_t k) { return (((u128)1) << k) - 1; }  // k <= 64

__constant__ uint64_t kPow10[20] = {1ull,
                                    10ull,
                                    100ull,
                                    1000ull,
                                    10000ull,
                                    100000ull,
                                    1000000ull,
                                    10000000ull,
                                    100000000ull,
                                    1000000000ull,
                                    10000000000ull,
                                    100000000000ull,
                                    1000000000000ull,
                                    10000000000000ull,
                                    100000000000000ull,
                                    1000000000000000ull,
                                    10000000000000000ull,
                                    100000000000000000ull,
                                    1000000000000000000ull,
                                    10000000000000000000ull};

__device__ inline uint32_t tz_dec(uint32_t v) {  // trailing decimal zeros of 0 < v < 1e9
    uint32_t z = 0;
    if (v % 100000000u == 0) z += 8, v /= 100000000u;
    if (v % 10000u == 0) z += 4, v /= 10000u;
    if (v % 100u == 0) z += 2, v /= 100u;
    if (v % 10u == 0) z += 1;
    return z;
}

template <class S>
__device__ __noinline__ S fmt_fixed6_slow(S s, double v);
template <class S>
__device__ __noinline__ S fmt_g17_slow(S s, double v);

// "%f" (std::to_string(double), src/order_types.cpp:164): all integer digits, six decimals,
// round half to even on the exact value; inf / nan as glibc prints them.
template <class S>
__device__ OJ_HELPER S fmt_fixed6(S s, double v) {
    const uint64_t bits = (uint64_t)__double_as_longlong(v);
    const bool neg = (bits >> 63) != 0;
    if (__builtin_isnan(v)) {
        if (neg) s.put('-');
        lit(s, "nan");
        return s;
    }
    if (neg) s.put('-');
    if (__builtin_isinf(v)) {
        lit(s, "inf");
        return s;
    }
    if ((bits << 1) == 0) {
        lit(s, "0.000000");
        return s;
    }
    uint64_t I, F;
    uint32_t k;
    if (!small_parts(v, I, F, k)) return fmt_fixed6_slow(s, v);
    uint32_t kept = 0;  // the six decimals, rounded half to even on the exact remainder
    if (k) {
        const u128 t = (u128)F * 1000000u;
        kept = (uint32_t)(t >> k);
        const u128 rem = t & low_bits(k), half = ((u128)1) << (k - 1);
        if (rem > half || (rem == half && (kept & 1)))
            if (++kept == 1000000u) kept = 0, ++I;
    }
    dec_u64(s, I);
    s.put('.');
    s.run(make_uint4(asc4(kept / 10000u), asc4(kept % 10000u), 0u, 0u), 2, 6);
    return s;
}

template <class S>
__device__ __noinline__ S fmt_fixed6_slow(S s, double v) {  // |v| outside the register path (sign printed)
    Exact x;
    x.init(v);
    const uint32_t c1 = x.frac_next9();
    uint32_t kept = c1 / 1000;
    const uint32_t rest = c1 % 1000;
    const bool up = rest > 500 || (rest == 500 && (x.frac_nonzero() || (kept & 1)));
    bool carry = false;
    if (up && ++kept == 1000000) kept = 0, carry = true;
    if (carry && x.small) {
        x.set_small_int(x.sI + 1);
    } else if (carry) {  // add one to the integer limbs
        int j = x.nl - 1;
        for (; j >= 0; --j) {
            if (++x.lim[j] < kE9) break;
            x.lim[j] = 0;
        }
        if (j < 0) {  // all limbs overflowed (or there were none): a new leading limb 1
            for (int q = x.nl; q > 0; --q) x.lim[q] = x.lim[q - 1];
            x.lim[0] = 1;
            ++x.nl;
        }
    }
    if (x.nl == 0) {
        s.put('0');
    } else {
        dec_u64(s, x.limb(0));
        for (int j = 1; j < x.nl; ++j)
            put_digits(s, x.limb(j), 9);
    }
    s.put('.');
    put_digits(s, kept, 6);
    return s;
}

// jsoncpp valueToString(double, false, 17, significantDigits): "%.17g" then ".0" when the text
// has neither '.' nor 'e'; NaN → null, ±inf → ±1e+9999.
template <class S>
__device__ OJ_HELPER S fmt_g17(S s, double v) {
    const uint64_t bits = (uint64_t)__double_as_longlong(v);
    if (__builtin_isnan(v)) {
        lit(s, "null");
        return s;
    }
    const bool neg = (bits >> 63) != 0;
    if (__builtin_isinf(v)) {
        if (neg) lit(s, "-1e+9999");
        else lit(s, "1e+9999");
        return s;
    }
    if (neg) s.put('-');
    if ((bits << 1) == 0) {
        lit(s, "0.0");
        return s;
    }
    uint64_t I, F;
    uint32_t k;
    if (!small_parts(v, I, F, k)) return fmt_g17_slow(s, v);
    // D: the first 18 significant digits, X: the decimal exponent of the first, sticky: any
    // nonzero digit past them
    uint64_t D;
    int X;
    bool sticky;
    if (I) {
        const uint32_t nd = ndig64(I);  // 1..17
        const uint64_t p = kPow10[18 - nd];
        const u128 t = (u128)F * p;
        D = I * p + (k ? (uint64_t)(t >> k) : 0ull);
        sticky = k && (t & low_bits(k)) != 0;
        X = (int)nd - 1;
    } else {  // 0 < F / 2^k < 1: nine-digit chunks until the first nonzero one
        X = -1;
        uint32_t c;
        for (;;) {
            const u128 t = (u128)F * kE9;
            c = (uint32_t)(t >> k);
            F = (uint64_t)(t & low_bits(k));
            if (c) break;
            X -= 9;
        }
        const uint32_t w0 = ndig64(c);
        X -= 9 - (int)w0;
        const uint64_t p = kPow10[18 - w0];
        const u128 t = (u128)F * p;
        D = (uint64_t)c * p + (uint64_t)(t >> k);
        sticky = (t & low_bits(k)) != 0;
    }
    // round to 17 digits, half to even
    uint64_t M = D / 10;
    const uint32_t r = (uint32_t)(D - 10 * M);
    M += (r > 5 || (r == 5 && (sticky || (M & 1)))) ? 1 : 0;
    if (M == 100000000000000000ull) M = 10000000000000000ull, ++X;
    const uint32_t mhi = (uint32_t)(M / 100000000u), mlo = (uint32_t)(M - (uint64_t)mhi * 100000000u);
    const int last = 16 - (int)(mlo ? tz_dec(mlo) : 8 + tz_dec(mhi));  // trailing zeros dropped
    const Dec20 dg = dec20(M);  // digit j of the 17 at byte 3 + j
    if (X < -4 || X >= 17) {
        dec_run(s, dg, 3, 1);
        if (last > 0) {
            s.put('.');
            dec_run(s, dg, 4, (uint32_t)last);
        }
        s.put('e');
        int ax = X;
        if (ax < 0) s.put('-'), ax = -ax;
        else s.put('+');
        if (ax < 10) s.put('0');
        dec_u64(s, (uint64_t)ax);
    } else if (X >= 0) {
        dec_run(s, dg, 3, (uint32_t)X + 1);
        if (last > X) {
            s.put('.');
            dec_run(s, dg, 4 + (uint32_t)X, (uint32_t)(last - X));
        } else {
            lit(s, ".0");
        }
    } else {
        s.put('0');
        s.put('.');
        for (int j = 0; j < -X - 1; ++j) s.put('0');
        dec_run(s, dg, 3, (uint32_t)last + 1);
    }
    return s;
}

template <class S>
__device__ __noinline__ S fmt_g17_slow(S s, double v) {  // |v| outside the register path (sign printed)
    Exact x;
    x.init(v);
    // first 18 significant digits of the expansion, the decimal exponent X of the first, sticky
    uint8_t d[18];
    int cnt = 0, X = 0;
    bool sticky = false;
    auto take = [&](uint32_t chunk, int width) {  // `width` digits of chunk, most significant first
        uint8_t dg[9];
        split9(chunk, dg);
#pragma unroll
        for (int q = 0; q < 9; ++q) {
            if (q < 9 - width) continue;
            if (cnt < 18) d[cnt++] = dg[q];
            else if (dg[q]) sticky = true;
        }
    };
    if (x.nl) {
        const int w0 = ndig9(x.limb(0));
        X = w0 - 1 + 9 * (x.nl - 1);
        take(x.limb(0), w0);
        for (int j = 1; j < x.nl; ++j) take(x.limb(j), 9);
    } else {
        X = -1;
        uint32_t c;
        while ((c = x.frac_next9()) == 0) X -= 9;
        const int w0 = ndig9(c);
        X -= 9 - w0;
        take(c, w0);
    }
    while (cnt < 18 && x.frac_nonzero()) take(x.frac_next9(), 9);
    while (cnt < 18) d[cnt++] = 0;
    if (x.frac_nonzero()) sticky = true;
    // round to 17 digits, half to even
    const bool up = d[17] > 5 || (d[17] == 5 && (sticky || (d[16] & 1)));
    if (up) {
        int j = 16;
        for (; j >= 0; --j) {
            if (++d[j] < 10) break;
            d[j] = 0;
        }
        if (j < 0) d[0] = 1, ++X;  // 99..9 → 10..0
    }
    int last = 16;  // trailing zeros are dropped (%g without '#')
    while (last > 0 && d[last] == 0) --last;
    if (X < -4 || X >= 17) {
        s.put((uint8_t)('0' + d[0]));
        if (last > 0) {
            s.put('.');
            for (int j = 1; j <= last; ++j) s.put((uint8_t)('0' + d[j]));
        }
        s.put('e');
        int ax = X;
        if (ax < 0) s.put('-'), ax = -ax;
        else s.put('+');
        if (ax < 10) s.put('0');
        dec_u64(s, (uint64_t)ax);
        return s;  // has an 'e': no ".0"
    }
    if (X >= 0) {
        for (int j = 0; j <= X; ++j) s.put((uint8_t)('0' + d[j]));
        if (last > X) {
            s.put('.');
            for (int j = X + 1; j <= last; ++j) s.put((uint8_t)('0' + d[j]));
        } else {
            lit(s, ".0");
        }
    } else {
        s.put('0');
        s.put('.');
        for (int j = 0; j < -X - 1; ++j) s.put('0');
        for (int j = 0; j <= last; ++j) s.put((uint8_t)('0' + d[j]));
    }
    return s;
}

// status == "UPDATED" || status == "CANCELLED" (publish_order's messageType choice): the string's
// first 16 bytes from the one or two blocks holding them, compared as two 64-bit words (instead of
// a byte loop over two literals)
template <class P>
__device__ inline bool is_update_status(P p, uint64_t n) {
    if (n != 7 && n != 9) return false;
    BlockReader<P> rd;
    (void)rd.at(p);
    const uint4 v0 = rd.v;
    const uint32_t o = (uint32_t)((uintptr_t)p & 15);
    uint4 v1 = make_uint4(0u, 0u, 0u, 0u);
    if (o + n > 16) {
        (void)rd.at(p + (16 - o));
        v1 = rd.v;
    }
    const u128 a = (u128)v0.x | (u128)v0.y << 32 | (u128)v0.z << 64 | (u128)v0.w << 96;
    const u128 b = (u128)v1.x | (u128)v1.y << 32 | (u128)v1.z << 64 | (u128)v1.w << 96;
    const u128 w = o ? (a >> (8 * o)) | (b << (8 * (16 - o))) : a;
    const uint64_t lo = (uint64_t)w, hi = (uint64_t)(w >> 64);
    constexpr uint64_t kUpdated = 0x0044455441445055ull;    // "UPDATED" little-endian
    constexpr uint64_t kCancelle = 0x454c4c45434e4143ull;   // "CANCELLE"
    return n == 7 ? (lo & 0x00ffffffffffffffull) == kUpdated : (lo == kCancelle && (hi & 0xff) == 'D');
}

// One Order's text (src/order_types.cpp:122-181, src/cluster_client.cpp:308-323).
template <uint32_t kWhat, class S, class P>
__device__ __forceinline__ void order_text(S& s, const JsonArgs& a, uint64_t i, P const f[kFields],
                           const uint32_t l[kFields]) {
    if (kWhat == SBE_JSON_PUBLISH_HEADERS) {
        const bool upd = is_update_status(f[7], l[7]);
        lit(s, "{\"messageId\":");
        s = quoted(s, f[6], l[6]);
        if (upd) lit(s, ",\"messageType\":\"UPDATE_ORDER\",\"orderId\":");
        else lit(s, ",\"messageType\":\"CREATE_ORDER\",\"orderId\":");
        s = quoted(s, f[5], l[5]);
        s.put('}');
        return;
    }
    const double q = a.quantity[i];
    uint32_t id_len = l[1];  // headers["origin_id"] = identifier.c_str(): up to the first NUL
    {
        BlockReader<P> rd;
        for (uint32_t j = 0; j < id_len;) {  // one SWAR test per 16-byte block
            (void)rd.at(f[1] + j);
            const uint32_t o = (uint32_t)((uintptr_t)(f[1] + j) & 15);
            const uint32_t nul = (nul16(rd.v) >> o) & ((1u << (16 - o)) - 1);
            if (nul) {
                const uint32_t at = j + (uint32_t)__builtin_ctz(nul);
                id_len = at < id_len ? at : id_len;
                break;
            }
            j += 16 - o;
        }
    }
    lit(s, "{\"message\":{\"headers\":{\"auth_token\":\"Bearer xxx\",\"connection_uuid\":\"130032\",\"create_ts\":\"");
    dec_i64(s, a.timestamp[i] / 1000000);
    lit(s, "\",\"customer_id\":\"");
    dec_i64(s, a.customer_id[i]);
    lit(s, "\",\"ip_address\":\"10.37.62.251\",\"origin\":\"fix\",\"origin_id\":");
    s = quoted(s, f[1], id_len);
    lit(s, ",\"origin_name\":\"FIX_GATEWAY\"},\"message\":{\"action\":\"CREATE\",\"order_details\":{\"client_order_id\":");
    s = quoted(s, f[0], l[0]);
    lit(s, ",\"order_type\":\"market\",\"quantity\":{\"token\":");
    s = quoted(s, f[2], l[2]);
    lit(s, ",\"value\":");
    s = fmt_g17(s, q);
    lit(s, "},\"quantity_value_str\":\"");
    s = fmt_fixed6(s, q);
    lit(s, "\",\"side\":");
    s = quoted(s, f[4], l[4]);
    lit(s, ",\"token_pair\":{\"base_token\":");
    s = quoted(s, f[2], l[2]);
    lit(s, ",\"quote_token\":");
    s = quoted(s, f[3], l[3]);
    lit(s, "}}}},\"msg_type\":\"D\",\"uuid\":");
    s = quoted(s, f[0], l[0]);
    s.put('}');
}


// ---- offsets without a device-wide scan library call ----
// Orders are taken in blocks of kBlock: a block's string bytes (packed arena) and text bytes are
// summed per block, the block sums scanned by one small launch, and each Order's offset is its
// block's prefix plus a scan inside the block (sizing launch: string bases; writing launch: text
// offsets, from the sizes of the block's earlier Orders).

// exclusive scan of v over the block (every thread calls it); total = the block's sum
__device__ inline uint64_t block_excl_scan(uint64_t v, uint64_t* wtot, uint32_t lane, uint32_t wv, uint64_t& total) {
    const uint64_t incl = wave_incl_scan64(v, (int)lane);
    if (lane == kWave - 1) wtot[wv] = incl;
    __syncthreads();
    uint64_t before = 0;
    total = 0;
    for (uint32_t w = 0; w < kBlock / kWave; ++w) {
        const uint64_t t = wtot[w];
        before += w < wv ? t : 0;
        total += t;
    }
    __syncthreads();
    return before + incl - v;
}

// Packed arena: each block's string bytes into blk_str.
__global__ __launch_bounds__(kBlock) void order_json_totals(JsonArgs a) {
    __shared__ uint64_t wtot[kBlock / kWave];
    const uint64_t i = (uint64_t)blockIdx.x * kBlock + threadIdx.x;
    uint64_t t = 0;
    if (i < a.n)
        for (uint32_t j = 0; j < kFields; ++j) t += a.str_len[kFields * i + j];
    uint64_t total;
    (void)block_excl_scan(t, wtot, threadIdx.x % kWave, threadIdx.x / kWave, total);
    if (threadIdx.x == 0) a.blk_str[blockIdx.x] = total;
}

// Exclusive scan of v[0, m) in place: one block of 1024 threads, 4096 values per step.
constexpr uint32_t kScanThreads = 1024;
__global__ __launch_bounds__(kScanThreads) void order_json_scan_blocks(uint64_t* v, uint64_t m) {
    __shared__ uint64_t wt[kScanThreads / kWave];
    const uint32_t lane = threadIdx.x % kWave, wv = threadIdx.x / kWave;
    uint64_t carry = 0;
    for (uint64_t c0 = 0; c0 < m; c0 += 4 * kScanThreads) {
        const uint64_t k0 = c0 + 4 * (uint64_t)threadIdx.x;
        uint64_t x[4], sum = 0;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            x[r] = k0 + r < m ? v[k0 + r] : 0;
            sum += x[r];
        }
        const uint64_t incl = wave_incl_scan64(sum, (int)lane);
        if (lane == kWave - 1) wt[wv] = incl;
        __syncthreads();
        uint64_t before = carry, tot = 0;
        for (uint32_t w = 0; w < kScanThreads / kWave; ++w) {
            const uint64_t t = wt[w];
            before += w < wv ? t : 0;
            tot += t;
        }
        __syncthreads();
        uint64_t run = before + incl - sum;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            if (k0 + r < m) v[k0 + r] = run;
            run += x[r];
        }
        carry += tot;
    }
}

// Sizing launch: the text length of record i into sz[i], the block's text bytes into blk_txt
// (and, packed arena, the string base of record i into str_base[i]).  With a packed arena the
// strings of a wave's 64 Orders are one contiguous range: the wave copies it into LDS with
// coalesced 16-byte loads issued back to back, and sizes the texts from there, instead of each
// lane walking its strings with a chain of dependent HBM loads (the launch's latency bound).  A
// range larger than the wave's LDS share is read from HBM as before.
#ifndef SBE_OJ_MSTR  // LDS bytes per wave for the staged strings (0: never staged)
#define SBE_OJ_MSTR 10240
#endif
// A/B builds: 0 = headers texts (3 of the 8 strings) sized from HBM, not staged: measured slower
// (row 0.560 -> 0.580 ms, profiles/r05_ab_ojhstage.log), so the headers launch stages all 8 as well
#ifndef SBE_OJ_HSTAGE
#define SBE_OJ_HSTAGE 1
#endif
template <uint32_t kWhat>
__global__ __launch_bounds__(kBlock) void order_json_measure(JsonArgs a) {
    __shared__ uint64_t wtot[kBlock / kWave];
    const uint64_t i = (uint64_t)blockIdx.x * kBlock + threadIdx.x;
    const bool live = i < a.n;
    const uint32_t lane = threadIdx.x % kWave, wv = threadIdx.x / kWave;
    uint32_t l[kFields];
    uint64_t tot = 0;
    if (live)
        for (uint32_t j = 0; j < kFields; ++j) {
            l[j] = a.str_len[kFields * i + j];
            tot += l[j];
        }
    uint64_t len = 0, total;
    bool done = false;
    if (!a.str_off) {  // uniform over the launch
        const uint64_t base = a.blk_str[blockIdx.x] + block_excl_scan(tot, wtot, lane, wv, total);
        if (live) a.str_base[i] = base;
#if SBE_OJ_MSTR > 0
        typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
        constexpr bool kStage = kWhat != SBE_JSON_PUBLISH_HEADERS || SBE_OJ_HSTAGE;
        __shared__ __attribute__((aligned(16))) uint8_t sbuf[kBlock / kWave][kStage ? SBE_OJ_MSTR : 16];
        const uint64_t i0 = i - lane;
        bool staged = false;
        uint64_t g0 = 0;
        if (kStage && i0 < a.n) {  // uniform per wave
            g0 = lane_u64(base, 0) & ~15ull;
            const uint64_t last = a.n - 1 - i0 < kWave - 1 ? a.n - 1 - i0 : kWave - 1;
            const uint64_t end = lane_u64(base + tot, (int)last);
            staged = end - g0 <= (kStage ? SBE_OJ_MSTR : 0);
            if (staged) {
                typedef const __attribute__((address_space(1))) u32x4 g128;
                typedef __attribute__((address_space(3))) u32x4 l128;
                const uint64_t nb = (end - g0 + 15) / 16;
                for (uint64_t c = lane; c < nb; c += kWave) {
                    const uint64_t o = g0 + 16 * c;
                    if (o + 16 <= end) {
                        *(l128*)(sbuf[wv] + 16 * c) = *(g128*)(a.arena + o);
                    } else {  // the range's partial last chunk: bytewise, never past the wave's last
                              // string byte (the arena may end there, at the end of a mapping)
                        for (uint64_t k = 0; k < end - o; ++k) sbuf[wv][16 * c + k] = a.arena[o + k];
                    }
                }
            }
        }
        __syncthreads();
        if (staged && live) {
            lr8* f[kFields];
            uint64_t at = base - g0;
            for (uint32_t j = 0; j < kFields; ++j) {
                f[j] = (lr8*)(sbuf[wv] + at);
                at += l[j];
            }
            CountSink c;
            order_text<kWhat>(c, a, i, f, l);
            len = c.n;
        }
        done = staged;
#endif
        if (!done && live) {
            gu8* f[kFields];
            uint64_t at = base;
            for (uint32_t j = 0; j < kFields; ++j) {
                f[j] = (gu8*)(a.arena + at);
                at += l[j];
            }
            CountSink c;
            order_text<kWhat>(c, a, i, f, l);
            len = c.n;
        }
    } else if (live) {
        gu8* f[kFields];
        for (uint32_t j = 0; j < kFields; ++j) f[j] = (gu8*)(a.arena + a.str_off[kFields * i + j]);
        CountSink c;
        order_text<kWhat>(c, a, i, f, l);
        len = c.n;
    }
    if (live) a.sz[i] = len;
    (void)block_excl_scan(len, wtot, lane, wv, total);
    if (threadIdx.x == 0) a.blk_txt[blockIdx.x] = total;
}

// Writing launch: one wave per kOpw Orders (WShape).  Their texts are contiguous in `out`: the
// wave stages them in an LDS window (byte writes; a plain string run as one 16-byte store), stores the window with 16-byte
// coalesced stores and moves the window on to the first record not yet written, until every record
// is out.  Only a record larger than the window is written from its lane straight to HBM.  Records
// past out_capacity are written by nobody.  The window is sized so that a wave's texts fit it in
// one pass (a second pass would serialise the lanes it leaves over): payload texts (~560 B) 32 per
// wave in 18 KiB, headers texts (~95 B) 64 per wave in 8 KiB; 8 waves per CU either way (the
// payload writer's 207 VGPRs allow 2 per SIMD).  Measured (1 M orders, both texts): 64 payload
// texts in a 24 KiB window (two passes) 1.54 ms, 32 in 18 KiB 1.29 ms, plus the 8 KiB headers
// window 1.25 ms.
constexpr uint32_t kWWave = 64;
#ifndef SBE_OJ_WIN
#define SBE_OJ_WIN 18432
#endif
#ifndef SBE_OJ_OPW
#define SBE_OJ_OPW 32
#endif
#ifndef SBE_OJ_HDR_WIN
#define SBE_OJ_HDR_WIN 8192
#endif
// Orders per wave (lanes past it idle) and LDS window bytes of the writing launch, per text kind
template <uint32_t kWhat>
struct WShape {
    static constexpr uint32_t kOpw = kWhat == SBE_JSON_PUBLISH_HEADERS ? 64u : (uint32_t)SBE_OJ_OPW;
    static constexpr uint32_t kWinB = kWhat == SBE_JSON_PUBLISH_HEADERS ? (uint32_t)SBE_OJ_HDR_WIN : (uint32_t)SBE_OJ_WIN;
};
static_assert(SBE_OJ_WIN >= 4096 && SBE_OJ_HDR_WIN >= 4096, "the window must hold a typical record");

__device__ inline uint64_t wave_max(uint64_t v) {
    for (int d = 32; d >= 1; d >>= 1) {
        const uint64_t t = __shfl_xor(v, d, kWWave);
        v = t > v ? t : v;
    }
    return v;
}

// The staging and storing half of the writing launch: every live lane knows its text's output
// range [o, e) and its fields; the wave's texts go through the LDS window `win`.
template <uint32_t kWhat, class P>
__device__ __forceinline__ void write_texts(const JsonArgs& a, lw8* win, uint32_t lane, uint64_t i, bool live,
                                            uint64_t o, uint64_t e, P const f[kFields], const uint32_t l[kFields]) {
    constexpr uint32_t kWin = WShape<kWhat>::kWinB;
    bool done = true;
    if (live) {
        const bool fits = e <= a.cap;
        if (a.status) a.status[i] = fits ? SBE_JSON_OK : SBE_JSON_OVERFLOW;
        done = !fits;
        if (fits && e - o > kWin - 16) {  // larger than any window: straight to HBM
            HbmSink w((gw8*)(a.out + o));
            order_text<kWhat>(w, a, i, f, l);
            done = true;
        }
    }
    uint64_t start = ~0ull;  // output coordinate of the first record still to stage
    for (int d = 32; d >= 1; d >>= 1) {
        const uint64_t t = __shfl_xor(done ? ~0ull : o, d, kWWave);
        start = t < start ? t : start;
    }
    start = done ? start : (o < start ? o : start);
    for (int d = 32; d >= 1; d >>= 1) {
        const uint64_t t = __shfl_xor(start, d, kWWave);
        start = t < start ? t : start;
    }
    while (start != ~0ull) {  // uniform: every lane holds the same start
        const uint64_t wbase = start - (uint64_t)((uintptr_t)(a.out + start) & 15);  // win[0] ≡ out + wbase (mod 16)
        uint64_t my_end = 0;
        if (!done && e - wbase <= kWin) {
            LdsSink w(win + (o - wbase), (uint32_t)(e - o));
            order_text<kWhat>(w, a, i, f, l);
            done = true;
            my_end = e;
        }
        const uint64_t cend = wave_max(my_end);
        __syncthreads();
        const uint64_t nch = (cend - wbase + 15) / 16;
        for (uint64_t c = lane; c < nch; c += kWWave) {
            const uint64_t x0 = wbase + 16 * c;  // output coordinate of this 16-byte chunk
            if (x0 >= start && x0 + 16 <= cend) {
                typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
                typedef const __attribute__((address_space(3))) u32x4 lu128;
                const u32x4 v = *(lu128*)(win + 16 * c);
                // out + x0 is 16-byte aligned (wbase's choice): one dwordx4 store a chunk
                __builtin_nontemporal_store(v, reinterpret_cast<u32x4*>(a.out + x0));
            } else {
                for (uint64_t x = x0 < start ? start : x0; x < x0 + 16 && x < cend; ++x) a.out[x] = win[x - wbase];
            }
        }
        __syncthreads();
        uint64_t nx = done ? ~0ull : o;
        for (int d = 32; d >= 1; d >>= 1) {
            const uint64_t t = __shfl_xor(nx, d, kWWave);
            nx = t < nx ? t : nx;
        }
        start = nx;
    }
}

#ifndef SBE_OJ_MINW  // A/B builds: minimum waves per SIMD the writing launch's registers must allow
#define SBE_OJ_MINW 1
#endif
template <uint32_t kWhat>
__global__ __launch_bounds__(kWWave, SBE_OJ_MINW) void order_json_write(JsonArgs a) {
    constexpr uint32_t kOpw = WShape<kWhat>::kOpw;
    static_assert(kBlock % kOpw == 0, "a writing tile lies inside one sizing block");
    __shared__ __attribute__((aligned(16))) uint8_t win[WShape<kWhat>::kWinB];
    const uint32_t lane = threadIdx.x;
    const uint64_t i0 = (uint64_t)blockIdx.x * kOpw, i = i0 + lane;
    const bool live = lane < kOpw && i < a.n;
    // text offsets: the block's prefix, the sizes of the block's Orders before the tile, the tile's scan
    const uint64_t bs = i0 / kBlock * kBlock;
    uint64_t pre = 0;
#pragma unroll
    for (uint32_t r = 0; r < kBlock / kWave; ++r) {
        const uint64_t k = bs + lane + kWave * r;
        if (k < i0) pre += a.sz[k];
    }
    pre = a.blk_txt[i0 / kBlock] + wave_sum64(pre);
    const uint64_t len = live ? a.sz[i] : 0;
    const uint64_t o = pre + wave_incl_scan64(len, (int)lane) - len, e = o + len;
    uint32_t l[kFields];
    if (live) {
        a.out_off[i] = o;
        if (i + 1 == a.n) a.out_off[a.n] = e;
        for (uint32_t j = 0; j < kFields; ++j) l[j] = a.str_len[kFields * i + j];
    }
    gu8* f[kFields];
    if (live) {
        uint64_t at = a.str_off ? 0 : a.str_base[i];
        for (uint32_t j = 0; j < kFields; ++j) {
            if (a.str_off) {
                f[j] = (gu8*)(a.arena + a.str_off[kFields * i + j]);
            } else {
                f[j] = (gu8*)(a.arena + at);
                at += l[j];
            }
        }
    }
    write_texts<kWhat>(a, (lw8*)win, lane, i, live, o, e, f, l);
}



}  // namespace oj
