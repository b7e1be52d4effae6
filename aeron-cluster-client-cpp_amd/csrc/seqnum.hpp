// seqnum.hpp — included by sbe_codec.hip inside its anonymous namespace.
//
// ParseResult.sequence_number on the device (src/sbe_encoder.cpp:1031-1125): the payload is
// parsed with the semantics of jsoncpp 1.9.5's CharReaderBuilder defaults (OurReader: comments
// and trailing commas allowed, extra content after the root ignored, no single quotes / numeric
// keys / special floats, stack limit 1000, UTF-8 BOM skipped; a NUL byte outside a string ends
// the stream), then "_sequence_number" is looked up in root, root.message, root.message.message
// and root.message.message.message; the first non-zero extractSequence value wins.  Any parse
// failure or exception gives 0.  jsoncpp is absent from this image: parity with it is unpinned;
// the tests check this code against the oracle's restatement (oracle/sbe_oracle.c
// orc_seq_eval), which converts decimals with glibc strtod where this code rounds exactly with
// integer arithmetic (jnum_seq).
//
// One lane per flagged record: the work is serial byte parsing of rare records (payloads that
// contain the key or a backslash, SBE_FL_SEQ_KEY / SBE_FL_SEQ_ESC).  The decode kernel calls it
// out of line (json_seq_eval_call) after its descriptor stores, from the lanes that hold such a
// record, so it does not widen the kernel's register budget; sbe_seqnum_kernel runs the same
// reader as a standalone launch over finished descriptors (sbe_eval_sequence_numbers).

enum : int { JT_OBEG, JT_OEND, JT_ABEG, JT_AEND, JT_STR, JT_NUM, JT_LIT, JT_COMMA, JT_COLON, JT_COMMENT,
             JT_EOS, JT_ERR };

struct JCur {
    const uint8_t* p;
    uint32_t n, i;
    __device__ __forceinline__ int get() { return i < n ? p[i++] : 0; }  // OurReader::getNextChar
    __device__ __forceinline__ void skip_spaces() {
        while (i < n) {
            const uint8_t c = p[i];
            if (c != ' ' && c != '\t' && c != '\r' && c != '\n') break;
            ++i;
        }
    }
    __device__ __forceinline__ bool match(const char* pat, uint32_t k) {  // OurReader::match
        if (n - i < k) return false;
        for (uint32_t j = 0; j < k; ++j)
            if (p[i + j] != (uint8_t)pat[j]) return false;
        i += k;
        return true;
    }
};

// OurReader::readToken (after skipSpaces); [s, e) is the token
__device__ int jtoken(JCur& c, uint32_t& s, uint32_t& e) {
    c.skip_spaces();
    s = c.i;
    const int ch = c.get();
    int t = JT_ERR;
    switch (ch) {
        case '{': t = JT_OBEG; break;
        case '}': t = JT_OEND; break;
        case '[': t = JT_ABEG; break;
        case ']': t = JT_AEND; break;
        case ',': t = JT_COMMA; break;
        case ':': t = JT_COLON; break;
        case 0: t = JT_EOS; break;
        case '"': {  // readString: the last character read must be the closing quote
            int last = 0;
            while (c.i < c.n) {
                last = c.get();
                if (last == '\\') c.get();
                else if (last == '"') break;
            }
            t = last == '"' ? JT_STR : JT_ERR;
            break;
        }
        case '/': {  // readComment
            const int x = c.get();
            if (x == '*') {  // readCStyleComment: scans while one byte remains, then wants '/'
                while (c.i + 1 < c.n) {
                    const int y = c.get();
                    if (y == '*' && c.p[c.i] == '/') break;
                }
                t = c.get() == '/' ? JT_COMMENT : JT_ERR;
            } else if (x == '/') {  // readCppStyleComment
                while (c.i < c.n) {
                    const int y = c.get();
                    if (y == '\n') break;
                    if (y == '\r') {
                        if (c.i < c.n && c.p[c.i] == '\n') ++c.i;
                        break;
                    }
                }
                t = JT_COMMENT;
            }
            break;
        }
        case 't': t = c.match("rue", 3) ? JT_LIT : JT_ERR; break;
        case 'f': t = c.match("alse", 4) ? JT_LIT : JT_ERR; break;
        case 'n': t = c.match("ull", 3) ? JT_LIT : JT_ERR; break;
        default:
            if (ch == '-' && c.i < c.n && c.p[c.i] == 'I') {  // readNumber(true): -Infinity, not allowed
                ++c.i;
            } else if ((ch >= '0' && ch <= '9') || ch == '-') {  // readNumber
                uint32_t k = c.i;
                int x = '0';
                auto nx = [&] { c.i = k; x = k < c.n ? c.p[k++] : 0; };
                while (x >= '0' && x <= '9') nx();
                if (x == '.') {
                    nx();
                    while (x >= '0' && x <= '9') nx();
                }
                if (x == 'e' || x == 'E') {
                    nx();
                    if (x == '+' || x == '-') nx();
                    while (x >= '0' && x <= '9') nx();
                }
                t = JT_NUM;
            }
            break;
    }
    e = c.i;
    return t;
}

// --- decodeString, streamed into a sink (codePointToUTF8 for \u escapes) -------------------
__device__ __forceinline__ bool jhex4(const uint8_t* p, uint32_t i, uint32_t end, uint32_t& v) {
    if (end - i < 4) return false;
    uint32_t r = 0;
    for (int j = 0; j < 4; ++j) {
        const uint32_t h = p[i + j];
        r <<= 4;
        if (h >= '0' && h <= '9') r |= h - '0';
        else if (h >= 'a' && h <= 'f') r |= h - 'a' + 10;
        else if (h >= 'A' && h <= 'F') r |= h - 'A' + 10;
        else return false;
    }
    v = r;
    return true;
}
template <class Sink>
__device__ __forceinline__ void jutf8(uint32_t cp, Sink& k) {
    if (cp <= 0x7f) {
        k.put(cp);
    } else if (cp <= 0x7ff) {
        k.put(0xc0 | (cp >> 6));
        k.put(0x80 | (cp & 0x3f));
    } else if (cp <= 0xffff) {
        k.put(0xe0 | (cp >> 12));
        k.put(0x80 | ((cp >> 6) & 0x3f));
        k.put(0x80 | (cp & 0x3f));
    } else if (cp <= 0x10ffff) {
        k.put(0xf0 | (cp >> 18));
        k.put(0x80 | ((cp >> 12) & 0x3f));
        k.put(0x80 | ((cp >> 6) & 0x3f));
        k.put(0x80 | (cp & 0x3f));
    }
}
template <class Sink>
__device__ bool jdecode_string(const uint8_t* p, uint32_t s, uint32_t e, Sink& k) {
    uint32_t i = s + 1;
    const uint32_t end = e - 1;
    while (i < end) {
        const uint32_t ch = p[i++];
        if (ch == '"') break;
        if (ch != '\\') {
            k.put(ch);
            continue;
        }
        if (i == end) return false;  // "Empty escape sequence in string"
        const uint32_t x = p[i++];
        switch (x) {
            case '"': k.put('"'); break;
            case '/': k.put('/'); break;
            case '\\': k.put('\\'); break;
            case 'b': k.put('\b'); break;
            case 'f': k.put('\f'); break;
            case 'n': k.put('\n'); break;
            case 'r': k.put('\r'); break;
            case 't': k.put('\t'); break;
            case 'u': {
                uint32_t cp;
                if (!jhex4(p, i, end, cp)) return false;
                i += 4;
                if (cp >= 0xD800 && cp <= 0xDBFF) {  // surrogate pair: "\uXXXX" must follow
                    if (end - i < 6 || p[i] != '\\' || p[i + 1] != 'u') return false;
                    uint32_t lo;
                    if (!jhex4(p, i + 2, end, lo)) return false;
                    i += 6;
                    cp = 0x10000 + ((cp & 0x3FF) << 10) + (lo & 0x3FF);
                }
                jutf8(cp, k);
                break;
            }
            default: return false;  // "Bad escape sequence in string"
        }
    }
    return true;
}

struct NullSink {
    __device__ __forceinline__ void put(uint32_t) {}
};
// member name: "_sequence_number" or "message"?
struct KeySink {
    uint32_t len = 0;
    bool seq = true, msg = true;
    __device__ __forceinline__ void put(uint32_t ch) {
        // the names' bytes, little-endian: "_sequenc" "e_number", "message"
        constexpr uint64_t kS0 = 0x636e65757165735full, kS1 = 0x7265626d756e5f65ull, kM = 0x006567617373656dull;
        const uint32_t es = (uint32_t)(((len < 8 ? kS0 : kS1) >> (8 * (len & 7))) & 0xff);
        const uint32_t em = (uint32_t)((kM >> (8 * (len & 7))) & 0xff);
        seq = seq && len < 16 && ch == es;
        msg = msg && len < 7 && ch == em;
        ++len;
    }
};
// std::stoull(asString()) (base 10, over c_str(): stops at a NUL); invalid_argument /
// out_of_range are caught by extractSequence and give 0
struct StoullSink {
    uint64_t v = 0;
    uint32_t phase = 0;  // 0 leading space, 1 after the sign, 2 digits, 3 stopped
    bool neg = false, any = false, ovf = false;
    __device__ __forceinline__ void put(uint32_t ch) {
        if (phase == 3) return;
        if (ch == 0) {
            phase = 3;
            return;
        }
        if (phase == 0) {
            if (ch == ' ' || (ch >= 9 && ch <= 13)) return;
            phase = 1;
            if (ch == '+' || ch == '-') {
                neg = ch == '-';
                return;
            }
        }
        if (ch >= '0' && ch <= '9') {
            const uint64_t dg = ch - '0';
            any = true;
            if (v > (~0ull - dg) / 10) ovf = true;
            else v = v * 10 + dg;
            phase = 2;
        } else {
            phase = 3;
        }
    }
    __device__ __forceinline__ uint64_t value() const { return (!any || ovf) ? 0 : (neg ? 0 - v : v); }
};

// --- numbers: decodeNumber / decodeDouble, then extractSequence ----------------------------
// Decimal digits of 1 - 2^-q (q = 1..54), the round-up threshold of a fraction (see jnum_seq):
// row q-1 is (10^q - 5^q) written with exactly q digits.
__constant__ const char kRoundThr[54][55] = {
    "5", "75", "875",
    "9375", "96875", "984375",
    "9921875", "99609375", "998046875",
    "9990234375", "99951171875", "999755859375",
    "9998779296875", "99993896484375", "999969482421875",
    "9999847412109375", "99999237060546875", "999996185302734375",
    "9999980926513671875", "99999904632568359375", "999999523162841796875",
    "9999997615814208984375", "99999988079071044921875", "999999940395355224609375",
    "9999999701976776123046875", "99999998509883880615234375", "999999992549419403076171875",
    "9999999962747097015380859375", "99999999813735485076904296875", "999999999068677425384521484375",
    "9999999995343387126922607421875", "99999999976716935634613037109375", "999999999883584678173065185546875",
    "9999999999417923390865325927734375", "99999999997089616954326629638671875", "999999999985448084771633148193359375",
    "9999999999927240423858165740966796875", "99999999999636202119290828704833984375", "999999999998181010596454143524169921875",
    "9999999999990905052982270717620849609375", "99999999999954525264911353588104248046875", "999999999999772626324556767940521240234375",
    "9999999999998863131622783839702606201171875", "99999999999994315658113919198513031005859375", "999999999999971578290569595992565155029296875",
    "9999999999999857891452847979962825775146484375", "99999999999999289457264239899814128875732421875", "999999999999996447286321199499070644378662109375",
    "9999999999999982236431605997495353221893310546875", "99999999999999911182158029987476766109466552734375", "999999999999999555910790149937383830547332763671875",
    "9999999999999997779553950749686919152736663818359375", "99999999999999988897769753748434595763683319091796875", "999999999999999944488848768742172978818416595458984375"};

// The u64 that extractSequence returns for the number token [s, e).  Integer tokens that fit
// (jsoncpp's threshold test) are exact.  Others are realValues d = RN(x), the correctly rounded
// double: isUInt64 / isInt64 take integral d in range, else static_cast<uint64_t>(d) as x86-64
// gcc compiles it (d >= 2^64, +inf included → 0; d < -2^63 → 0x8000000000000000; else
// truncation).  All of these depend on RN(x) only through V = |RN(x)| truncated, computed here
// with integer arithmetic over all the digits: the integer part I of |x| (≤ 20 digits, else
// |x| ≥ 2^64), rounded to 53 bits with the fraction as sticky when I ≥ 2^53; when I < 2^53, RN
// rounds up to I + 1 exactly when the fraction F ≥ 1 - 2^-q, q = 53 - floor(log2 I) (I = 0: q =
// 54), a tie going to I + 1 except for q = 1, where the even one of I, I + 1 wins.
// Returns false when decodeDouble fails ("'...' is not a number.").
__device__ bool jnum_seq(const uint8_t* p, uint32_t s, uint32_t e, uint64_t& out) {
    uint32_t i = s;
    const bool neg = p[i] == '-';
    if (neg) ++i;
    {  // decodeNumber
        const uint64_t maxv = neg ? (1ull << 63) : ~0ull, thr = maxv / 10, lastd = maxv % 10;
        uint64_t v = 0;
        bool dbl = false;
        for (uint32_t k = i; k < e; ++k) {
            const uint32_t ch = p[k];
            if (ch < '0' || ch > '9') {
                dbl = true;
                break;
            }
            const uint64_t dg = ch - '0';
            if (v >= thr && (v > thr || k + 1 != e || dg > lastd)) {
                dbl = true;
                break;
            }
            v = v * 10 + dg;
        }
        if (!dbl) {
            out = neg ? 0 - v : v;
            return true;
        }
    }
    // decodeDouble: the token must convert whole
    auto isd = [&](uint32_t k) { return k < e && p[k] >= '0' && p[k] <= '9'; };
    uint32_t k = i;
    const uint32_t i0 = k;
    while (isd(k)) ++k;
    const uint32_t nint = k - i0;
    uint32_t fs = k, nfrac = 0;
    if (k < e && p[k] == '.') {
        fs = ++k;
        while (isd(k)) ++k;
        nfrac = k - fs;
    }
    if (nint + nfrac == 0) return false;
    int64_t ex = 0;
    if (k < e && (p[k] == 'e' || p[k] == 'E')) {
        ++k;
        bool en = false;
        if (k < e && (p[k] == '+' || p[k] == '-')) en = p[k++] == '-';
        if (!isd(k)) return false;
        for (; isd(k); ++k)
            if (ex < 100000000) ex = ex * 10 + (p[k] - '0');
        if (en) ex = -ex;
    }
    if (k != e) return false;
    const uint32_t m = nint + nfrac;
    auto dig = [&](uint32_t j) -> uint32_t { return j < nint ? p[i0 + j] - '0' : p[fs + (j - nint)] - '0'; };
    uint32_t lz = 0;
    while (lz < m && dig(lz) == 0) ++lz;
    if (lz == m) {  // zero (also -0.0: isUInt64)
        out = 0;
        return true;
    }
    const int64_t ms = m - lz;
    auto d = [&](int64_t j) -> uint32_t { return (j >= 0 && j < ms) ? dig((uint32_t)(lz + j)) : 0u; };
    const int64_t pt = (int64_t)nint - lz + ex;  // significant digits before the decimal point
    bool huge = pt > 20;
    uint64_t I = 0;
    for (int64_t j = 0; !huge && j < pt; ++j) {
        const uint64_t dg = d(j);
        if (I > (~0ull - dg) / 10) huge = true;
        else I = I * 10 + dg;
    }
    uint64_t V = 0;
    if (!huge) {
        bool fnz = false;  // fraction non-zero
        for (int64_t j = pt > 0 ? pt : 0; j < ms && !fnz; ++j) fnz = d(j) != 0;
        if (I >> 53) {
            const int p2 = 63 - __builtin_clzll(I), sh = p2 - 52;
            uint64_t keep = I >> sh;
            const uint64_t rem = I & ((1ull << sh) - 1), half = 1ull << (sh - 1);
            keep += (rem > half || (rem == half && (fnz || (keep & 1)))) ? 1 : 0;
            if (keep >> 53 && sh == 11) huge = true;  // rounded to 2^64
            else V = keep << sh;
        } else if (!fnz) {
            V = I;
        } else {
            const int p2 = I ? 63 - __builtin_clzll(I) : -1, q = 53 - p2;
            int cmp = 0;
            for (int j = 0; j < q && cmp == 0; ++j) {
                const uint32_t a = d(pt + j), b = (uint32_t)(kRoundThr[q - 1][j] - '0');
                cmp = a > b ? 1 : (a < b ? -1 : 0);
            }
            if (cmp == 0) {  // F ≥ 1 - 2^-q; equal unless a later digit is non-zero
                for (int64_t j = pt + q > 0 ? pt + q : 0; j < ms && cmp == 0; ++j) cmp = d(j) != 0;
            }
            const bool up = cmp > 0 || (cmp == 0 && (q != 1 || (I & 1)));
            V = I + (up ? 1 : 0);
        }
    }
    if (!neg) out = huge ? 0 : V;
    else out = (huge || V >= (1ull << 63)) ? 0x8000000000000000ull : 0 - V;
    return true;
}

// --- the document ---------------------------------------------------------------------------
constexpr int kJsonStackLimit = 1000;  // CharReaderBuilder "stackLimit"
__device__ uint64_t json_seq_eval(const uint8_t* p, uint32_t n) {
    JCur c{p, n, 0};
    if (n >= 3 && p[0] == 0xEF && p[1] == 0xBB && p[2] == 0xBF) c.i = 3;  // skipBom
    uint64_t kind_bits[(kJsonStackLimit + 63) / 64];  // 1: object, 0: array, per open container
    int depth = 0, chain = 0;                         // chain: containers [0, chain) are root.message^k objects
    uint64_t res[4] = {0, 0, 0, 0};
    bool hobj[4] = {false, false, false, false}, root_obj = false;
    int pend_kind = 0, pend_level = 0;  // member whose value comes next: 1 _sequence_number, 2 message
    uint32_t s, e;
    int t;
    enum { S_VALUE, S_KEY, S_OAFTER, S_AFIRST, S_AAFTER } st = S_VALUE;
    auto is_obj = [&](int dd) { return (kind_bits[dd >> 6] >> (dd & 63)) & 1; };
    auto push = [&](bool obj) {
        const uint64_t b = 1ull << (depth & 63);
        kind_bits[depth >> 6] = obj ? (kind_bits[depth >> 6] | b) : (kind_bits[depth >> 6] & ~b);
        ++depth;
    };
    for (;;) {
        bool value_done = false;
        if (st == S_VALUE || st == S_AFIRST) {
            if (st == S_AFIRST) {  // readArray: ']' right after '[' or ',' (spaces only)
                c.skip_spaces();
                if (c.i < c.n && c.p[c.i] == ']') {
                    ++c.i;
                    --depth;
                    value_done = true;
                }
            }
            if (!value_done) {
                if (depth >= kJsonStackLimit) return 0;  // "Exceeded stackLimit in readValue()" (thrown)
                do t = jtoken(c, s, e);
                while (t == JT_COMMENT);
                const int kind = pend_kind, level = pend_level;
                pend_kind = 0;
                if (t == JT_OBEG) {
                    push(true);
                    if (depth == 1) {
                        root_obj = true;
                        chain = 1;
                    } else if (kind == 2 && depth - 1 == level + 1 && chain == level + 1) {
                        chain = depth;
                        hobj[level + 1] = true;
                    }
                    if (kind == 1) res[level] = 0;
                    st = S_KEY;
                    continue;
                }
                if (t == JT_ABEG) {
                    push(false);
                    if (kind == 1) res[level] = 0;
                    st = S_AFIRST;
                    continue;
                }
                if (t == JT_NUM) {
                    uint64_t v;
                    if (!jnum_seq(p, s, e, v)) return 0;
                    if (kind == 1) res[level] = v;
                } else if (t == JT_STR) {
                    if (kind == 1) {
                        StoullSink k;
                        if (!jdecode_string(p, s, e, k)) return 0;
                        res[level] = k.value();
                    } else {
                        NullSink k;
                        if (!jdecode_string(p, s, e, k)) return 0;
                    }
                } else if (t == JT_LIT) {
                    if (kind == 1) res[level] = 0;
                } else {
                    return 0;  // "Syntax error: value, object or array expected."
                }
                value_done = true;
            }
        } else if (st == S_KEY) {  // member name, or '}' (empty object / trailing comma)
            do t = jtoken(c, s, e);
            while (t == JT_COMMENT);
            if (t == JT_OEND) {
                if (depth == chain) chain = depth - 1;
                --depth;
                value_done = true;
            } else {
                if (t != JT_STR) return 0;
                KeySink k;
                if (!jdecode_string(p, s, e, k)) return 0;
                if (depth == chain && depth <= 4) {
                    const int level = depth - 1;
                    if (k.seq && k.len == 16) {
                        pend_kind = 1;
                        pend_level = level;
                    } else if (k.msg && k.len == 7 && level < 3) {
                        pend_kind = 2;
                        pend_level = level;
                        for (int j = level + 1; j < 4; ++j) {  // the member is replaced
                            res[j] = 0;
                            hobj[j] = false;
                        }
                    }
                }
                if (jtoken(c, s, e) != JT_COLON) return 0;  // "Missing ':' after object member name"
                st = S_VALUE;
                continue;
            }
        } else if (st == S_OAFTER) {  // ',' or '}'; after comments, the next token stands as separator
            t = jtoken(c, s, e);
            if (t != JT_OEND && t != JT_COMMA && t != JT_COMMENT) return 0;  // "Missing ',' or '}' ..."
            while (t == JT_COMMENT) t = jtoken(c, s, e);
            if (t == JT_OEND) {
                if (depth == chain) chain = depth - 1;
                --depth;
                value_done = true;
            } else {
                st = S_KEY;
                continue;
            }
        } else {  // S_AAFTER
            do t = jtoken(c, s, e);
            while (t == JT_COMMENT);
            if (t == JT_AEND) {
                --depth;
                value_done = true;
            } else {
                if (t != JT_COMMA) return 0;  // "Missing ',' or ']' in array declaration"
                st = S_AFIRST;
                continue;
            }
        }
        if (value_done) {
            if (depth == 0) break;  // the root is complete; what follows is ignored
            st = is_obj(depth - 1) ? S_OAFTER : S_AAFTER;
        }
    }
    if (!root_obj) return 0;  // isMember on a non-object root throws (null: false)
    if (res[0]) return res[0];
    for (int j = 1; j < 4 && hobj[j]; ++j)
        if (res[j]) return res[j];
    return 0;
}

#ifndef SEQNUM_HOST_CHECK  // tests/cpp/seqnum_host_check.cpp compiles the parser above for the host
// the decode kernel's call (parse mode with sbe_decoded.seq): kept out of line so the rare
// evaluation does not widen the decode kernel's register allocation
__device__ __noinline__ uint64_t json_seq_eval_call(const uint8_t* p, uint32_t n) { return json_seq_eval(p, n); }
// the serve kernel's own copy: a callee shared with that one-wave kernel would be compiled for its
// occupancy (more registers) and lower the decode kernels' occupancy with it
__device__ __noinline__ uint64_t json_seq_eval_call_serve(const uint8_t* p, uint32_t n) { return json_seq_eval(p, n); }

struct SeqArgs {
    const uint8_t* in;
    const uint64_t* rec_off;
    uint64_t n;
    const uint8_t* status;
    const uint8_t* flags;
    const uint32_t* view_off;
    const uint32_t* view_len;
    uint64_t* seq;
};

// Standalone launch (sbe_eval_sequence_numbers), for descriptors decoded without sbe_decoded.seq.
// One lane per flagged record.  A thread first tests the flags of 16 records with one 16-B load
// (the common batch has no candidate at all, so the launch is a 1-B/record flag read).
constexpr uint32_t kSeqCand = SBE_FL_SEQ_KEY | SBE_FL_SEQ_ESC;
__device__ __forceinline__ void seq_eval_one(const SeqArgs& a, uint64_t i) {
    if (a.status[i] != SBE_ST_TM || !(a.flags[i] & kSeqCand)) return;
    const uint8_t* pl = a.in + a.rec_off[i] + a.view_off[5 * i + 3];
    a.seq[i] = json_seq_eval(pl, a.view_len[5 * i + 3]);
}
__global__ __launch_bounds__(256) void sbe_seqnum_kernel(SeqArgs a) {
    const uint64_t groups = (a.n + 15) / 16;
    const bool vec = (reinterpret_cast<uintptr_t>(a.flags) & 15u) == 0;
    for (uint64_t g = (uint64_t)blockIdx.x * 256 + threadIdx.x; g < groups; g += (uint64_t)gridDim.x * 256) {
        const uint64_t i0 = 16 * g;
        if (vec && i0 + 16 <= a.n) {
            typedef uint32_t u32x4_t __attribute__((ext_vector_type(4)));
            const u32x4_t f = __builtin_nontemporal_load(reinterpret_cast<const u32x4_t*>(a.flags + i0));
            constexpr uint32_t m4 = kSeqCand * 0x01010101u;
            if (!((f.x | f.y | f.z | f.w) & m4)) continue;
        }
        const uint64_t i1 = i0 + 16 < a.n ? i0 + 16 : a.n;
        for (uint64_t i = i0; i < i1; ++i) seq_eval_one(a, i);
    }
}
#endif
