// kdtn_parse.h — device-side parsers for the strings of the reconcile path.
//
// One GPU thread parses one DICTIONARY entry (unique string), so every parse below
// runs once per distinct string per epoch, not once per link. Semantics restate:
//   ParseDuration          common/qdisc.go:146-158  over Go 1.18 time.ParseDuration
//   ParseFloatPercentage   common/qdisc.go:128-143  over strconv.ParseFloat(s, 32)
//   ParseRate              common/qdisc.go:162-199  (strings.ToLower/TrimSpace, ParseUint)
//   MakeVeth               common/veth.go:21-36     (net.ParseCIDR, net.ParseMAC)
//   Percentage2u32/time2Tick  vishvananda/netlink @ d40f9887b852 (go.mod:20)
// The float32 conversion is this file's own exact algorithm (double approximation +
// exact decimal comparison at rounding boundaries); it shares no code with the CPU
// oracle, which uses glibc strtof.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace kdtn {

#define KD_INLINE __device__ __forceinline__

KD_INLINE int lower_ascii(int c) { return (c >= 'A' && c <= 'Z') ? c + 32 : c; }
KD_INLINE bool is_digit(int c) { return c >= '0' && c <= '9'; }

// pow10 as doubles (exact for 0..22): a table lookup (every power up to 1e22 is exact)
static __constant__ double kPow10[23] = {1e0,  1e1,  1e2,  1e3,  1e4,  1e5,  1e6,  1e7,  1e8,  1e9,  1e10, 1e11,
                                         1e12, 1e13, 1e14, 1e15, 1e16, 1e17, 1e18, 1e19, 1e20, 1e21, 1e22};
KD_INLINE double pow10_exact(int e) { return kPow10[e]; }

// ------------------------------------------------------------------------------------
// time.ParseDuration + common.ParseDuration → microseconds. Returns false on error.
// ------------------------------------------------------------------------------------
KD_INLINE uint64_t duration_unit(const uint8_t* u, uint32_t n) {
    if (n == 1) {
        if (u[0] == 's') return 1000000000ull;
        if (u[0] == 'm') return 60000000000ull;
        if (u[0] == 'h') return 3600000000000ull;
        return 0;
    }
    if (n == 2 && u[1] == 's') {
        if (u[0] == 'n') return 1ull;
        if (u[0] == 'u') return 1000ull;
        if (u[0] == 'm') return 1000000ull;
        return 0;
    }
    if (n == 3 && u[2] == 's' &&
        ((u[0] == 0xC2 && u[1] == 0xB5) || (u[0] == 0xCE && u[1] == 0xBC)))  // µs, μs
        return 1000ull;
    return 0;
}

KD_INLINE bool parse_duration_us(const uint8_t* s, uint32_t n, uint32_t* out_us) {
    *out_us = 0;
    if (n == 0) return true;  // "" → 0, nil
    const uint64_t TOP = 1ull << 63;
    uint32_t i = 0;
    bool neg = false;
    if (s[0] == '-' || s[0] == '+') { neg = s[0] == '-'; i = 1; }
    if (n - i == 1 && s[i] == '0') return true;
    if (i == n) return false;
    uint64_t d = 0;
    while (i < n) {
        int c = s[i];
        if (!(c == '.' || is_digit(c))) return false;
        uint64_t v = 0;
        uint32_t st = i;
        for (; i < n && is_digit(s[i]); ++i) {
            if (v > TOP / 10) return false;
            v = v * 10 + (uint64_t)(s[i] - '0');
            if (v > TOP) return false;
        }
        bool pre = i != st, post = false;
        uint64_t f = 0;
        double scale = 1.0;
        if (i < n && s[i] == '.') {
            ++i;
            uint32_t st2 = i;
            bool ovf = false;
            for (; i < n && is_digit(s[i]); ++i) {
                if (ovf) continue;
                if (f > (TOP - 1) / 10) { ovf = true; continue; }
                uint64_t y = f * 10 + (uint64_t)(s[i] - '0');
                if (y > TOP) { ovf = true; continue; }
                f = y;
                scale = __dmul_rn(scale, 10.0);
            }
            post = i != st2;
        }
        if (!pre && !post) return false;
        uint32_t us = i;
        while (i < n && !(s[i] == '.' || is_digit(s[i]))) ++i;
        if (i == us) return false;
        uint64_t unit = duration_unit(s + us, i - us);
        if (unit == 0) return false;
        if (v > TOP / unit) return false;
        v *= unit;
        if (f > 0) {
            double fr = __dmul_rn((double)f, __ddiv_rn((double)unit, scale));
            v += (uint64_t)fr;
            if (v > TOP) return false;
        }
        d += v;
        if (d > TOP) return false;
    }
    int64_t dur;
    if (neg) dur = (int64_t)(0ull - d);
    else {
        if (d > TOP - 1) return false;
        dur = (int64_t)d;
    }
    if (dur < 0) return false;                 // "duration value must be positive"
    *out_us = (uint32_t)(dur / 1000);          // uint32(value.Microseconds())
    return true;
}


// ------------------------------------------------------------------------------------
// strconv.ParseFloat(s, 32) restricted to what ParseFloatPercentage can accept.
// ------------------------------------------------------------------------------------
// Exact decimal digits of a dyadic double M > 0 compared against the decimal number
// V = 0.<digits of s> × 10^dpv. Returns -1/0/+1 for V <, ==, > M.
// Digit source: bytes of s in [beg, end) skipping anything that is not a digit;
// the first emitted digit is the first NON-ZERO digit.
KD_INLINE int cmp_decimal_vs_dyadic(const uint8_t* s, uint32_t beg, uint32_t end, long dpv,
                                     double M) {
    // M = mi × 2^qe with mi odd-or-not 53-bit integer
    int ex;
    double fr = frexp(M, &ex);                // M = fr × 2^ex, fr in [0.5,1)
    uint64_t mi = (uint64_t)ldexp(fr, 53);    // exact
    int qe = ex - 53;
    while ((mi & 1ull) == 0ull) { mi >>= 1; ++qe; }
    // Big number B in base 1e9 limbs, little-endian: M = B × 10^-k
    uint32_t limb[24];
    int nl = 0;
    int k = 0;
    {
        uint64_t x = mi;
        while (x) { limb[nl++] = (uint32_t)(x % 1000000000ull); x /= 1000000000ull; }
    }
    if (qe >= 0) {
        for (int r = 0; r < qe; ++r) {          // multiply by 2 (qe small here: M < 2^64)
            uint64_t carry = 0;
            for (int q = 0; q < nl; ++q) {
                uint64_t t = (uint64_t)limb[q] * 2ull + carry;
                limb[q] = (uint32_t)(t % 1000000000ull);
                carry = t / 1000000000ull;
            }
            if (carry) limb[nl++] = (uint32_t)carry;
        }
    } else {
        k = -qe;                                // M = mi × 5^k / 10^k
        int rem = k;
        while (rem > 0) {
            int step = rem > 12 ? 12 : rem;
            uint64_t mul = 1;
            for (int q = 0; q < step; ++q) mul *= 5ull;
            uint64_t carry = 0;
            for (int q = 0; q < nl; ++q) {
                uint64_t t = (uint64_t)limb[q] * mul + carry;
                limb[q] = (uint32_t)(t % 1000000000ull);
                carry = t / 1000000000ull;
            }
            while (carry) { limb[nl++] = (uint32_t)(carry % 1000000000ull); carry /= 1000000000ull; }
            rem -= step;
        }
    }
    // number of decimal digits of B
    int top_digits = 1;
    {
        uint32_t t = limb[nl - 1];
        while (t >= 10) { t /= 10; ++top_digits; }
    }
    long L = (long)(nl - 1) * 9 + top_digits;
    long dpm = L - k;                            // M = 0.b1..bL × 10^dpm
    if (dpv != dpm) return dpv > dpm ? 1 : -1;
    // walk digits of B most-significant first and digits of V
    uint32_t pos = beg;
    auto next_v = [&](int* dig) -> bool {        // next significant digit of V
        while (pos < end) {
            int c = s[pos++];
            if (is_digit(c)) { *dig = c - '0'; return true; }
        }
        return false;
    };
    // skip leading zeros of V
    {
        // find first non-zero digit
        while (pos < end) {
            int c = s[pos];
            if (is_digit(c) && c != '0') break;
            ++pos;
        }
    }
    for (int q = nl - 1; q >= 0; --q) {
        uint32_t t = limb[q];
        int nd = (q == nl - 1) ? top_digits : 9;
        uint32_t div = 1;
        for (int z = 1; z < nd; ++z) div *= 10;
        for (int z = 0; z < nd; ++z) {
            int bd = (int)(t / div);
            t -= (uint32_t)bd * div;
            div /= 10;
            int vd;
            if (!next_v(&vd)) return -1;         // V ran out of digits: V < M (B has more)
            if (vd != bd) return vd > bd ? 1 : -1;
        }
    }
    int vd;
    while (next_v(&vd))
        if (vd != 0) return 1;
    return 0;
}

// The value of a syntactically valid float string from its readFloat state (mantissa,
// significant digits, decimal point, digit range for the exact compare): the rounding to
// float32 and the percentage range check.
KD_INLINE bool pct_finish(const uint8_t* s, bool neg, bool hex, bool trunc, uint64_t mant, int ndmant, long dp,
                          uint32_t dig_beg, uint32_t dig_end, float* out) {
    if (mant == 0) { *out = 0.0f; return true; }   // ±0 → 0 (−0 is not < 0)

    // Only |V| <= 100 matters. Values below 1e-30 (float32 normal range starts at
    // ~1.18e-38) need just one fact: whether they round to zero, i.e. |V| <= 2^-150
    // (the tie at exactly 2^-150 goes to the even value 0). Positive tiny values are
    // accepted either way and Percentage2u32 maps them to 0; negative ones are an
    // error unless they round to -0. This keeps all float32 arithmetic normal.
    float v;
    const double TWO_M150 = 7.006492321624085354618647916449580656401309709382578858785341e-46;
    if (hex) {
        // value = mant × 2^(dp - 4*ndmant), plus a sticky bit when digits were cut
        long e2 = dp - 4L * ndmant;
        int lz = __clzll(mant);
        uint64_t m = mant << lz;                 // top bit at 63
        long E = e2 + 63 - lz;                   // value in [2^E, 2^(E+1))
        if (E >= 7) return false;                // >= 128: > 100 or < 0
        if (E < -100) {
            if (!neg) { *out = 0.0f; return true; }
            bool nonzero = E > -150 || (E == -150 && ((m << 1) != 0 || trunc));
            if (nonzero) return false;
            *out = 0.0f;
            return true;
        }
        uint64_t kept = m >> 40;                 // 24 significant bits
        uint64_t rest = m << 24;
        bool half = (rest >> 63) & 1ull;
        bool low = ((rest << 1) != 0) || trunc;
        if (half && (low || (kept & 1ull))) ++kept;
        v = (float)ldexp((double)kept, (int)(E - 23));   // exact
    } else {
        // decimal: V = 0.<digits> × 10^dp
        if (dp >= 4) return false;               // |V| >= 100.0 × 10: > 100 or < 0
        if (dp <= -46) { *out = 0.0f; return true; }  // |V| < 1e-46 < 2^-150 → ±0
        int e10 = (int)(dp - ndmant);            // V ≈ mant × 10^e10
        if (e10 >= -8 && e10 <= 0 && !trunc && mant < (1ull << 53)) {
            // V = mant / 10^k with k <= 8: the quotient rounded once to double, then to float32,
            // is V correctly rounded. Were it not, the double would have to lie on a float32
            // midpoint m = M / 2^e (M < 2^25) while V does not: then |V - m| >= 1 / (10^k 2^e)
            // >= V / (10^k 2^25) > V 2^-53 (10^8 < 2^28), beyond the division's rounding
            // error; and a V that is a midpoint is exact in double and rounds to even. (k = 0:
            // V = mant, exact.)
            v = (float)(e10 == 0 ? (double)mant : __ddiv_rn((double)mant, pow10_exact(-e10)));
            if (neg) v = -v;
            if (v < 0.0f || v > 100.0f) return false;
            *out = v;
            return true;
        }
        double approx = (double)mant;
        if (e10 >= 0) approx = __dmul_rn(approx, pow10_exact(e10));
        else if (e10 >= -22) approx = __ddiv_rn(approx, pow10_exact(-e10));
        else {
            approx = __ddiv_rn(approx, 1e22);
            int r = -e10 - 22;
            while (r > 22) { approx = __ddiv_rn(approx, 1e22); r -= 22; }
            approx = __ddiv_rn(approx, pow10_exact(r));
        }
        if (approx < 1e-30) {
            if (!neg) { *out = 0.0f; return true; }
            int r = cmp_decimal_vs_dyadic(s, dig_beg, dig_end, dp, TWO_M150);
            if (r > 0) return false;
            *out = 0.0f;
            return true;
        }
        float c = (float)approx;
        float cd = nextafterf(c, 0.0f);
        float cu = nextafterf(c, 3.4e38f);
        double mlo = ((double)cd + (double)c) * 0.5;
        double mhi = ((double)c + (double)cu) * 0.5;
        double tol = approx * 1e-13;
        v = c;
        if (fabs(approx - mhi) <= tol) {
            int r = cmp_decimal_vs_dyadic(s, dig_beg, dig_end, dp, mhi);
            if (r > 0) v = cu;
            else if (r == 0) v = (__float_as_uint(c) & 1u) ? cu : c;
        } else if (fabs(approx - mlo) <= tol) {
            int r = cmp_decimal_vs_dyadic(s, dig_beg, dig_end, dp, mlo);
            if (r < 0) v = cd;
            else if (r == 0) v = (__float_as_uint(c) & 1u) ? cd : c;
        }
    }
    if (neg) v = -v;
    if (v < 0.0f || v > 100.0f) return false;
    *out = v;
    return true;
}

KD_INLINE bool parse_pct_generic(const uint8_t* s, uint32_t n, float* out) {
    *out = 0.0f;
    if (n == 0) return true;
    // special(): inf/infinity/nan forms are all errors for a percentage (NaN → error,
    // ±Inf → out of range, anything with trailing junk → syntax error).
    {
        int c0 = s[0];
        int c1 = n > 1 ? lower_ascii(s[1]) : 0;
        if (c0 == 'i' || c0 == 'I' || c0 == 'n' || c0 == 'N') return false;
        if ((c0 == '+' || c0 == '-') && (c1 == 'i')) return false;
    }
    // readFloat
    uint32_t i = 0;
    bool neg = false, hex = false, underscores = false, sawdot = false, sawdigits = false;
    long nd = 0, dp = 0;
    uint64_t mant = 0;
    int ndmant = 0;
    bool trunc = false;
    uint32_t dig_beg = 0;  // byte index where mantissa digits begin (for exact compare)
    if (s[i] == '+' || s[i] == '-') { neg = s[i] == '-'; ++i; }
    if (i + 2 < n && s[i] == '0' && lower_ascii(s[i + 1]) == 'x') { hex = true; i += 2; }
    const int maxmant = hex ? 16 : 19;
    dig_beg = i;
    for (; i < n; ++i) {
        int c = s[i];
        if (c == '_') { underscores = true; continue; }
        if (c == '.') {
            if (sawdot) break;
            sawdot = true;
            dp = nd;
            continue;
        }
        int dv = -1;
        if (is_digit(c)) dv = c - '0';
        else if (hex && lower_ascii(c) >= 'a' && lower_ascii(c) <= 'f') dv = lower_ascii(c) - 'a' + 10;
        if (dv < 0) break;
        sawdigits = true;
        if (dv == 0 && nd == 0 && is_digit(c)) { --dp; continue; }
        ++nd;
        if (ndmant < maxmant) {
            mant = mant * (hex ? 16ull : 10ull) + (uint64_t)dv;
            ++ndmant;
        } else if (dv != 0) {
            trunc = true;
        }
    }
    uint32_t dig_end = i;
    if (!sawdigits) return false;
    if (!sawdot) dp = nd;
    if (hex) { dp *= 4; }
    const int expc = hex ? 'p' : 'e';
    if (i < n && lower_ascii(s[i]) == expc) {
        ++i;
        if (i >= n) return false;
        long esign = 1;
        if (s[i] == '+') ++i;
        else if (s[i] == '-') { ++i; esign = -1; }
        if (i >= n || !is_digit(s[i])) return false;
        long e = 0;
        for (; i < n && (is_digit(s[i]) || s[i] == '_'); ++i) {
            if (s[i] == '_') { underscores = true; continue; }
            if (e < 10000) e = e * 10 + (s[i] - '0');
        }
        dp += e * esign;
    } else if (hex) {
        return false;  // hexadecimal mantissa requires a 'p' exponent
    }
    if (underscores) {
        // underscoreOK over s[:i]
        uint32_t q = 0;
        int saw = '^';
        if (q < i && (s[q] == '+' || s[q] == '-')) ++q;
        bool hx = false;
        if (i - q >= 2 && s[q] == '0') {
            int l1 = lower_ascii(s[q + 1]);
            if (l1 == 'b' || l1 == 'o' || l1 == 'x') { q += 2; saw = '0'; hx = l1 == 'x'; }
        }
        for (; q < i; ++q) {
            int c = s[q];
            if (is_digit(c) || (hx && lower_ascii(c) >= 'a' && lower_ascii(c) <= 'f')) { saw = '0'; continue; }
            if (c == '_') {
                if (saw != '0') return false;
                saw = '_';
                continue;
            }
            if (saw == '_') return false;
            saw = '!';
        }
        if (saw == '_') return false;
    }
    if (i != n) return false;
    return pct_finish(s, neg, hex, trunc, mant, ndmant, dp, dig_beg, dig_end, out);
}

// ParseFloatPercentage of a plain decimal of at most 16 bytes (digits and at most one '.',
// starting with a digit or '.'): its bytes are loaded at once and scanned by a fully
// unrolled, predicated readFloat (no sign, base prefix, underscore or exponent can occur, and
// 16 digits never reach the 19-digit mantissa limit); anything else takes the generic parser.
KD_INLINE bool parse_pct(const uint8_t* s, uint32_t n, float* out) {
    if (n == 0 || n > 16) return parse_pct_generic(s, n, out);
    // the 16 bytes from five dword loads (the arena and the LDS slices have slack past a string)
    const uint32_t mis = (uint32_t)(reinterpret_cast<uintptr_t>(s) & 3u);
    const uint32_t* p = reinterpret_cast<const uint32_t*>(s - mis);
    const uint32_t d0 = p[0], d1 = p[1], d2 = p[2], d3 = p[3], d4 = p[4];
    const uint32_t w[4] = {__builtin_amdgcn_alignbyte(d1, d0, mis), __builtin_amdgcn_alignbyte(d2, d1, mis),
                           __builtin_amdgcn_alignbyte(d3, d2, mis), __builtin_amdgcn_alignbyte(d4, d3, mis)};
    bool ok = true, sawdot = false, sawdigits = false;
    long nd = 0, dp = 0;
    uint64_t mant = 0;
    int ndmant = 0;
#pragma unroll
    for (int k = 0; k < 16; ++k) {
        if (__ballot((uint32_t)k < n) == 0) break;      // no lane of the wave has byte k
        if ((uint32_t)k < n) {
            const uint32_t ch = (w[k >> 2] >> (8 * (k & 3))) & 0xFFu;
            const bool dig = ch - '0' <= 9u;
            if (ch == '.') {
                ok &= !sawdot;
                sawdot = true;
                dp = nd;
            } else if (dig) {
                sawdigits = true;
                if (ch == '0' && nd == 0) {
                    --dp;
                } else {
                    ++nd;
                    mant = mant * 10u + (ch - '0');
                    ++ndmant;
                }
            } else {
                ok = false;
            }
        }
    }
    if (!ok || !sawdigits) return parse_pct_generic(s, n, out);
    if (!sawdot) dp = nd;
    return pct_finish(s, false, false, false, mant, ndmant, dp, 0u, n, out);
}

// netlink Percentage2u32: float32 arithmetic, amd64 float→uint32 (via int64, truncate).
KD_INLINE uint32_t p2u(float p) {
    if (p == 100.0f) return 0xFFFFFFFFu;
    float q = __fdiv_rn(p, 100.0f);
    float r = __fmul_rn(4294967296.0f, q);
    return (uint32_t)(int64_t)r;
}

// netlink time2Tick: uint32(float64(t) * tickInUsec)
KD_INLINE uint32_t time2tick(uint32_t t, double tick) {
    return (uint32_t)(int64_t)__dmul_rn((double)t, tick);
}

// ------------------------------------------------------------------------------------
// ParseRate: strings.TrimSpace(strings.ToLower(rate)), suffixes, strconv.ParseUint.
// ------------------------------------------------------------------------------------
KD_INLINE uint32_t utf8_rune(const uint8_t* s, uint32_t n, uint32_t* w) {
    uint32_t c0 = s[0];
    if (c0 < 0x80) { *w = 1; return c0; }
    if (c0 >= 0xC2 && c0 <= 0xDF) {
        if (n >= 2 && (s[1] & 0xC0) == 0x80) { *w = 2; return ((c0 & 0x1F) << 6) | (s[1] & 0x3F); }
    } else if (c0 >= 0xE0 && c0 <= 0xEF) {
        uint32_t lo = c0 == 0xE0 ? 0xA0 : 0x80, hi = c0 == 0xED ? 0x9F : 0xBF;
        if (n >= 3 && s[1] >= lo && s[1] <= hi && (s[2] & 0xC0) == 0x80) {
            *w = 3;
            return ((c0 & 0x0F) << 12) | ((uint32_t)(s[1] & 0x3F) << 6) | (s[2] & 0x3F);
        }
    } else if (c0 >= 0xF0 && c0 <= 0xF4) {
        uint32_t lo = c0 == 0xF0 ? 0x90 : 0x80, hi = c0 == 0xF4 ? 0x8F : 0xBF;
        if (n >= 4 && s[1] >= lo && s[1] <= hi && (s[2] & 0xC0) == 0x80 && (s[3] & 0xC0) == 0x80) {
            *w = 4;
            return ((c0 & 0x07) << 18) | ((uint32_t)(s[1] & 0x3F) << 12) |
                   ((uint32_t)(s[2] & 0x3F) << 6) | (s[3] & 0x3F);
        }
    }
    *w = 1;
    return 0xFFFDu;
}

KD_INLINE bool unicode_space(uint32_t r) {
    return r == '\t' || r == '\n' || r == '\v' || r == '\f' || r == '\r' || r == ' ' ||
           r == 0x85 || r == 0xA0 || r == 0x1680 || (r >= 0x2000 && r <= 0x200A) ||
           r == 0x2028 || r == 0x2029 || r == 0x202F || r == 0x205F || r == 0x3000;
}

// lower-cased rune as one "ASCII-ish" char; non-ASCII runes other than U+0130/U+212A
// (whose unicode.ToLower is ASCII 'i'/'k') map to 0x80, which no later step accepts.
KD_INLINE int rate_char(uint32_t r) {
    if (r < 0x80) return lower_ascii((int)r);
    if (r == 0x130) return 'i';
    if (r == 0x212A) return 'k';
    return 0x80;
}

KD_INLINE bool parse_rate_generic(const uint8_t* s, uint32_t n, uint64_t* out) {
    *out = 0;
    // pass 1: trimmed rune range and the last 5 mapped chars
    uint32_t a = 0;
    {
        while (a < n) {
            uint32_t w;
            uint32_t r = utf8_rune(s + a, n - a, &w);
            if (!unicode_space(r)) break;
            a += w;
        }
    }
    uint32_t b = a, m = 0;
    int tail[5] = {0, 0, 0, 0, 0};  // tail[0] = last char
    {
        uint32_t p = a;
        uint32_t cnt = 0;
        int ring[5] = {0, 0, 0, 0, 0};
        uint32_t last_end = a, count_at_last = 0;
        int ring_at_last[5] = {0, 0, 0, 0, 0};
        while (p < n) {
            uint32_t w;
            uint32_t r = utf8_rune(s + p, n - p, &w);
            p += w;
            for (int q = 4; q > 0; --q) ring[q] = ring[q - 1];
            ring[0] = rate_char(r);
            ++cnt;
            if (!unicode_space(r)) {
                last_end = p;
                count_at_last = cnt;
                for (int q = 0; q < 5; ++q) ring_at_last[q] = ring[q];
            }
        }
        b = last_end;
        m = count_at_last;
        for (int q = 0; q < 5; ++q) tail[q] = ring_at_last[q];
    }
    if (m == 0) return true;  // "" after trim → 0, nil
    uint32_t strip = 0;
    uint64_t mult = 1;
    auto tc = [&](uint32_t k) -> int { return (k < 5 && k < m) ? tail[k] : -1; };  // k-th from end
    if (m >= 3 && tc(2) == 'b' && tc(1) == 'i' && tc(0) == 't') strip = 3;
    else if (m >= 3 && tc(2) == 'b' && tc(1) == 'p' && tc(0) == 's') { strip = 3; mult = 8; }
    uint64_t base = 1000;
    if (m - strip >= 1 && tc(strip) == 'i') { ++strip; base = 1024; }
    if (m - strip >= 1) {
        int u = tc(strip);
        int idx = u == 'k' ? 0 : u == 'm' ? 1 : u == 'g' ? 2 : u == 't' ? 3 : -1;
        if (idx >= 0) {
            ++strip;
            for (int j = 0; j <= idx; ++j) mult *= base;
        }
    }
    uint32_t keep = m - strip;
    if (keep == 0) return false;  // ParseUint("") → syntax error
    // pass 2: ParseUint over the first `keep` mapped chars
    uint64_t v = 0;
    const uint64_t cutoff = 0xFFFFFFFFFFFFFFFFull / 10 + 1;
    uint32_t p = a;
    for (uint32_t k = 0; k < keep; ++k) {
        uint32_t w;
        uint32_t r = utf8_rune(s + p, b - p, &w);
        p += w;
        int c = rate_char(r);
        if (!is_digit(c)) return false;
        if (v >= cutoff) return false;
        v *= 10;
        uint64_t v1 = v + (uint64_t)(c - '0');
        if (v1 < v) return false;
        v = v1;
    }
    *out = v * mult;
    return true;
}

// ParseRate of a string of printable ASCII without spaces (every synthetic and nearly every
// real rate string): TrimSpace is the identity, each byte is one rune and ToLower is ASCII,
// so the suffix test reads the last bytes and ParseUint the first ones directly — the same
// result as parse_rate_generic without its rune decoding and ring buffer per character.
KD_INLINE bool parse_rate(const uint8_t* s, uint32_t n, uint64_t* out) {
    bool simple = n > 0;
    for (uint32_t i = 0; i < n; ++i) simple &= s[i] >= 0x21 && s[i] <= 0x7E;
    if (!simple) return parse_rate_generic(s, n, out);
    *out = 0;
    auto tc = [&](uint32_t k) -> int { return k < n ? lower_ascii(s[n - 1 - k]) : -1; };   // k-th from end
    uint32_t strip = 0;
    uint64_t mult = 1;
    if (n >= 3 && tc(2) == 'b' && tc(1) == 'i' && tc(0) == 't') strip = 3;
    else if (n >= 3 && tc(2) == 'b' && tc(1) == 'p' && tc(0) == 's') { strip = 3; mult = 8; }
    uint64_t base = 1000;
    if (n - strip >= 1 && tc(strip) == 'i') { ++strip; base = 1024; }
    if (n - strip >= 1) {
        const int u = tc(strip);
        const int idx = u == 'k' ? 0 : u == 'm' ? 1 : u == 'g' ? 2 : u == 't' ? 3 : -1;
        if (idx >= 0) {
            ++strip;
            for (int j = 0; j <= idx; ++j) mult *= base;
        }
    }
    const uint32_t keep = n - strip;
    if (keep == 0) return false;                    // ParseUint("") → syntax error
    uint64_t v = 0;
    const uint64_t cutoff = 0xFFFFFFFFFFFFFFFFull / 10 + 1;
    for (uint32_t k = 0; k < keep; ++k) {
        const int c = s[k];
        if (!is_digit(c)) return false;
        if (v >= cutoff) return false;
        v *= 10;
        const uint64_t v1 = v + (uint64_t)(c - '0');
        if (v1 < v) return false;
        v = v1;
    }
    *out = v * mult;
    return true;
}

// ------------------------------------------------------------------------------------
// net.ParseCIDR / net.ParseMAC (validity only; MakeVeth aborts on error)
// ------------------------------------------------------------------------------------
#define KD_BIG 0xFFFFFF
KD_INLINE bool dec_int(const uint8_t* s, uint32_t n, long* v, uint32_t* used) {  // dtoi
    long x = 0;
    uint32_t i = 0;
    for (; i < n && is_digit(s[i]); ++i) {
        x = x * 10 + (s[i] - '0');
        if (x >= KD_BIG) { *v = KD_BIG; *used = i; return false; }
    }
    *v = x;
    *used = i;
    return i != 0;
}
KD_INLINE int hexval(int c) {
    if (is_digit(c)) return c - '0';
    if (c >= 'a' && c <= 'f') return c - 'a' + 10;
    if (c >= 'A' && c <= 'F') return c - 'A' + 10;
    return -1;
}
KD_INLINE bool hex_int(const uint8_t* s, uint32_t n, long* v, uint32_t* used) {  // xtoi
    long x = 0;
    uint32_t i = 0;
    for (; i < n; ++i) {
        int h = hexval(s[i]);
        if (h < 0) break;
        x = x * 16 + h;
        if (x >= KD_BIG) { *v = 0; *used = i; return false; }
    }
    *v = x;
    *used = i;
    return i != 0;
}
KD_INLINE bool ipv4_ok(const uint8_t* s, uint32_t n) {
    uint32_t p = 0;
    for (int k = 0; k < 4; ++k) {
        if (p >= n) return false;
        if (k > 0) {
            if (s[p] != '.') return false;
            ++p;
        }
        long v;
        uint32_t c;
        if (!dec_int(s + p, n - p, &v, &c) || v > 0xFF) return false;
        if (c > 1 && s[p] == '0') return false;
        p += c;
    }
    return p == n;
}
KD_INLINE bool ipv6_ok(const uint8_t* s, uint32_t n) {
    int ell = -1;
    uint32_t p = 0;
    if (n >= 2 && s[0] == ':' && s[1] == ':') {
        ell = 0;
        p = 2;
        if (p == n) return true;
    }
    int i = 0;
    while (i < 16) {
        long v;
        uint32_t c;
        if (!hex_int(s + p, n - p, &v, &c) || v > 0xFFFF) return false;
        if (p + c < n && s[p + c] == '.') {
            if (ell < 0 && i != 12) return false;
            if (i + 4 > 16) return false;
            if (!ipv4_ok(s + p, n - p)) return false;
            p = n;
            i += 4;
            break;
        }
        i += 2;
        p += c;
        if (p == n) break;
        if (s[p] != ':' || p + 1 == n) return false;
        ++p;
        if (s[p] == ':') {
            if (ell >= 0) return false;
            ell = i;
            ++p;
            if (p == n) break;
        }
    }
    if (p != n) return false;
    if (i < 16) return ell >= 0;
    return ell < 0;
}
KD_INLINE bool cidr_ok(const uint8_t* s, uint32_t n) {
    uint32_t sl = 0;
    while (sl < n && s[sl] != '/') ++sl;
    if (sl == n) return false;
    int bits_max = 32;
    bool ok = ipv4_ok(s, sl);
    if (!ok) { bits_max = 128; ok = ipv6_ok(s, sl); }
    long bits;
    uint32_t used;
    bool dok = dec_int(s + sl + 1, n - sl - 1, &bits, &used);
    return ok && dok && used == n - sl - 1 && bits >= 0 && bits <= bits_max;
}
KD_INLINE bool mac_pair(const uint8_t* s, uint32_t n, int sep) {  // xtoi2
    if (n > 2 && s[2] != sep) return false;
    return n >= 2 && hexval(s[0]) >= 0 && hexval(s[1]) >= 0;
}
KD_INLINE bool mac_ok(const uint8_t* s, uint32_t n) {
    if (n < 14) return false;
    if (s[2] == ':' || s[2] == '-') {
        if ((n + 1) % 3 != 0) return false;
        uint32_t cnt = (n + 1) / 3;
        if (cnt != 6 && cnt != 8 && cnt != 20) return false;
        for (uint32_t x = 0, i = 0; i < cnt; ++i, x += 3)
            if (!mac_pair(s + x, n - x, s[2])) return false;
        return true;
    }
    if (s[4] == '.') {
        if ((n + 1) % 5 != 0) return false;
        uint32_t cnt = 2 * (n + 1) / 5;
        if (cnt != 6 && cnt != 8 && cnt != 20) return false;
        for (uint32_t x = 0, i = 0; i < cnt; i += 2, x += 5) {
            if (!mac_pair(s + x, 2, 0)) return false;
            if (!mac_pair(s + x + 2, n - x - 2, s[4])) return false;
        }
        return true;
    }
    return false;
}

}  // namespace kdtn
