/*
 * kdtn_oracle.c — TEST INFRASTRUCTURE ONLY: CPU restatement of the reference
 * kube-dtn reconcile hot path, used as the parity checker for libkdtn.so and as
 * bench.py's cpu_baseline ("port"). Never linked into, or called by, the product.
 *
 * Every function cites the reference file:line (relative to the reference root) or
 * the third-party algorithm it restates. Build: oracle/Makefile (gcc -O2
 * -ffp-contract=off; SSE float math, so float32/float64 ops round like Go/amd64).
 */
#define _GNU_SOURCE
#include "kdtn_oracle.h"

#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

typedef struct { const char* p; uint32_t n; } ostr;

static ostr tab_get(const kdtn_strtab* t, uint32_t id) {
    ostr s;
    s.p = (const char*)t->bytes + t->offs[id];
    s.n = t->offs[id + 1] - t->offs[id];
    return s;
}
static int ostr_eq(ostr a, ostr b) { return a.n == b.n && (a.n == 0 || memcmp(a.p, b.p, a.n) == 0); }
static int ostr_is(ostr a, const char* lit) { return ostr_eq(a, (ostr){lit, (uint32_t)strlen(lit)}); }

/* ======================================================================================
 * time.ParseDuration (Go 1.18 time/format.go) + common.ParseDuration (common/qdisc.go:146-158)
 * ==================================================================================== */
static uint64_t go_unit(const char* u, size_t n) {
    if (n == 2 && u[0] == 'n' && u[1] == 's') return 1ull;
    if (n == 2 && u[0] == 'u' && u[1] == 's') return 1000ull;
    if (n == 3 && (unsigned char)u[0] == 0xC2 && (unsigned char)u[1] == 0xB5 && u[2] == 's') return 1000ull; /* µs U+00B5 */
    if (n == 3 && (unsigned char)u[0] == 0xCE && (unsigned char)u[1] == 0xBC && u[2] == 's') return 1000ull; /* μs U+03BC */
    if (n == 2 && u[0] == 'm' && u[1] == 's') return 1000000ull;
    if (n == 1 && u[0] == 's') return 1000000000ull;
    if (n == 1 && u[0] == 'm') return 60000000000ull;
    if (n == 1 && u[0] == 'h') return 3600000000000ull;
    return 0;
}

/* Returns 0 and the Duration (ns) or -1 on the Go error paths. */
static int go_parse_duration(const char* s, size_t n, int64_t* out) {
    const uint64_t TOP = 1ull << 63;
    size_t i = 0;
    uint64_t d = 0;
    int neg = 0;
    if (n > 0 && (s[0] == '-' || s[0] == '+')) { neg = s[0] == '-'; i = 1; }
    if (n - i == 1 && s[i] == '0') { *out = 0; return 0; }   /* special case "0" */
    if (i == n) return -1;
    while (i < n) {
        uint64_t v = 0, f = 0;
        double scale = 1.0;
        char c = s[i];
        if (!(c == '.' || (c >= '0' && c <= '9'))) return -1;
        size_t st = i;                                        /* leadingInt */
        for (; i < n && s[i] >= '0' && s[i] <= '9'; i++) {
            if (v > TOP / 10) return -1;
            v = v * 10 + (uint64_t)(s[i] - '0');
            if (v > TOP) return -1;
        }
        int pre = i != st, post = 0;
        if (i < n && s[i] == '.') {                           /* leadingFraction */
            i++;
            size_t st2 = i;
            int overflow = 0;
            for (; i < n && s[i] >= '0' && s[i] <= '9'; i++) {
                if (overflow) continue;
                if (f > (TOP - 1) / 10) { overflow = 1; continue; }
                uint64_t y = f * 10 + (uint64_t)(s[i] - '0');
                if (y > TOP) { overflow = 1; continue; }
                f = y;
                scale *= 10.0;
            }
            post = i != st2;
        }
        if (!pre && !post) return -1;
        size_t us = i;                                        /* unit: run of [^0-9.] */
        for (; i < n; i++) {
            c = s[i];
            if (c == '.' || (c >= '0' && c <= '9')) break;
        }
        if (i == us) return -1;
        uint64_t unit = go_unit(s + us, i - us);
        if (!unit) return -1;
        if (v > TOP / unit) return -1;
        v *= unit;
        if (f > 0) {
            v += (uint64_t)((double)f * ((double)unit / scale));
            if (v > TOP) return -1;
        }
        d += v;
        if (d > TOP) return -1;
    }
    if (neg) { *out = (int64_t)(0ull - d); return 0; }
    if (d > TOP - 1) return -1;
    *out = (int64_t)d;
    return 0;
}

int or_parse_duration(const char* s, uint32_t n, uint32_t* us) {
    *us = 0;
    if (n == 0) return 0;                                     /* qdisc.go:147-149 */
    int64_t d;
    if (go_parse_duration(s, n, &d)) return 1;                /* :150-153 */
    if (d < 0) return 1;                                      /* :154-156 */
    *us = (uint32_t)(d / 1000);                               /* :157 uint32(Microseconds()) */
    return 0;
}

/* ======================================================================================
 * strconv.ParseFloat(s, 32) (Go 1.18 strconv/atof.go): grammar restated (special,
 * readFloat, underscoreOK); the value is the correctly rounded float32 of the number
 * Go's scanner reads: decimal by glibc strtof on a canonical spelling, hexadecimal by
 * hex_to_f32 (integer rounding).
 * ==================================================================================== */
static int lower_c(int c) { return (c >= 'A' && c <= 'Z') ? c + 32 : c; }

static size_t common_prefix_ci(const char* s, size_t n, const char* pre) {
    size_t k = 0;
    while (k < n && pre[k] && lower_c((unsigned char)s[k]) == pre[k]) k++;
    return k;
}

static int underscore_ok(const char* s, size_t n) {
    char saw = '^';
    size_t i = 0;
    if (n >= 1 && (s[0] == '-' || s[0] == '+')) { s++; n--; }
    int hex = 0;
    if (n >= 2 && s[0] == '0' && (lower_c(s[1]) == 'b' || lower_c(s[1]) == 'o' || lower_c(s[1]) == 'x')) {
        i = 2;
        saw = '0';
        hex = lower_c(s[1]) == 'x';
    }
    for (; i < n; i++) {
        int c = (unsigned char)s[i];
        if ((c >= '0' && c <= '9') || (hex && lower_c(c) >= 'a' && lower_c(c) <= 'f')) { saw = '0'; continue; }
        if (c == '_') {
            if (saw != '0') return 0;
            saw = '_';
            continue;
        }
        if (saw == '_') return 0;
        saw = '!';
    }
    return saw != '_';
}

/* A hexadecimal mantissa (its first 16 digits in mant; trunc: a nonzero digit after them)
 * × 2^e2, correctly rounded to float32: ties to even, subnormals (lsb 2^-149), ±Inf past the
 * largest finite value (atofHex's rounding, Go strconv/atof.go). Restated in integers because
 * glibc's strtof rounds some hexadecimal subnormals down (0x0.1234569p-125 → 0x123456 × 2^-149
 * where Go's atof32 table, and the exact value, give 0x123457). */
static float hex_to_f32(uint64_t mant, int trunc, long e2, int neg) {
    if (mant == 0) return neg ? -0.0f : 0.0f;
    int lz = __builtin_clzll(mant);
    uint64_t m = mant << lz;                                  /* top bit at 63 */
    long E = e2 + 63 - lz;                                    /* value in [2^E, 2^(E+1)) */
    double v;
    if (E > 127) {
        v = INFINITY;
    } else {
        long keep = E + 150 < 24 ? E + 150 : 24;              /* significand bits down to 2^-149 */
        uint64_t kept;
        int half, low;
        if (keep <= 0) {                                      /* below 2^-149 */
            kept = 0;
            half = keep == 0;                                 /* [2^-150, 2^-149): the half bit is the top one */
            low = keep == 0 ? ((m << 1) != 0 || trunc) : 1;
            keep = 0;
        } else {
            kept = m >> (64 - keep);
            uint64_t rest = keep < 64 ? m << keep : 0;
            half = (int)(rest >> 63);
            low = (rest << 1) != 0 || trunc;
        }
        if (half && (low || (kept & 1))) kept++;
        v = ldexp((double)kept, (int)(E - keep + 1));         /* exact; 2^128 → Inf below */
    }
    float f = (float)v;
    return neg ? -f : f;
}

int or_parse_float32(const char* s, uint32_t n, float* out) {
    *out = 0.0f;
    if (n == 0) return 1;
    /* special(): [+-]?(inf|infinity) or nan, case-insensitive */
    {
        size_t nsign = 0, k = 0;
        int sign = 1, is_inf = 0, is_nan = 0;
        char c0 = s[0];
        if (c0 == '+' || c0 == '-') {
            if (c0 == '-') sign = -1;
            nsign = 1;
            k = common_prefix_ci(s + 1, n - 1, "infinity");
            if (k > 3 && k < 8) k = 3;
            if (k == 3 || k == 8) is_inf = 1;
        } else if (c0 == 'i' || c0 == 'I') {
            k = common_prefix_ci(s, n, "infinity");
            if (k > 3 && k < 8) k = 3;
            if (k == 3 || k == 8) is_inf = 1;
        } else if (c0 == 'n' || c0 == 'N') {
            if (common_prefix_ci(s, n, "nan") == 3) { is_nan = 1; k = 3; }
        }
        if (is_inf || is_nan) {
            if (nsign + k != n) return 1;                     /* trailing junk: syntax error */
            *out = is_nan ? NAN : (sign > 0 ? INFINITY : -INFINITY);
            return is_inf ? 1 : 0;   /* +-Inf: ParseFloat returns Inf, nil → caller range-checks */
        }
    }
    /* readFloat */
    size_t i = 0;
    int neg = 0, hex = 0, underscores = 0, sawdot = 0, sawdigits = 0;
    long nd = 0, dp = 0;
    char expc = 'e';
    char* digs = (char*)malloc(n + 1);
    size_t nds = 0;
    if (!digs) return 1;
    if (i < n && (s[i] == '+' || s[i] == '-')) { neg = s[i] == '-'; i++; }
    if (i + 2 < n && s[i] == '0' && lower_c(s[i + 1]) == 'x') { hex = 1; i += 2; expc = 'p'; }
    for (; i < n; i++) {
        int c = (unsigned char)s[i];
        if (c == '_') { underscores = 1; continue; }
        if (c == '.') {
            if (sawdot) break;
            sawdot = 1;
            dp = nd;
            continue;
        }
        if (c >= '0' && c <= '9') {
            sawdigits = 1;
            if (c == '0' && nd == 0) { dp--; continue; }
            nd++;
            digs[nds++] = (char)c;
            continue;
        }
        if (hex && lower_c(c) >= 'a' && lower_c(c) <= 'f') {
            sawdigits = 1;
            nd++;
            digs[nds++] = (char)c;
            continue;
        }
        break;
    }
    if (!sawdigits) { free(digs); return 1; }
    if (!sawdot) dp = nd;
    if (hex) dp *= 4;
    if (i < n && lower_c((unsigned char)s[i]) == expc) {
        i++;
        if (i >= n) { free(digs); return 1; }
        long esign = 1;
        if (s[i] == '+') i++;
        else if (s[i] == '-') { i++; esign = -1; }
        if (i >= n || s[i] < '0' || s[i] > '9') { free(digs); return 1; }
        long e = 0;
        for (; i < n && ((s[i] >= '0' && s[i] <= '9') || s[i] == '_'); i++) {
            if (s[i] == '_') { underscores = 1; continue; }
            if (e < 10000) e = e * 10 + (s[i] - '0');
        }
        dp += e * esign;
    } else if (hex) { free(digs); return 1; }                 /* hex mantissa needs 'p' */
    if (underscores && !underscore_ok(s, i)) { free(digs); return 1; }
    if (i != n) { free(digs); return 1; }                     /* ParseFloat: whole string */
    if (nds == 0) { free(digs); *out = neg ? -0.0f : 0.0f; return 0; }
    if (hex) {
        uint64_t mant = 0;
        int trunc = 0;
        size_t nm = nds < 16 ? nds : 16;
        for (size_t q = 0; q < nds; q++) {
            int c = lower_c((unsigned char)digs[q]);
            int dv = c <= '9' ? c - '0' : c - 'a' + 10;
            if (q < nm) mant = mant * 16 + (uint64_t)dv;
            else if (dv) trunc = 1;
        }
        free(digs);
        float v = hex_to_f32(mant, trunc, dp - 4L * (long)nm, neg);
        *out = v;
        return isinf(v) ? 1 : 0;                              /* ErrRange */
    }
    /* canonical spelling: [-]0.DIGITSe<dp> (decimal only; glibc strtof rounds it correctly,
     * tests/test_oracle_golden.py::test_float32_parse_exact_rounding) */
    char* canon = (char*)malloc(nds + 48);
    if (!canon) { free(digs); return 1; }
    size_t w = 0;
    if (neg) canon[w++] = '-';
    canon[w++] = '0';
    canon[w++] = '.';
    memcpy(canon + w, digs, nds);
    w += nds;
    w += (size_t)sprintf(canon + w, "e%ld", dp);
    canon[w] = 0;
    float v = strtof(canon, NULL);
    free(canon);
    free(digs);
    *out = v;
    if (isinf(v)) return 1;                                   /* ErrRange */
    return 0;
}

int or_parse_pct(const char* s, uint32_t n, float* out) {
    *out = 0.0f;
    if (n == 0) return 0;                                     /* qdisc.go:129-131 */
    float v;
    if (or_parse_float32(s, n, &v)) return 1;                 /* :132-135 (syntax/range) */
    if (isnan(v)) return 1;                                   /* :136-138 */
    if ((double)v < 0.0 || (double)v > 100.0) return 1;       /* :139-141 */
    *out = v;
    return 0;
}

/* ======================================================================================
 * common.ParseRate (common/qdisc.go:162-199): strings.ToLower + strings.TrimSpace
 * (Unicode-aware, Go 1.18), suffix handling, strconv.ParseUint(rest, 10, 64).
 * ==================================================================================== */
static uint32_t utf8_decode(const unsigned char* s, size_t n, size_t* w) {
    unsigned c0 = s[0];
    if (c0 < 0x80) { *w = 1; return c0; }
    if (c0 >= 0xC2 && c0 <= 0xDF) {
        if (n >= 2 && (s[1] & 0xC0) == 0x80) { *w = 2; return ((c0 & 0x1F) << 6) | (s[1] & 0x3F); }
    } else if (c0 >= 0xE0 && c0 <= 0xEF) {
        unsigned lo = 0x80, hi = 0xBF;
        if (c0 == 0xE0) lo = 0xA0;
        if (c0 == 0xED) hi = 0x9F;
        if (n >= 3 && s[1] >= lo && s[1] <= hi && (s[2] & 0xC0) == 0x80) {
            *w = 3;
            return ((c0 & 0x0F) << 12) | ((s[1] & 0x3Fu) << 6) | (s[2] & 0x3Fu);
        }
    } else if (c0 >= 0xF0 && c0 <= 0xF4) {
        unsigned lo = 0x80, hi = 0xBF;
        if (c0 == 0xF0) lo = 0x90;
        if (c0 == 0xF4) hi = 0x8F;
        if (n >= 4 && s[1] >= lo && s[1] <= hi && (s[2] & 0xC0) == 0x80 && (s[3] & 0xC0) == 0x80) {
            *w = 4;
            return ((c0 & 0x07) << 18) | ((s[1] & 0x3Fu) << 12) | ((s[2] & 0x3Fu) << 6) | (s[3] & 0x3Fu);
        }
    }
    *w = 1;
    return 0xFFFD;                                            /* utf8.RuneError */
}

static int go_is_space(uint32_t r) {                         /* unicode.IsSpace */
    switch (r) {
    case '\t': case '\n': case '\v': case '\f': case '\r': case ' ': case 0x85: case 0xA0:
    case 0x1680: case 0x2028: case 0x2029: case 0x202F: case 0x205F: case 0x3000:
        return 1;
    }
    return r >= 0x2000 && r <= 0x200A;
}

int or_parse_rate(const char* s0, uint32_t n, uint64_t* out) {
    const unsigned char* s = (const unsigned char*)s0;
    *out = 0;
    /* decode runes, lower-case them (unicode.ToLower; only U+0130→'i' and U+212A→'k'
     * land in ASCII), then trim Unicode white space at both ends. */
    uint32_t* runes = (uint32_t*)malloc((n + 1) * sizeof(uint32_t));
    if (!runes) return 1;
    size_t nr = 0;
    for (size_t i = 0; i < n;) {
        size_t w;
        runes[nr++] = utf8_decode(s + i, n - i, &w);
        i += w;
    }
    size_t a = 0, b = nr;
    while (a < b && go_is_space(runes[a])) a++;
    while (b > a && go_is_space(runes[b - 1])) b--;
    char* t = (char*)malloc(b - a + 1);
    if (!t) { free(runes); return 1; }
    size_t m = 0;
    for (size_t k = a; k < b; k++) {
        uint32_t r = runes[k];
        char c;
        if (r < 0x80) c = (char)lower_c((int)r);
        else if (r == 0x130) c = 'i';
        else if (r == 0x212A) c = 'k';
        else c = (char)0x80;                                  /* any other rune: not a digit */
        t[m++] = c;
    }
    free(runes);
    if (m == 0) { free(t); return 0; }                        /* :164-166 */
    uint64_t mult = 1;
    if (m >= 3 && memcmp(t + m - 3, "bit", 3) == 0) m -= 3;           /* :169-170 */
    else if (m >= 3 && memcmp(t + m - 3, "bps", 3) == 0) { m -= 3; mult = 8; } /* :171-173 */
    uint64_t base = 1000;
    if (m >= 1 && t[m - 1] == 'i') { m -= 1; base = 1024; }           /* :179-182 */
    static const char units[4] = {'k', 'm', 'g', 't'};
    for (int u = 0; u < 4; u++) {                                     /* :184-192 */
        if (m >= 1 && t[m - 1] == units[u]) {
            m -= 1;
            for (int j = 0; j < u + 1; j++) mult *= base;
            break;
        }
    }
    /* strconv.ParseUint(rest, 10, 64) */
    if (m == 0) { free(t); return 1; }
    uint64_t v = 0;
    const uint64_t cutoff = UINT64_MAX / 10 + 1;
    for (size_t k = 0; k < m; k++) {
        unsigned char c = (unsigned char)t[k];
        if (c < '0' || c > '9') { free(t); return 1; }
        if (v >= cutoff) { free(t); return 1; }
        v *= 10;
        uint64_t v1 = v + (uint64_t)(c - '0');
        if (v1 < v) { free(t); return 1; }
        v = v1;
    }
    free(t);
    *out = v * mult;                                          /* :198 wrapping multiply */
    return 0;
}

/* ======================================================================================
 * net.ParseCIDR / net.ParseMAC (Go 1.18 net/ip.go, net/mac.go) — MakeVeth common/veth.go:13-41
 * ==================================================================================== */
#define GO_BIG 0xFFFFFF
static int go_dtoi(const char* s, size_t n, long* val, size_t* used) {
    long v = 0;
    size_t i;
    for (i = 0; i < n && s[i] >= '0' && s[i] <= '9'; i++) {
        v = v * 10 + (s[i] - '0');
        if (v >= GO_BIG) { *val = GO_BIG; *used = i; return 0; }
    }
    if (i == 0) { *val = 0; *used = 0; return 0; }
    *val = v;
    *used = i;
    return 1;
}
static int go_xtoi(const char* s, size_t n, long* val, size_t* used) {
    long v = 0;
    size_t i;
    for (i = 0; i < n; i++) {
        int c = (unsigned char)s[i];
        if (c >= '0' && c <= '9') v = v * 16 + (c - '0');
        else if (c >= 'a' && c <= 'f') v = v * 16 + (c - 'a' + 10);
        else if (c >= 'A' && c <= 'F') v = v * 16 + (c - 'A' + 10);
        else break;
        if (v >= GO_BIG) { *val = 0; *used = i; return 0; }
    }
    if (i == 0) { *val = 0; *used = i; return 0; }
    *val = v;
    *used = i;
    return 1;
}

static int go_parse_ipv4(const char* s, size_t n) {
    size_t pos = 0;
    for (int k = 0; k < 4; k++) {
        if (pos >= n) return 0;
        if (k > 0) {
            if (s[pos] != '.') return 0;
            pos++;
        }
        long v;
        size_t c;
        if (!go_dtoi(s + pos, n - pos, &v, &c) || v > 0xFF) return 0;
        if (c > 1 && s[pos] == '0') return 0;                 /* leading zeros rejected */
        pos += c;
    }
    return pos == n;
}

static int go_parse_ipv6(const char* s, size_t n) {
    int ellipsis = -1;
    size_t pos = 0;
    if (n >= 2 && s[0] == ':' && s[1] == ':') {
        ellipsis = 0;
        pos = 2;
        if (pos == n) return 1;
    }
    int i = 0;
    while (i < 16) {
        long v;
        size_t c;
        if (!go_xtoi(s + pos, n - pos, &v, &c) || v > 0xFFFF) return 0;
        if (pos + c < n && s[pos + c] == '.') {               /* trailing IPv4 */
            if (ellipsis < 0 && i != 12) return 0;
            if (i + 4 > 16) return 0;
            if (!go_parse_ipv4(s + pos, n - pos)) return 0;
            pos = n;
            i += 4;
            break;
        }
        i += 2;
        pos += c;
        if (pos == n) break;
        if (s[pos] != ':' || pos + 1 == n) return 0;
        pos++;
        if (s[pos] == ':') {
            if (ellipsis >= 0) return 0;
            ellipsis = i;
            pos++;
            if (pos == n) break;
        }
    }
    if (pos != n) return 0;
    if (i < 16) {
        if (ellipsis < 0) return 0;
    } else if (ellipsis >= 0) {
        return 0;
    }
    return 1;
}

int or_parse_cidr(const char* s, uint32_t n) {
    size_t slash = n;
    for (size_t k = 0; k < n; k++)
        if (s[k] == '/') { slash = k; break; }
    if (slash == n) return 0;
    int iplen = 4;
    int ok = go_parse_ipv4(s, slash);
    if (!ok) {
        iplen = 16;
        ok = go_parse_ipv6(s, slash);
    }
    long bits;
    size_t used;
    int dok = go_dtoi(s + slash + 1, n - slash - 1, &bits, &used);
    if (!ok || !dok || used != n - slash - 1 || bits < 0 || bits > 8 * iplen) return 0;
    return 1;
}

static int go_xtoi2(const char* s, size_t n, char e) {
    if (n > 2 && s[2] != e) return 0;
    if (n < 2) {
        /* xtoi over fewer than 2 chars cannot yield ei == 2 */
        return 0;
    }
    long v;
    size_t used;
    int ok = go_xtoi(s, 2, &v, &used);
    return ok && used == 2;
}

int or_parse_mac(const char* s, uint32_t n) {
    if (n < 14) return 0;
    if (s[2] == ':' || s[2] == '-') {
        if ((n + 1) % 3 != 0) return 0;
        size_t cnt = (n + 1) / 3;
        if (cnt != 6 && cnt != 8 && cnt != 20) return 0;
        for (size_t x = 0, i = 0; i < cnt; i++, x += 3)
            if (!go_xtoi2(s + x, n - x, s[2])) return 0;
        return 1;
    }
    if (s[4] == '.') {
        if ((n + 1) % 5 != 0) return 0;
        size_t cnt = 2 * (n + 1) / 5;
        if (cnt != 6 && cnt != 8 && cnt != 20) return 0;
        for (size_t x = 0, i = 0; i < cnt; i += 2, x += 5) {
            if (!go_xtoi2(s + x, 2, 0)) return 0;
            if (!go_xtoi2(s + x + 2, n - x - 2, s[4])) return 0;
        }
        return 1;
    }
    return 0;
}

/* ======================================================================================
 * netlink NewNetem / Percentage2u32 / time2Tick (vishvananda/netlink @ d40f9887b852)
 * ==================================================================================== */
uint32_t or_p2u(float p) {
    if (p == 100.0f) return 0xFFFFFFFFu;                      /* math.MaxUint32 */
    float q = p / 100.0f;                                     /* float32 division */
    float r = 4294967296.0f * q;                              /* float32(MaxUint32) = 2^32 */
    return (uint32_t)(int64_t)r;                              /* amd64: CVTTSS2SQ, truncate */
}

uint32_t or_time2tick(uint32_t t, double tick) {
    return (uint32_t)(int64_t)((double)t * tick);             /* uint32(float64(t)*tickInUsec) */
}

uint32_t or_tbf_burst(uint64_t rate) {
    uint32_t burst = (uint32_t)(rate / 250);                  /* qdisc.go:363 */
    if (burst < 5000) burst = 5000;                           /* :365-367 */
    return burst;
}

int32_t or_vni_from_uid(int64_t uid, int32_t base) {
    return (int32_t)(uint32_t)((uint64_t)(int64_t)base + (uint64_t)uid);   /* int32(VxlanBase + uid) */
}

/* common.MakeQdiscs (common/qdisc.go:20-126) */
void or_make_qdisc(const char* const* strs, const uint32_t* lens, uint32_t gap,
                   double tick, kdtn_qdisc* q) {
    memset(q, 0, sizeof(*q));
    int empty = gap == 0;
    for (int k = 0; k < KDTN_NPROP; k++)
        if (lens[k] != 0) empty = 0;
    if (empty) return;                                        /* :24-26 proto.Size == 0 */
#define S(k) strs[k], lens[k]
    uint32_t lat, jit;
    float lc, loss, lossc, dup, dupc, rp, rc, cp, cc;
    int e = 0;
    if (or_parse_duration(S(KDTN_P_LATENCY), &lat)) e = KDTN_E_LATENCY;                /* :28 */
    else if (or_parse_pct(S(KDTN_P_LATENCY_CORR), &lc)) e = KDTN_E_LATENCY_CORR;        /* :34 */
    else if (or_parse_duration(S(KDTN_P_JITTER), &jit)) e = KDTN_E_JITTER;              /* :40 */
    else if (or_parse_pct(S(KDTN_P_LOSS), &loss)) e = KDTN_E_LOSS;                      /* :46 */
    else if (or_parse_pct(S(KDTN_P_LOSS_CORR), &lossc)) e = KDTN_E_LOSS_CORR;           /* :52 */
    else if (or_parse_pct(S(KDTN_P_DUPLICATE), &dup)) e = KDTN_E_DUPLICATE;             /* :58 */
    else if (or_parse_pct(S(KDTN_P_DUPLICATE_CORR), &dupc)) e = KDTN_E_DUPLICATE_CORR;  /* :64 */
    else if (or_parse_pct(S(KDTN_P_REORDER_PROB), &rp)) e = KDTN_E_REORDER_PROB;        /* :70 */
    else if (or_parse_pct(S(KDTN_P_REORDER_CORR), &rc)) e = KDTN_E_REORDER_CORR;        /* :76 */
    else if (or_parse_pct(S(KDTN_P_CORRUPT_PROB), &cp)) e = KDTN_E_CORRUPT_PROB;        /* :82 */
    else if (or_parse_pct(S(KDTN_P_CORRUPT_CORR), &cc)) e = KDTN_E_CORRUPT_CORR;        /* :88 */
    if (e) { q->err = (uint8_t)e; return; }
    /* NewNetem (:94-107) */
    uint32_t latency = lat, jitter = jit, g = gap;
    uint32_t u_loss = or_p2u(loss), u_dup = or_p2u(dup);
    uint32_t delay_corr = 0, loss_corr = 0, dup_corr = 0;
    if (latency > 0 && jitter > 0) delay_corr = or_p2u(lc);
    if (u_loss > 0) loss_corr = or_p2u(lossc);
    if (u_dup > 0) dup_corr = or_p2u(dupc);
    latency = or_time2tick(latency, tick);
    if (latency > 0) jitter = or_time2tick(jitter, tick);
    uint32_t u_rp = or_p2u(rp), u_rc = or_p2u(rc);
    if (u_rp > 0 && g == 0) g = 1;
    uint32_t u_cp = or_p2u(cp), u_cc = or_p2u(cc);
    uint64_t rate;
    if (or_parse_rate(S(KDTN_P_RATE), &rate)) { q->err = KDTN_E_RATE; return; }        /* :110-114 */
#undef S
    q->latency = latency;
    q->delay_corr = delay_corr;
    q->limit = 1000;
    q->loss = u_loss;
    q->loss_corr = loss_corr;
    q->gap = g;
    q->duplicate = u_dup;
    q->duplicate_corr = dup_corr;
    q->jitter = jitter;
    q->reorder_prob = u_rp;
    q->reorder_corr = u_rc;
    q->corrupt_prob = u_cp;
    q->corrupt_corr = u_cc;
    q->has_netem = 1;
    if (rate != 0) {                                          /* :115-123 */
        q->has_tbf = 1;
        q->tbf_rate = rate;
        q->tbf_buffer = or_tbf_burst(rate);
        q->tbf_minburst = 1500;
    }
}

/* ======================================================================================
 * Reconcile epoch: gate (topology_controller.go:77-88), CalcDiff (:288-318),
 * EqualWithoutProperties (:342-351), daemon pure prefix (handler.go:316-492, 592-671).
 * ==================================================================================== */
static int link_key_eq(const kdtn_epoch_in* in, const kdtn_link_table* a, uint32_t i,
                       const kdtn_link_table* b, uint32_t j) {
    /* EqualWithoutProperties: LocalIntf, LocalIP, LocalMAC, PeerIntf, PeerIP, PeerMAC, PeerPod, UID */
    for (int k = 0; k < KDTN_NKEY; k++)
        if (!ostr_eq(tab_get(&in->kdict, a->key[k][i]), tab_get(&in->kdict, b->key[k][j]))) return 0;
    return a->uid[i] == b->uid[j];
}
static int link_props_eq(const kdtn_epoch_in* in, const kdtn_link_table* a, uint32_t i,
                         const kdtn_link_table* b, uint32_t j) {
    /* reflect.DeepEqual(oldLink.Properties, newLink.Properties): 12 strings + Gap */
    for (int k = 0; k < KDTN_NPROP; k++)
        if (!ostr_eq(tab_get(&in->pdict, a->prop[k][i]), tab_get(&in->pdict, b->prop[k][j]))) return 0;
    return a->gap[i] == b->gap[j];
}

/* pod map: informer store key "ns/name" (handler.go:27-41) */
typedef struct { char* key; uint32_t klen; uint32_t val; } pm_slot;
typedef struct { pm_slot* slots; uint64_t cap; } pmap;
static uint64_t fnv1a(const char* p, size_t n, uint64_t h) {
    for (size_t i = 0; i < n; i++) { h ^= (unsigned char)p[i]; h *= 1099511628211ull; }
    return h;
}
static void pm_init(pmap* m, uint64_t n) {
    m->cap = 16;
    while (m->cap < 2 * n + 16) m->cap <<= 1;
    m->slots = (pm_slot*)calloc(m->cap, sizeof(pm_slot));
}
static void pm_free(pmap* m) {
    for (uint64_t i = 0; i < m->cap; i++) free(m->slots[i].key);
    free(m->slots);
}
static char* make_key(ostr a, ostr b, uint32_t* klen) {
    char* k = (char*)malloc(a.n + b.n + 2);
    memcpy(k, a.p, a.n);
    k[a.n] = '/';
    memcpy(k + a.n + 1, b.p, b.n);
    *klen = a.n + 1 + b.n;
    return k;
}
static void pm_put_first(pmap* m, char* key, uint32_t klen, uint32_t val) {
    uint64_t h = fnv1a(key, klen, 1469598103934665603ull) & (m->cap - 1);
    for (;;) {
        pm_slot* s = &m->slots[h];
        if (!s->key) { s->key = key; s->klen = klen; s->val = val; return; }
        if (s->klen == klen && memcmp(s->key, key, klen) == 0) { free(key); return; } /* first wins */
        h = (h + 1) & (m->cap - 1);
    }
}
static int pm_get(const pmap* m, const char* key, uint32_t klen, uint32_t* val) {
    uint64_t h = fnv1a(key, klen, 1469598103934665603ull) & (m->cap - 1);
    for (;;) {
        const pm_slot* s = &m->slots[h];
        if (!s->key) return 0;
        if (s->klen == klen && memcmp(s->key, key, klen) == 0) { *val = s->val; return 1; }
        h = (h + 1) & (m->cap - 1);
    }
}

static void make_qdisc_rec(const kdtn_epoch_in* in, const kdtn_link_table* t, uint32_t j,
                           double tick, kdtn_qdisc* q) {
    const char* strs[KDTN_NPROP];
    uint32_t lens[KDTN_NPROP];
    for (int k = 0; k < KDTN_NPROP; k++) {
        ostr s = tab_get(&in->pdict, t->prop[k][j]);
        strs[k] = s.p;
        lens[k] = s.n;
    }
    or_make_qdisc(strs, lens, t->gap[j], tick, q);
}

/* MakeVeth(netns, intf, ip, mac): ParseCIDR then ParseMAC (common/veth.go:21-36) */
static int make_veth_err(ostr ip, ostr mac, int cidr_err, int mac_err) {
    if (ip.n != 0 && !or_parse_cidr(ip.p, ip.n)) return cidr_err;
    if (mac.n != 0 && !or_parse_mac(mac.p, mac.n)) return mac_err;
    return 0;
}

static double now_s(void) {
    struct timespec ts;
    clock_gettime(CLOCK_MONOTONIC, &ts);
    return (double)ts.tv_sec + 1e-9 * (double)ts.tv_nsec;
}

int or_reconcile_epoch(const kdtn_epoch_in* in, const or_pods* pods_in, double tick,
                       int32_t vxlan_base, uint32_t t_begin, uint32_t t_end, kdtn_batches* out) {
    return or_reconcile_epoch_timed(in, pods_in, tick, vxlan_base, t_begin, t_end, out, NULL);
}

int or_reconcile_epoch_timed(const kdtn_epoch_in* in, const or_pods* pods_in, double tick,
                             int32_t vxlan_base, uint32_t t_begin, uint32_t t_end,
                             kdtn_batches* out, double* loop_seconds) {
    const kdtn_topo_table* T = &in->topos;
    const kdtn_link_table* O = &in->realised;
    const kdtn_link_table* N = &in->desired;
    or_pods local;
    if (!pods_in) {
        local.n = T->n; local.ns = T->ns; local.name = T->name; local.src_ip = T->src_ip;
        local.net_ns = T->net_ns; local.flags = T->flags; local.base = 0;
        pods_in = &local;
    }
    const or_pods* P = pods_in;
    const kdtn_strtab* KD = &in->kdict;

    /* informer store: "ns/name" → pod index (first wins) */
    pmap pm;
    pm_init(&pm, P->n);
    for (uint32_t p = 0; p < P->n; p++) {
        uint32_t kl;
        char* k = make_key(tab_get(KD, P->ns[p]), tab_get(KD, P->name[p]), &kl);
        pm_put_first(&pm, k, kl, p);
    }
    /* VxlanManager maps per node: key "node\0vni" → net_ns id (first wins) */
    pmap vm;
    pm_init(&vm, in->vnis.n);
    for (uint32_t v = 0; v < in->vnis.n; v++) {
        ostr node = tab_get(KD, in->vnis.node[v]);
        uint32_t kl = node.n + 1 + 4;
        char* k = (char*)malloc(kl);
        memcpy(k, node.p, node.n);
        k[node.n] = 0;
        memcpy(k + node.n + 1, &in->vnis.vni[v], 4);
        pm_put_first(&vm, k, kl, in->vnis.net_ns[v]);
    }
    ostr dflt = {"default", 7};

    uint32_t nd = 0, na = 0, nu = 0;
    int rc = 0;
    const double t_start = now_s();   /* informer store + VNI maps exist before Reconcile */
    for (uint32_t t = t_begin; t < t_end; t++) {
        uint32_t rt = t - t_begin;
        if (out->del_off) out->del_off[rt] = nd;
        if (out->add_off) out->add_off[rt] = na;
        if (out->upd_off) out->upd_off[rt] = nu;
        uint32_t o0 = T->real_off[t], o1 = T->real_off[t + 1];
        uint32_t n0 = T->des_off[t], n1 = T->des_off[t + 1];
        int status_nil = (T->flags[t] & KDTN_TOPO_STATUS_NIL) != 0;
        int spec_nil = (T->flags[t] & KDTN_TOPO_SPEC_NIL) != 0;
        /* reflect.DeepEqual(topology.Status.Links, topology.Spec.Links)  (:77) */
        int same;
        if (status_nil || spec_nil) same = status_nil && spec_nil;
        else if (o1 - o0 != n1 - n0) same = 0;
        else {
            same = 1;
            for (uint32_t r = 0; r < o1 - o0 && same; r++)
                same = link_key_eq(in, O, o0 + r, N, n0 + r) && link_props_eq(in, O, o0 + r, N, n0 + r);
        }
        uint8_t act = same ? KDTN_ACT_SKIP : (status_nil ? KDTN_ACT_CREATED : KDTN_ACT_DIFF);
        if (out->action) out->action[rt] = act;
        if (act != KDTN_ACT_DIFF) continue;

        ostr l_srcip = tab_get(KD, T->src_ip[t]);
        ostr l_netns = tab_get(KD, T->net_ns[t]);
        ostr l_ns = tab_get(KD, T->ns[t]);

        /* CalcDiff(old = status.links, new = spec.links) — literal loops (:289-316) */
        for (uint32_t i = o0; i < o1; i++) {
            int found = 0;
            for (uint32_t j = n0; j < n1; j++) {
                if (link_key_eq(in, O, i, N, j)) {
                    found = 1;
                    if (!link_props_eq(in, O, i, N, j)) {          /* propertiesChanged */
                        if (nu >= out->upd_cap) { rc = KDTN_ENOSPC; goto done; }
                        if (out->upd_idx) out->upd_idx[nu] = j;
                        /* UpdateLinks (handler.go:644-663): MakeVeth(local) then MakeQdiscs */
                        kdtn_qdisc q;
                        make_qdisc_rec(in, N, j, tick, &q);
                        if (out->upd_qdisc) out->upd_qdisc[nu] = q;
                        if (out->upd_res) {
                            kdtn_resolved r;
                            memset(&r, 0, sizeof r);
                            r.peer_topo = 0xFFFFFFFFu;
                            r.vni = or_vni_from_uid(N->uid[j], vxlan_base);
                            int e = make_veth_err(tab_get(KD, N->key[KDTN_K_LOCAL_IP][j]),
                                                  tab_get(KD, N->key[KDTN_K_LOCAL_MAC][j]),
                                                  KDTN_E_VETH_CIDR, KDTN_E_VETH_MAC);
                            r.err = (uint8_t)(e ? e : q.err);
                            out->upd_res[nu] = r;
                        }
                        nu++;
                    }
                    break;
                }
            }
            if (!found) {
                if (nd >= out->del_cap) { rc = KDTN_ENOSPC; goto done; }
                if (out->del_idx) out->del_idx[nd] = i;
                if (out->del_res) {
                    /* delLink (handler.go:461-492) */
                    kdtn_resolved r;
                    memset(&r, 0, sizeof r);
                    r.peer_topo = 0xFFFFFFFFu;
                    r.vni = or_vni_from_uid(O->uid[i], vxlan_base);
                    r.err = (uint8_t)make_veth_err(tab_get(KD, O->key[KDTN_K_LOCAL_IP][i]),
                                                   tab_get(KD, O->key[KDTN_K_LOCAL_MAC][i]),
                                                   KDTN_E_VETH_CIDR, KDTN_E_VETH_MAC);
                    if (!r.err) {
                        /* vxlanManager.Get(vni) == localPod.NetNs on this node (:482-486) */
                        uint32_t kl = l_srcip.n + 5, val;
                        char* k = (char*)malloc(kl);
                        memcpy(k, l_srcip.p, l_srcip.n);
                        k[l_srcip.n] = 0;
                        memcpy(k + l_srcip.n + 1, &r.vni, 4);
                        if (pm_get(&vm, k, kl, &val) && ostr_eq(tab_get(KD, val), l_netns)) r.vni_hit = 1;
                        free(k);
                    }
                    out->del_res[nd] = r;
                }
                nd++;
            }
        }
        for (uint32_t j = n0; j < n1; j++) {
            int found = 0;
            for (uint32_t i = o0; i < o1; i++)
                if (link_key_eq(in, O, i, N, j)) { found = 1; break; }
            if (found) continue;
            if (na >= out->add_cap) { rc = KDTN_ENOSPC; goto done; }
            if (out->add_idx) out->add_idx[na] = j;
            kdtn_qdisc q;
            make_qdisc_rec(in, N, j, tick, &q);
            if (out->add_qdisc) out->add_qdisc[na] = q;
            if (out->add_res) {
                /* addLink pure prefix (handler.go:316-459) */
                kdtn_resolved r;
                memset(&r, 0, sizeof r);
                r.peer_topo = 0xFFFFFFFFu;
                r.vni = or_vni_from_uid(N->uid[j], vxlan_base);
                r.err = (uint8_t)make_veth_err(tab_get(KD, N->key[KDTN_K_LOCAL_IP][j]),
                                               tab_get(KD, N->key[KDTN_K_LOCAL_MAC][j]),
                                               KDTN_E_VETH_CIDR, KDTN_E_VETH_MAC);   /* :327 */
                ostr peer_pod = tab_get(KD, N->key[KDTN_K_PEER_POD][j]);
                if (r.err) {
                } else if (ostr_is(peer_pod, "localhost")) {                         /* :333 */
                    r.kind = KDTN_KIND_MACVLAN;
                } else if (peer_pod.n >= 9 && memcmp(peer_pod.p, "physical/", 9) == 0) { /* :348 */
                    r.kind = KDTN_KIND_PHYSICAL;
                    r.vtep = N->key[KDTN_K_PEER_POD][j];
                    /* m.Update: VNI held by another netns on this node (:177-179) */
                    uint32_t kl = l_srcip.n + 5, val;
                    char* k = (char*)malloc(kl);
                    memcpy(k, l_srcip.p, l_srcip.n);
                    k[l_srcip.n] = 0;
                    memcpy(k + l_srcip.n + 1, &r.vni, 4);
                    if (pm_get(&vm, k, kl, &val) && !ostr_eq(tab_get(KD, val), l_netns)) r.vni_hit = 1;
                    free(k);
                } else {
                    /* getPod(PeerPod, KubeNs || "default") (:375, :27-41) */
                    uint32_t kl, p;
                    char* k = make_key(l_ns.n ? l_ns : dflt, peer_pod, &kl);
                    int hit = pm_get(&pm, k, kl, &p);
                    free(k);
                    if (!hit) {
                        r.err = KDTN_E_PEER_LOOKUP;
                    } else {
                        r.peer_topo = P->base + p;
                        if (P->flags[p] & KDTN_TOPO_SPEC_NIL) {
                            r.err = KDTN_E_PEER_NO_LINKS;                             /* :380-384 */
                        } else {
                            ostr p_srcip = tab_get(KD, P->src_ip[p]);
                            ostr p_netns = tab_get(KD, P->net_ns[p]);
                            if (p_srcip.n == 0 || p_netns.n == 0) {
                                r.kind = KDTN_KIND_PEER_DEAD;                        /* :386-395 */
                            } else if (ostr_eq(p_srcip, l_srcip)) {
                                r.kind = KDTN_KIND_SAME_NODE;                        /* :399-418 */
                                r.err = (uint8_t)make_veth_err(tab_get(KD, N->key[KDTN_K_PEER_IP][j]),
                                                               tab_get(KD, N->key[KDTN_K_PEER_MAC][j]),
                                                               KDTN_E_PEER_VETH_CIDR, KDTN_E_PEER_VETH_MAC);
                            } else {
                                r.kind = KDTN_KIND_CROSS_NODE;                       /* :419-453 */
                                r.vtep = P->src_ip[p];
                                /* UpdateRemote → peer's Update → SetupVxLan → CreateOrUpdate:
                                 * net.ParseCIDR(IntfIp = link.PeerIp) (common/utils.go:45,
                                 * daemon/vxlan/vxlan.go:80-83); its error returns from addLink
                                 * (handler.go:448-451) after the local steps */
                                ostr pip = tab_get(KD, N->key[KDTN_K_PEER_IP][j]);
                                if (pip.n != 0 && !or_parse_cidr(pip.p, pip.n)) r.remote_err = KDTN_E_REMOTE_CIDR;
                                /* remote Update on the peer's node (:177-179) */
                                uint32_t kl2 = p_srcip.n + 5, val;
                                char* k2 = (char*)malloc(kl2);
                                memcpy(k2, p_srcip.p, p_srcip.n);
                                k2[p_srcip.n] = 0;
                                memcpy(k2 + p_srcip.n + 1, &r.vni, 4);
                                if (pm_get(&vm, k2, kl2, &val) && !ostr_eq(tab_get(KD, val), p_netns)) r.vni_hit = 1;
                                free(k2);
                            }
                        }
                    }
                }
                out->add_res[na] = r;
            }
            na++;
        }
    }
done:
    if (loop_seconds) *loop_seconds = now_s() - t_start;
    if (rc == 0) {
        uint32_t rt = t_end - t_begin;
        if (out->del_off) out->del_off[rt] = nd;
        if (out->add_off) out->add_off[rt] = na;
        if (out->upd_off) out->upd_off[rt] = nu;
    }
    out->n_del = nd;
    out->n_add = na;
    out->n_upd = nu;
    pm_free(&pm);
    pm_free(&vm);
    return rc;
}
