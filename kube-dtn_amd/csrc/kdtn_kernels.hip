// kdtn_kernels.hip — device code of the reconcile epoch. See kdtn_kernels.h for the
// data layout and launch order; DESIGN.md for the roofline accounting.
#include "kdtn_kernels.h"

namespace kdtn {

// ======================================================================================
// small helpers
// ======================================================================================
KD_INLINE uint32_t mix32(uint32_t h, uint32_t w) {
    h ^= w;
    h *= 0x85EBCA6Bu;
    h ^= h >> 13;
    return h;
}
KD_INLINE uint32_t fin32(uint32_t h) {
    h ^= h >> 16;
    h *= 0xC2B2AE35u;
    h ^= h >> 16;
    return h;
}

// EqualWithoutProperties key (7 string ids + uid as two words) and the DeepEqual'd
// properties (12 ids + Gap) of one record, loaded with independent loads (no short-circuit
// chains: every load of a comparison is in flight at once).
constexpr int KEYW = KDTN_NKEY + 2, PROPW = KDTN_NPROP + 1;
KD_INLINE void load_key(const DevLinks& L, uint32_t i, uint32_t* k) {
    const uint32_t* r = L.rec(i);
#pragma unroll
    for (int c = 0; c < KDTN_NKEY; ++c) k[c] = r[(COL_KEY0 + c) * TILE_RECS];
    const uint64_t u = (uint64_t)L.uid_at<false>(r, i);
    k[KDTN_NKEY] = (uint32_t)u;
    k[KDTN_NKEY + 1] = (uint32_t)(u >> 32);
}
KD_INLINE void load_props(const DevLinks& L, uint32_t i, uint32_t* p) {
    const uint32_t* r = L.rec(i);
#pragma unroll
    for (int c = 0; c < KDTN_NPROP; ++c) p[c] = r[(COL_PROP0 + c) * TILE_RECS];
    p[KDTN_NPROP] = r[COL_GAP * TILE_RECS];
}
template <int W>
KD_INLINE bool words_eq(const uint32_t* a, const uint32_t* b) {
    uint32_t d = 0;
#pragma unroll
    for (int c = 0; c < W; ++c) d |= a[c] ^ b[c];
    return d == 0;
}
// 32-bit hash of the EqualWithoutProperties key (controllers/topology_controller.go:342-351);
// interned ids: equal ids ⇔ equal strings.
KD_INLINE uint32_t key_hash_w(const uint32_t* k) {
    uint32_t h = 0x9E3779B9u;
#pragma unroll
    for (int c = 0; c < KEYW; ++c) h = mix32(h, k[c]);
    return fin32(h);
}

// Table gather with a 32-bit byte offset from a uniform base: selects the global_load
// "saddr" form (SGPR base + one offset VGPR) instead of a per-lane 64-bit address, which
// saves a VGPR pair and the 64-bit address arithmetic per gather. Every gathered table is
// well under 4 GiB (dictionaries, pod/VNI tables, bitsets).
template <typename T>
KD_INLINE T ldg(const T* base, uint32_t idx) {
    return *reinterpret_cast<const T*>(reinterpret_cast<const uint8_t*>(base) + idx * (uint32_t)sizeof(T));
}
template <typename T>
KD_INLINE T ldg_nt(const T* base, uint32_t idx) {
    return __builtin_nontemporal_load(
        reinterpret_cast<const T*>(reinterpret_cast<const uint8_t*>(base) + idx * (uint32_t)sizeof(T)));
}

// largest tt in [lo, hi) with off[tt] <= idx  (the segment containing idx)
KD_INLINE int find_seg(const uint32_t* off, int lo, int hi, uint32_t idx) {
    while (hi - lo > 1) {
        int mid = (lo + hi) >> 1;
        if (off[mid] <= idx) lo = mid;
        else hi = mid;
    }
    return lo;
}

KD_INLINE uint64_t lanemask_lt() {
    const int lane = threadIdx.x & 63;
    return lane == 0 ? 0ull : (~0ull >> (64 - lane));
}

// Stage the arena bytes of strings [s0, s1) into LDS with 16-B coalesced loads.
// Returns the LDS image base (byte a0 of the arena maps to buf), or nullptr when the
// slice does not fit (caller then reads the strings from global memory).
template <int CAPB = STAGE>
KD_INLINE const uint8_t* stage_slice(const uint8_t* bytes, const uint32_t* offs, uint32_t s0,
                                     uint32_t s1, uint4* buf, uint32_t* a0_out) {
    const uint32_t b0 = offs[s0], b1 = offs[s1];
    const uint32_t a0 = b0 & ~15u;
    *a0_out = a0;
    const uint32_t words = (b1 - a0 + 15) >> 4;
    if (words * 16 + 32 > (uint32_t)CAPB) return nullptr;   // uniform across the block; 32 B of
                                                           // slack for the parsers' dword reads
    const uint4* src = reinterpret_cast<const uint4*>(bytes + a0);
    for (uint32_t w = threadIdx.x; w < words; w += BLOCK) buf[w] = src[w];
    return reinterpret_cast<const uint8_t*>(buf);
}

// ======================================================================================
// dictionary parsing (one thread per distinct string)
// ======================================================================================
// Word k of a string's first 24 bytes (bytes past the end are garbage; callers mask by len).
KD_INLINE uint32_t wbyte(const uint32_t* w, int k) { return (w[k >> 2] >> (8 * (k & 3))) & 0xFFu; }

// ---- SWAR character classes over 4 bytes (exact per byte, no compares: pure VALU) ----
// high bit of each byte set where the byte is an ASCII digit
KD_INLINE uint32_t swar_digit(uint32_t x) {
    const uint32_t t = x ^ 0x30303030u;
    return ~((t | 0x80808080u) - 0x0A0A0A0Au) & ~t & 0x80808080u;
}
// high bit of each byte set where the byte equals the byte replicated in `rep`
KD_INLINE uint32_t swar_eq(uint32_t x, uint32_t rep) {
    const uint32_t t = x ^ rep;
    return ~(((t & 0x7F7F7F7Fu) + 0x7F7F7F7Fu) | t) & 0x80808080u;
}
// gather the 4 byte-high bits into a nibble (byte k → bit k): the products never overlap
KD_INLINE uint32_t swar_nib(uint32_t m) { return (((m >> 7) * 0x204081u) >> 21) & 0xFu; }
// 4 bytes of the string starting at byte q (q <= 19) of the 24-byte register image
KD_INLINE uint32_t window4(const uint32_t* w, uint32_t q) {
    const uint32_t i = q >> 2;
    const uint32_t lo = i == 0 ? w[0] : i == 1 ? w[1] : i == 2 ? w[2] : i == 3 ? w[3] : w[4];
    const uint32_t hi = i == 0 ? w[1] : i == 1 ? w[2] : i == 2 ? w[3] : i == 3 ? w[4] : w[5];
    return __builtin_amdgcn_alignbyte(hi, lo, q & 3u);
}
// the same for q <= 19 without control flow: word pairs selected by the bits of q >> 2
// (window4's nested selects compiled to branches and exec-mask updates per window)
KD_INLINE uint32_t window4_bf(const uint32_t* w, uint32_t q) {
    const uint32_t i = q >> 2;
    const bool o = i & 1u, t = i & 2u, f = i & 4u;
    const uint32_t l0 = o ? w[1] : w[0], h0 = o ? w[2] : w[1];
    const uint32_t l1 = o ? w[3] : w[2], h1 = o ? w[4] : w[3];
    const uint32_t lo = f ? w[4] : t ? l1 : l0, hi = f ? w[5] : t ? h1 : h0;
    return __builtin_amdgcn_alignbyte(hi, lo, q & 3u);
}
KD_INLINE bool hexb(uint32_t c) { return (c - '0' < 10u) | ((c | 0x20u) - 'a' < 6u); }
// high bit of each byte set where the byte is a hex digit [0-9a-fA-F]
KD_INLINE uint32_t swar_hex(uint32_t x) {
    const uint32_t t = (x | 0x20202020u) & 0x7F7F7F7Fu;                 // lower case, 7 bits
    const uint32_t ge_a = (t | 0x80808080u) - 0x61616161u;               // byte >= 'a' (no borrow)
    const uint32_t le_f = 0xE6E6E6E6u - t;                               // byte <= 'f' (no borrow)
    return swar_digit(x) | (ge_a & le_f & ~x & 0x80808080u);
}
// net.ParseMAC of the 6- and 8-group colon / hyphen forms (17 / 23 bytes) from the register
// image: hex digits at 3g and 3g+1, the separator s[2] at 3g+2 (common/veth.go:33; Go's
// xtoi2 groups). The byte-wise mac_ok decides the other layouts.
KD_INLINE bool mac_swar(const uint32_t* w, uint32_t len) {
    const uint32_t sep = wbyte(w, 2) * 0x01010101u;
    uint32_t H = 0, S = 0;
#pragma unroll
    for (int k = 0; k < 6; ++k) {
        H |= swar_nib(swar_hex(w[k])) << (4 * k);
        S |= swar_nib(swar_eq(w[k], sep)) << (4 * k);
    }
    // 17 bytes: hex at 0,1 3,4 ... 15,16; separators at 2,5,8,11,14
    constexpr uint32_t H17 = 0x1B6DBu, S17 = 0x4924u, H23 = 0x6DB6DBu, S23 = 0x124924u;
    const uint32_t hm = len == 17u ? H17 : H23, sm = len == 17u ? S17 : S23;
    return (H & hm) == hm && (S & sm) == sm;
}
// one dotted-quad field of n digits starting with the 4-byte window c: dtoi, <= 255 and no
// leading zero (net.parseIPv4, Go 1.18)
KD_INLINE uint32_t octet_ok(uint32_t c, uint32_t n) {
    const uint32_t d0 = (c & 0xFFu) - '0', d1 = ((c >> 8) & 0xFFu) - '0', d2 = ((c >> 16) & 0xFFu) - '0';
    const uint32_t v = d0 * 100u + d1 * 10u + d2;
    return (n >= 1u) & (n <= 3u) & ((n == 1u) | (d0 != 0u)) & ((n != 3u) | (v <= 255u));
}

// net.ParseCIDR validity from the register image of a string of <= 24 bytes
// (common/veth.go:22). Decides every string without ':' whose prefix has <= 2 digits;
// sets *slow for the rest (IPv6 candidates, long prefixes), which take cidr_ok().
KD_INLINE bool cidr_swar(const uint32_t* w, uint32_t len, bool* slow) {
    uint32_t D = 0, P = 0, S = 0, C = 0;
#pragma unroll
    for (int k = 0; k < 6; ++k) {
        D |= swar_nib(swar_digit(w[k])) << (4 * k);
        P |= swar_nib(swar_eq(w[k], 0x2E2E2E2Eu)) << (4 * k);   // '.'
        S |= swar_nib(swar_eq(w[k], 0x2F2F2F2Fu)) << (4 * k);   // '/'
        C |= swar_nib(swar_eq(w[k], 0x3A3A3A3Au)) << (4 * k);   // ':'
    }
    const uint32_t L = (1u << len) - 1u;
    D &= L;
    P &= L;
    S &= L;
    C &= L;
    const uint32_t s = __builtin_ctz(S | 0x1000000u);           // first '/' (24 if none)
    const uint32_t m = len - s - 1u;                             // prefix digits
    // generic parser only for IPv6 candidates (any IPv6 text has a colon) and for IPv4-looking
    // strings (first byte a digit) with a prefix of 3+ digits; anything else cannot parse
    // (ParseCIDR fails at once without a '/': MAC-shaped strings with ':' need no IPv6 parse)
    *slow = (C != 0u && S != 0u) | ((D & 1u) != 0u && m > 2u && s < len);
    const uint32_t sep = P | S;
    uint32_t ok = ((D | sep) == L) & (__builtin_popcount(P) == 3) & (__builtin_popcount(S) == 1) &
                  ((P >> s) == 0u) & ((sep & (sep << 1)) == 0u) & (D & 1u) & (s + 1u < len) & (s <= 15u);
    const uint32_t p1 = __builtin_ctz(P | 0x1000000u);
    const uint32_t P2 = P & (P - 1u);
    const uint32_t p2 = __builtin_ctz(P2 | 0x1000000u);
    const uint32_t p3 = __builtin_ctz((P2 & (P2 - 1u)) | 0x1000000u);
    if (!ok) return false;                                       // positions below are in range
    ok &= octet_ok(window4(w, 0), p1);
    ok &= octet_ok(window4(w, p1 + 1u), p2 - p1 - 1u);
    ok &= octet_ok(window4(w, p2 + 1u), p3 - p2 - 1u);
    ok &= octet_ok(window4(w, p3 + 1u), s - p3 - 1u);
    const uint32_t c = window4(w, s + 1u);                       // dtoi(prefix) <= 32
    const uint32_t bits = m == 1u ? (c & 0xFFu) - '0' : ((c & 0xFFu) - '0') * 10u + (((c >> 8) & 0xFFu) - '0');
    return ok && bits <= 32u;
}

// High-bit byte masks of two words → 8 position bits (bytes of lo at bits 0-3, of hi at 4-7):
// lo >> 7 and hi >> 3 put the flags at bits 8j and 8j + 4, and one multiply by
// 2^21 + 2^14 + 2^7 + 1 moves byte j's pair to bits 21 + j and 25 + j; the cross products land
// on distinct bits outside [21, 29), so nothing carries into the field.
KD_INLINE uint32_t swar_nib8(uint32_t lo, uint32_t hi) {
    return __builtin_amdgcn_ubfe(((lo >> 7) | (hi >> 3)) * 0x204081u, 21, 8);
}
// net.ParseCIDR validity from the register image, same contract as cidr_swar (decides every
// string of <= 24 bytes except the ones it routes to cidr_ok through *slow), with fewer VALU
// operations — k_kdict_flags is VALU-issue bound (380 VALU instructions per wave at HEAD,
// 4 cycles each on a SIMD16 = the kernel's time). No IPv4 CIDR with a prefix of <= 2 digits is
// longer than 18 bytes ("255.255.255.255/32"), so strings of <= 18 bytes are classified over
// five words in byte space with one range test: every byte of a valid one is in '.'..'9'
// (0x2E-0x39), the separators are the bytes below '0', and bit 0 tells '/' from '.'.
// Longer strings only need the routing decision: every slow case contains a '/'.
KD_INLINE bool cidr_swar2(const uint32_t* w, uint32_t len, bool* slow) {
    if (len > 18u) {
        uint32_t any = 0;
#pragma unroll
        for (int k = 0; k < 6; ++k) {
            const uint32_t lm = len >= 4u * k + 4u ? 0xFFFFFFFFu : len <= 4u * k ? 0u : (1u << (8u * (len - 4u * k))) - 1u;
            any |= swar_eq(w[k], 0x2F2F2F2Fu) & lm;
        }
        *slow = any != 0u;
        return false;
    }
    uint32_t r[5], d[5], s[5];
#pragma unroll
    for (int k = 0; k < 5; ++k) {
        const uint32_t x = w[k], t = x & 0x7F7F7F7Fu;
        const uint32_t ge2e = t + 0x52525252u, ge3a = t + 0x46464646u, ge30 = t + 0x50505050u;
        r[k] = ge2e & ~ge3a & ~x & 0x80808080u;                 // '.' .. '9'
        const uint32_t sep = r[k] & ~ge30;                       // '.' or '/'
        s[k] = sep & (x << 7);                                   // '/'
        d[k] = sep & ~(x << 7);                                  // '.'
    }
    const uint32_t L = (1u << len) - 1u;
    const uint32_t R = (swar_nib8(r[0], r[1]) | (swar_nib8(r[2], r[3]) << 8) | (swar_nib8(r[4], 0u) << 16)) & L;
    const uint32_t P = (swar_nib8(d[0], d[1]) | (swar_nib8(d[2], d[3]) << 8) | (swar_nib8(d[4], 0u) << 16)) & L;
    const uint32_t S = (swar_nib8(s[0], s[1]) | (swar_nib8(s[2], s[3]) << 8) | (swar_nib8(s[4], 0u) << 16)) & L;
    const uint32_t D = R & ~(P | S);
    const uint32_t sl = __builtin_ctz(S | 0x1000000u);          // first '/' (24 if none)
    const uint32_t m = len - sl - 1u;                            // prefix digits
    bool sv = (D & 1u) != 0u && m > 2u && sl < len;              // long prefix: generic parser
    if (R != L && S != 0u) {                                     // IPv6 candidate: a ':' and a '/'
        uint32_t c = 0;
#pragma unroll
        for (int k = 0; k < 5; ++k) c |= swar_nib(swar_eq(w[k], 0x3A3A3A3Au)) << (4 * k);
        sv |= (c & L) != 0u;
    }
    *slow = sv;
    const uint32_t sep = P | S;
    uint32_t ok = (R == L) & (__builtin_popcount(P) == 3) & (__builtin_popcount(S) == 1) &
                  ((P >> sl) == 0u) & ((sep & (sep << 1)) == 0u) & (D & 1u) & (sl + 1u < len) & (sl <= 15u);
    if (!ok) return false;                                       // positions below are in range
    const uint32_t p1 = __builtin_ctz(P);
    const uint32_t P2 = P & (P - 1u);
    const uint32_t p2 = __builtin_ctz(P2);
    const uint32_t p3 = __builtin_ctz(P2 & (P2 - 1u));
    ok &= octet_ok(w[0], p1);
    ok &= octet_ok(window4_bf(w, p1 + 1u), p2 - p1 - 1u);
    ok &= octet_ok(window4_bf(w, p2 + 1u), p3 - p2 - 1u);
    ok &= octet_ok(window4_bf(w, p3 + 1u), sl - p3 - 1u);
    const uint32_t c = window4_bf(w, sl + 1u);                      // dtoi(prefix) <= 32
    const uint32_t bits = m == 1u ? (c & 0xFFu) - '0' : ((c & 0xFFu) - '0') * 10u + (((c >> 8) & 0xFFu) - '0');
    return ok && bits <= 32u;
}

// One thread per key string, no LDS: the first 24 bytes are loaded as 7 aligned dwords and
// funnel-shifted into registers; CIDR/MAC validity, "localhost", "physical/" and "default"
// are decided there with SWAR class masks (no per-character control flow: the scalar unit,
// which executes every lane-mask operation of a branchy parser, was this kernel's bound).
// Strings longer than 24 bytes, with ':' (IPv6), long prefixes or shaped like a MAC take
// the generic parsers (kdtn_parse.h) on global memory. Each wave packs its 64
// predicate bits per set with a ballot (two u32 words per set, lanes 0 and 32).
// Predicate bits of one key string from its register image (first 24 bytes in w[]).
template <bool V1 = false>          // V1: the round-2 classifier (cidr_swar), A/B only
KD_INLINE uint32_t kdict_bits(const uint8_t* bytes, uint32_t b, uint32_t len, const uint32_t* w, uint32_t i,
                              uint32_t* special) {
    uint32_t f = 0;
    const uint32_t c0 = w[0] & 0xFFu;
    if (len && !hexb(c0) && c0 != ':') {
        // neither an IP (digit, hex digit or ':' first: parseIPv4 / parseIPv6) nor a MAC (hex
        // digit first): both predicates fail without classifying the bytes
        f = (1u << KB_CIDR_BAD) | (1u << KB_MAC_BAD);
    } else if (len) {
        bool slow = true, cok = false;
        if (len <= 24) cok = V1 ? cidr_swar(w, len, &slow) : cidr_swar2(w, len, &slow);
        if (slow) cok = cidr_ok(bytes + b, len);                       // common/veth.go:22
        if (!cok) f |= 1u << KB_CIDR_BAD;
        const uint32_t c2 = wbyte(w, 2), c4 = wbyte(w, 4);
        bool mok = false;                                              // common/veth.go:33
        // net.ParseMAC's necessary conditions, decided in registers: the length of one of its
        // six layouts and hex digits in the first group (s[0..1] for ':'/'-', s[0..3] for '.').
        // Only candidates run the byte-wise parser (an IPv4 CIDR like "10.5.123.45/31" has
        // s[4] == '.' and len 14, and used to take it in most waves).
        bool cand = false;
        if (c2 == ':' || c2 == '-') cand = (len == 17 || len == 23 || len == 59) && hexb(wbyte(w, 0)) && hexb(wbyte(w, 1));
        else if (c4 == '.') cand = (len == 14 || len == 19 || len == 49) && hexb(wbyte(w, 0)) && hexb(wbyte(w, 1)) &&
                                   hexb(c2) && hexb(wbyte(w, 3));
        if (cand) mok = (len == 17 || len == 23) ? mac_swar(w, len) : mac_ok(bytes + b, len);
        if (!mok) f |= 1u << KB_MAC_BAD;
    }
    const uint32_t w2b = w[2] & 0xFFu;
    if (len >= 9 && w[0] == 0x73796870u && w[1] == 0x6C616369u && w2b == '/')   // "phys" "ical" '/'
        f |= 1u << KB_PHYSICAL;                                        // handler.go:348
    if (len == 9 && w[0] == 0x61636F6Cu && w[1] == 0x736F686Cu && w2b == 't')   // "loca" "lhos" 't'
        atomicMin(special + SPECIAL_LOCALHOST, i);                     // handler.go:333
    if (len == 7 && w[0] == 0x61666564u && (w[1] & 0xFFFFFFu) == 0x746C75u)     // "defa" "ult"
        atomicMin(special + SPECIAL_DEFAULT, i);                       // getPod ns "" (handler.go:29-31)
    return f;
}

// Special key-string ids (SPECIAL_DEFAULT, SPECIAL_LOCALHOST) persist across uploads of an
// append-only dictionary; before a parse from string k0 the ids >= k0 are forgotten.
__global__ void k_special_clip(uint32_t* special, uint32_t k0) {
    const int t = threadIdx.x;
    if ((t == SPECIAL_DEFAULT || t == SPECIAL_LOCALHOST) && special[t] >= k0) special[t] = 0xFFFFFFFFu;
}

// The 7 aligned dwords holding a key string's first 24 bytes. The first 3 decide the cheap
// rejects (a first byte that starts neither an IP nor a MAC: kdict_bits then reads only bytes
// 0-8, for "physical/" / "localhost"); only the other lanes load the rest, so a wave of pod
// names or netns paths issues 3 window loads instead of 7.
KD_INLINE void kdict_window(const uint8_t* bytes, uint32_t b, uint32_t len, uint32_t* d) {
    const uint32_t* p = reinterpret_cast<const uint32_t*>(bytes + (b & ~3u));   // arena has 64 B slack
#pragma unroll
    for (int k = 0; k < 3; ++k) d[k] = p[k];
    const uint32_t c0 = (d[0] >> ((b & 3u) * 8u)) & 0xFFu;
#pragma unroll
    for (int k = 3; k < 7; ++k) d[k] = 0u;
    if (len && (hexb(c0) || c0 == ':'))
#pragma unroll
        for (int k = 3; k < 7; ++k) d[k] = p[k];
}

// One block of k_kdict_flags (strings [i0 - tid, +BLOCK), i0 = this thread's string; the block
// start a multiple of 64: every wave writes whole predicate words).
KD_INLINE void kdict_block(const uint8_t* bytes, const uint32_t* offs, uint32_t s0, uint32_t n, uint32_t* kbits,
                           uint32_t kb_words, uint32_t* special) {
    const uint32_t i = s0 + threadIdx.x;
    const int lane = threadIdx.x & 63;
    const uint32_t ic = i < n ? i : n;                   // offs[n] exists
    const uint32_t b = offs[ic];
    const uint32_t len = (i < n ? offs[ic + 1] : b) - b;
    uint32_t d[7];
    kdict_window(bytes, b, len, d);
    const uint32_t sh = (b & 3u) * 8u;
    uint32_t w[6];
#pragma unroll
    for (int k = 0; k < 6; ++k) w[k] = sh ? (d[k] >> sh) | (d[k + 1] << (32u - sh)) : d[k];
    const uint32_t f = i < n ? kdict_bits(bytes, b, len, w, i, special) : 0u;
    const uint32_t w0 = (i - lane) >> 5;                 // first word of this wave
#pragma unroll
    for (int k = 0; k < KB_NSETS; ++k) {
        const uint64_t m = __ballot((f >> k) & 1u);
        if (w0 < kb_words && (lane == 0 || lane == 32))
            kbits[(size_t)k * kb_words + w0 + (lane >> 5)] = lane ? (uint32_t)(m >> 32) : (uint32_t)m;
    }
}

// SUB strings per thread (block covers SUB*BLOCK consecutive strings): every offset load
// of the thread's strings is issued, then every string's 7 dwords, then the parses run —
// the kernel is latency-bound, so a wave keeps SUB strings' round trips in flight at once.
// Strings [first, n) (first a multiple of 64: every wave writes whole predicate words).
// X4: the window comes from three 16-B aligned loads (48 bytes) instead of seven dwords.
template <int SUB, bool X4, int NT>
__global__ void __launch_bounds__(NT) k_kdict_flags(const uint8_t* bytes, const uint32_t* offs,
                                                       uint32_t first, uint32_t n, uint32_t* kbits,
                                                       uint32_t kb_words, uint32_t* special) {
    const uint32_t i0 = first + blockIdx.x * NT * SUB + threadIdx.x;
    uint32_t b[SUB], len[SUB];
#pragma unroll
    for (int s = 0; s < SUB; ++s) {
        const uint32_t i = i0 + s * NT;
        const uint32_t ic = i < n ? i : n;                 // offs[n] exists
        b[s] = offs[ic];
        len[s] = (i < n ? offs[ic + 1] : b[s]) - b[s];
    }
    uint32_t d[SUB][7];
#pragma unroll
    for (int s = 0; s < SUB; ++s) {
        if constexpr (X4) {
            const uint4* p = reinterpret_cast<const uint4*>(bytes + (b[s] & ~15u));    // arena has 64 B slack
            const uint4 q0 = p[0], q1 = p[1], q2 = p[2];
            const uint32_t D[12] = {q0.x, q0.y, q0.z, q0.w, q1.x, q1.y, q1.z, q1.w, q2.x, q2.y, q2.z, q2.w};
            const uint32_t o = (b[s] >> 2) & 3u;
#pragma unroll
            for (int k = 0; k < 7; ++k)
                d[s][k] = o == 0 ? D[k] : o == 1 ? D[k + 1] : o == 2 ? D[k + 2] : D[k + 3];
        } else {
            kdict_window(bytes, b[s], len[s], d[s]);
        }
    }
    const int lane = threadIdx.x & 63;
#pragma unroll
    for (int s = 0; s < SUB; ++s) {
        const uint32_t i = i0 + s * NT;
        const uint32_t sh = (b[s] & 3u) * 8u;
        uint32_t w[6];
#pragma unroll
        for (int k = 0; k < 6; ++k)
            w[k] = sh ? (d[s][k] >> sh) | (d[s][k + 1] << (32u - sh)) : d[s][k];
        const uint32_t f = i < n ? kdict_bits(bytes, b[s], len[s], w, i, special) : 0u;
        const uint32_t w0 = (i - lane) >> 5;                   // first word of this wave
#pragma unroll
        for (int k = 0; k < KB_NSETS; ++k) {
            const uint64_t m = __ballot((f >> k) & 1u);
            if (w0 < kb_words && (lane == 0 || lane == 32))
                kbits[(size_t)k * kb_words + w0 + (lane >> 5)] = lane ? (uint32_t)(m >> 32) : (uint32_t)m;
        }
    }
}
template __global__ void k_kdict_flags<1, false, BLOCK>(const uint8_t*, const uint32_t*, uint32_t, uint32_t, uint32_t*, uint32_t, uint32_t*);

#if KDTN_PROFILING
// (A/B, measured slower: 0.122 vs 0.112 ms at 1M pods, `KDTN_KD_SUB=16`) Wave-staged form:
// the wave's 64 strings are contiguous in the arena, so the wave loads their
// span once with 16-B coalesced loads into its LDS slot (one 128-B line per 8 lanes instead of
// seven unaligned dword loads per lane touching ~10 lines each) and every lane reads its
// seven window dwords from LDS. A span over KD_WS_BYTES (long strings) reads global memory.
constexpr int KD_WS_BYTES = 2048;
__global__ void __launch_bounds__(BLOCK) k_kdict_flags_ws(const uint8_t* bytes, const uint32_t* offs, uint32_t first,
                                                          uint32_t n, uint32_t* kbits, uint32_t kb_words,
                                                          uint32_t* special) {
    __shared__ uint4 stage[BLOCK / 64][KD_WS_BYTES / 16];
    const uint32_t i = first + blockIdx.x * BLOCK + threadIdx.x;
    const int lane = threadIdx.x & 63;
    uint4* st = stage[threadIdx.x >> 6];
    const uint32_t ic = i < n ? i : n;                 // offs[n] exists
    const uint32_t b = offs[ic];
    const uint32_t len = (i < n ? offs[ic + 1] : b) - b;
    const uint32_t base = (uint32_t)__shfl((int)b, 0, 64) & ~15u;
    const uint32_t end = (uint32_t)__shfl((int)b, 63, 64) + 28u;     // the last lane's 7-dword window
    const uint32_t n16 = (end - base + 15u) >> 4;
    uint32_t d[7];
    if (n16 <= (uint32_t)(KD_WS_BYTES / 16)) {                       // wave-uniform
        const uint4* src = reinterpret_cast<const uint4*>(bytes + base);   // arena has 64 B slack
        for (uint32_t w = lane; w < n16; w += 64) st[w] = src[w];
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        const uint32_t* lw = reinterpret_cast<const uint32_t*>(st) + (((b & ~3u) - base) >> 2);
#pragma unroll
        for (int k = 0; k < 7; ++k) d[k] = lw[k];
    } else {
        const uint32_t* p = reinterpret_cast<const uint32_t*>(bytes + (b & ~3u));
#pragma unroll
        for (int k = 0; k < 7; ++k) d[k] = p[k];
    }
    const uint32_t sh = (b & 3u) * 8u;
    uint32_t w[6];
#pragma unroll
    for (int k = 0; k < 6; ++k) w[k] = sh ? (d[k] >> sh) | (d[k + 1] << (32u - sh)) : d[k];
    const uint32_t f = i < n ? kdict_bits(bytes, b, len, w, i, special) : 0u;
    const uint32_t w0 = (i - lane) >> 5;                   // first word of this wave
#pragma unroll
    for (int k = 0; k < KB_NSETS; ++k) {
        const uint64_t m = __ballot((f >> k) & 1u);
        if (w0 < kb_words && (lane == 0 || lane == 32))
            kbits[(size_t)k * kb_words + w0 + (lane >> 5)] = lane ? (uint32_t)(m >> 32) : (uint32_t)m;
    }
}
// (A/B, KDTN_KD_SUB=32) Persistent waves, software-pipelined: each wave walks 64-string
// chunks c = wave, wave + W, ... and issues chunk c + W's offset and window loads before it
// parses chunk c, so a wave keeps one chunk's round trips in flight while it computes.
__global__ void __launch_bounds__(BLOCK) k_kdict_flags_pp(const uint8_t* bytes, const uint32_t* offs, uint32_t first,
                                                          uint32_t n, uint32_t* kbits, uint32_t kb_words,
                                                          uint32_t* special) {
    const int lane = threadIdx.x & 63;
    const uint32_t W = gridDim.x * (BLOCK / 64);
    uint32_t c = blockIdx.x * (BLOCK / 64) + (threadIdx.x >> 6);
    const uint32_t nch = (n - first + 63) >> 6;
    auto load = [&](uint32_t ch, uint32_t& b, uint32_t& len, uint32_t* d) {
        const uint32_t i = first + ch * 64 + lane;
        const uint32_t ic = i < n ? i : n;
        b = offs[ic];
        len = (i < n ? offs[ic + 1] : b) - b;
        const uint32_t* p = reinterpret_cast<const uint32_t*>(bytes + (b & ~3u));
#pragma unroll
        for (int k = 0; k < 7; ++k) d[k] = p[k];
    };
    if (c >= nch) return;
    uint32_t b, len, d[7];
    load(c, b, len, d);
    for (; c < nch; c += W) {
        uint32_t nb = 0, nlen = 0, nd[7] = {0, 0, 0, 0, 0, 0, 0};
        if (c + W < nch) load(c + W, nb, nlen, nd);
        const uint32_t i = first + c * 64 + lane;
        const uint32_t sh = (b & 3u) * 8u;
        uint32_t w[6];
#pragma unroll
        for (int k = 0; k < 6; ++k) w[k] = sh ? (d[k] >> sh) | (d[k + 1] << (32u - sh)) : d[k];
        const uint32_t f = i < n ? kdict_bits(bytes, b, len, w, i, special) : 0u;
        const uint32_t w0 = (i - lane) >> 5;
#pragma unroll
        for (int k = 0; k < KB_NSETS; ++k) {
            const uint64_t m = __ballot((f >> k) & 1u);
            if (w0 < kb_words && (lane == 0 || lane == 32))
                kbits[(size_t)k * kb_words + w0 + (lane >> 5)] = lane ? (uint32_t)(m >> 32) : (uint32_t)m;
        }
        b = nb;
        len = nlen;
#pragma unroll
        for (int k = 0; k < 7; ++k) d[k] = nd[k];
    }
}
// (A/B, KDTN_KD_SUB=42) the product kernel with the round-2 classifier (cidr_swar)
__global__ void __launch_bounds__(BLOCK) k_kdict_flags_v1(const uint8_t* bytes, const uint32_t* offs, uint32_t first,
                                                          uint32_t n, uint32_t* kbits, uint32_t kb_words,
                                                          uint32_t* special) {
    const uint32_t i = first + blockIdx.x * BLOCK + threadIdx.x;
    const int lane = threadIdx.x & 63;
    const uint32_t ic = i < n ? i : n;
    const uint32_t b = offs[ic];
    const uint32_t len = (i < n ? offs[ic + 1] : b) - b;
    const uint32_t* p = reinterpret_cast<const uint32_t*>(bytes + (b & ~3u));
    uint32_t d[7];
#pragma unroll
    for (int k = 0; k < 7; ++k) d[k] = p[k];
    const uint32_t sh = (b & 3u) * 8u;
    uint32_t w[6];
#pragma unroll
    for (int k = 0; k < 6; ++k) w[k] = sh ? (d[k] >> sh) | (d[k + 1] << (32u - sh)) : d[k];
    const uint32_t f = i < n ? kdict_bits<true>(bytes, b, len, w, i, special) : 0u;
    const uint32_t w0 = (i - lane) >> 5;
#pragma unroll
    for (int k = 0; k < KB_NSETS; ++k) {
        const uint64_t m = __ballot((f >> k) & 1u);
        if (w0 < kb_words && (lane == 0 || lane == 32))
            kbits[(size_t)k * kb_words + w0 + (lane >> 5)] = lane ? (uint32_t)(m >> 32) : (uint32_t)m;
    }
}
// (A/B, KDTN_KD_SUB=40) the launch floor: offsets only, one ballot store per wave and set
__global__ void __launch_bounds__(BLOCK) k_kdict_null(const uint8_t* bytes, const uint32_t* offs, uint32_t first,
                                                      uint32_t n, uint32_t* kbits, uint32_t kb_words, uint32_t*) {
    const uint32_t i = first + blockIdx.x * BLOCK + threadIdx.x;
    const int lane = threadIdx.x & 63;
    const uint32_t ic = i < n ? i : n;
    const uint32_t b = offs[ic];
    const uint32_t len = (i < n ? offs[ic + 1] : b) - b;
    const uint64_t m = __ballot(len > 12u);
    const uint32_t w0 = (i - lane) >> 5;
    if (w0 < kb_words && (lane == 0 || lane == 32))
        kbits[w0 + (lane >> 5)] = lane ? (uint32_t)(m >> 32) : (uint32_t)m;
}
// (A/B, KDTN_KD_SUB=41) the load floor: offsets and the 7-dword window, a hash ballot
__global__ void __launch_bounds__(BLOCK) k_kdict_loadonly(const uint8_t* bytes, const uint32_t* offs, uint32_t first,
                                                          uint32_t n, uint32_t* kbits, uint32_t kb_words, uint32_t*) {
    const uint32_t i = first + blockIdx.x * BLOCK + threadIdx.x;
    const int lane = threadIdx.x & 63;
    const uint32_t ic = i < n ? i : n;
    const uint32_t b = offs[ic];
    const uint32_t* p = reinterpret_cast<const uint32_t*>(bytes + (b & ~3u));
    uint32_t h = 0;
#pragma unroll
    for (int k = 0; k < 7; ++k) h = h * 31u + p[k];
    const uint64_t m = __ballot(h & 1u);
    const uint32_t w0 = (i - lane) >> 5;
    if (w0 < kb_words && (lane == 0 || lane == 32))
        kbits[w0 + (lane >> 5)] = lane ? (uint32_t)(m >> 32) : (uint32_t)m;
}
template __global__ void k_kdict_flags<1, true, BLOCK>(const uint8_t*, const uint32_t*, uint32_t, uint32_t, uint32_t*, uint32_t, uint32_t*);
template __global__ void k_kdict_flags<2, false, BLOCK>(const uint8_t*, const uint32_t*, uint32_t, uint32_t, uint32_t*, uint32_t, uint32_t*);
template __global__ void k_kdict_flags<4, false, BLOCK>(
    const uint8_t*, const uint32_t*, uint32_t, uint32_t, uint32_t*, uint32_t, uint32_t*);
template __global__ void k_kdict_flags<1, false, 64>(
    const uint8_t*, const uint32_t*, uint32_t, uint32_t, uint32_t*, uint32_t, uint32_t*);
template __global__ void k_kdict_flags<1, false, 1024>(const uint8_t*, const uint32_t*, uint32_t, uint32_t, uint32_t*, uint32_t, uint32_t*);
#endif

// One property string's interpretations: WHICH = 7 all three, else one of PD_DUR / PD_PCT /
// PD_RATE (the split launch gives each interpretation its own threads: more waves in flight
// for a latency-bound parse, and each parse path alone needs fewer registers).
template <int WHICH>
KD_INLINE void pdict_parse_one(const uint8_t* s, uint32_t len, double tick, uint32_t* pct_out,
                               uint2* dur_out, uint2* rate_out, bool* rate_bad) {
    if constexpr ((WHICH & PD_DUR) != 0) {
        uint32_t dur = 0;
        const bool dok = parse_duration_us(s, len, &dur);
        *dur_out = dok ? make_uint2(dur, time2tick(dur, tick)) : make_uint2(0u, 1u);   // DUR_ERR
    }
    if constexpr ((WHICH & PD_PCT) != 0) {
        float pct;
        *pct_out = parse_pct(s, len, &pct) ? p2u(pct) : PCT_ERR;
    }
    if constexpr ((WHICH & PD_RATE) != 0) {
        uint64_t r = 0;
        const bool rok = (WHICH & PD_RATE_GENERIC) ? parse_rate_generic(s, len, &r) : parse_rate(s, len, &r);
        *rate_out = rok ? make_uint2((uint32_t)r, (uint32_t)(r >> 32)) : make_uint2(0xFFFFFFFFu, 0xFFFFFFFFu);
        *rate_bad = !rok;
    }
}

template <int WHICH>
KD_INLINE void pdict_parse_block(const uint8_t* bytes, const uint32_t* offs, uint32_t s0, uint32_t n, double tick,
                                 uint32_t* ppct, uint2* pdur, uint2* prate, uint32_t* rate_err, uint4* buf) {
    const uint32_t s1 = min(s0 + BLOCK, n);
    uint32_t a0;
    const bool staged = stage_slice(bytes, offs, s0, s1, buf, &a0) != nullptr;
    __syncthreads();
    const uint32_t i = s0 + threadIdx.x;
    bool bad = false;
    if (i < n) {
        const uint32_t b = offs[i], len = offs[i + 1] - b;
        uint32_t pct;
        uint2 dur, rate;
        const uint8_t* str = staged ? reinterpret_cast<const uint8_t*>(buf) + (b - a0) : bytes + b;
        pdict_parse_one<WHICH>(str, len, tick, &pct, &dur, &rate, &bad);
        if constexpr ((WHICH & PD_PCT) != 0) ppct[i] = pct;
        if constexpr ((WHICH & PD_DUR) != 0) pdur[i] = dur;
        if constexpr ((WHICH & PD_RATE) != 0) prate[i] = rate;
    }
    if constexpr ((WHICH & PD_RATE) != 0) {
        const uint64_t m = __ballot(bad);
        const int lane = threadIdx.x & 63;
        if (lane == 0 || lane == 32) rate_err[((i - lane) >> 5) + (lane >> 5)] = lane ? (uint32_t)(m >> 32) : (uint32_t)m;
    }
}

// Strings [first, n) (first a multiple of 64: every wave writes whole rate_err words).
// SPLIT: gridDim.y = 3, blockIdx.y picks the interpretation.
template <bool SPLIT>
__global__ void __launch_bounds__(BLOCK) k_pdict_parse(const uint8_t* bytes, const uint32_t* offs,
                                                       uint32_t first, uint32_t n, double tick, uint32_t* ppct,
                                                       uint2* pdur, uint2* prate, uint32_t* rate_err) {
    __shared__ uint4 buf[STAGE / 16];
    const uint32_t s0 = first + blockIdx.x * BLOCK;
    if constexpr (SPLIT) {
        if (blockIdx.y == 0) pdict_parse_block<PD_PCT>(bytes, offs, s0, n, tick, ppct, pdur, prate, rate_err, buf);
        else if (blockIdx.y == 1) pdict_parse_block<PD_DUR>(bytes, offs, s0, n, tick, ppct, pdur, prate, rate_err, buf);
        else pdict_parse_block<PD_RATE>(bytes, offs, s0, n, tick, ppct, pdur, prate, rate_err, buf);
    } else {
        pdict_parse_block<PD_DUR | PD_PCT | PD_RATE>(bytes, offs, s0, n, tick, ppct, pdur, prate, rate_err, buf);
    }
}
// Both dictionaries' parses in one launch (independent work, one kernel boundary less per
// epoch): blocks [0, 3 * nbp) parse property strings [p0, P), interpretation b / nbp (the
// heavier blocks first), the rest classify key strings [k0, D) as k_kdict_flags does.
KD_INLINE void dict_parse_block(const uint8_t* kd_bytes, const uint32_t* kd_offs, uint32_t k0, uint32_t D,
                                 uint32_t* kbits, uint32_t kb_words, uint32_t* special, const uint8_t* pd_bytes,
                                 const uint32_t* pd_offs, uint32_t p0, uint32_t P, uint32_t nbp, double tick,
                                 uint32_t* ppct, uint2* pdur, uint2* prate, uint32_t* rate_err, uint32_t nbk,
                                 uint4* buf) {
    uint32_t b = blockIdx.x;
    if (nbk) {                              // (key-string blocks first)
        if (b < nbk) {
            kdict_block(kd_bytes, kd_offs, k0 + b * BLOCK, D, kbits, kb_words, special);
            return;
        }
        b -= nbk;
    } else if (b >= 3 * nbp) {
        kdict_block(kd_bytes, kd_offs, k0 + (b - 3 * nbp) * BLOCK, D, kbits, kb_words, special);
        return;
    }
    const uint32_t y = b / nbp, s0 = p0 + (b - y * nbp) * BLOCK;
    if (y == 0) pdict_parse_block<PD_PCT>(pd_bytes, pd_offs, s0, P, tick, ppct, pdur, prate, rate_err, buf);
    else if (y == 1) pdict_parse_block<PD_DUR>(pd_bytes, pd_offs, s0, P, tick, ppct, pdur, prate, rate_err, buf);
    else pdict_parse_block<PD_RATE>(pd_bytes, pd_offs, s0, P, tick, ppct, pdur, prate, rate_err, buf);
}
__global__ void __launch_bounds__(BLOCK) k_dict_parse(const uint8_t* kd_bytes, const uint32_t* kd_offs, uint32_t k0,
                                                      uint32_t D, uint32_t* kbits, uint32_t kb_words,
                                                      uint32_t* special, const uint8_t* pd_bytes,
                                                      const uint32_t* pd_offs, uint32_t p0, uint32_t P, uint32_t nbp,
                                                      double tick, uint32_t* ppct, uint2* pdur, uint2* prate,
                                                      uint32_t* rate_err, uint32_t nbk) {
    __shared__ uint4 buf[STAGE / 16];
    dict_parse_block(kd_bytes, kd_offs, k0, D, kbits, kb_words, special, pd_bytes, pd_offs, p0, P, nbp, tick, ppct,
                     pdur, prate, rate_err, nbk, buf);
}
#if KDTN_PROFILING
// (A/B) the same held to the SGPR budget of 7 waves per SIMD (k_kdict_flags alone runs at 7;
// the fused kernel's 112 SGPRs allow 6)
__global__ void __launch_bounds__(BLOCK) __attribute__((amdgpu_waves_per_eu(7, 8)))
k_dict_parse_w7(const uint8_t* kd_bytes, const uint32_t* kd_offs, uint32_t k0, uint32_t D, uint32_t* kbits,
                uint32_t kb_words, uint32_t* special, const uint8_t* pd_bytes, const uint32_t* pd_offs, uint32_t p0,
                uint32_t P, uint32_t nbp, double tick, uint32_t* ppct, uint2* pdur, uint2* prate, uint32_t* rate_err,
                uint32_t nbk) {
    __shared__ uint4 buf[STAGE / 16];
    dict_parse_block(kd_bytes, kd_offs, k0, D, kbits, kb_words, special, pd_bytes, pd_offs, p0, P, nbp, tick, ppct,
                     pdur, prate, rate_err, nbk, buf);
}
#endif

#if KDTN_PROFILING
// (profiling) one interpretation alone: WHICH = PD_DUR / PD_PCT / PD_RATE
template <int WHICH>
__global__ void __launch_bounds__(BLOCK) k_pdict_only(const uint8_t* bytes, const uint32_t* offs, uint32_t first,
                                                      uint32_t n, double tick, uint32_t* ppct, uint2* pdur,
                                                      uint2* prate, uint32_t* rate_err) {
    __shared__ uint4 buf[STAGE / 16];
    pdict_parse_block<WHICH>(bytes, offs, first + blockIdx.x * BLOCK, n, tick, ppct, pdur, prate, rate_err, buf);
}
template __global__ void k_pdict_only<PD_DUR>(const uint8_t*, const uint32_t*, uint32_t, uint32_t, double, uint32_t*,
                                              uint2*, uint2*, uint32_t*);
template __global__ void k_pdict_only<PD_PCT>(const uint8_t*, const uint32_t*, uint32_t, uint32_t, double, uint32_t*,
                                              uint2*, uint2*, uint32_t*);
template __global__ void k_pdict_only<PD_RATE>(const uint8_t*, const uint32_t*, uint32_t, uint32_t, double, uint32_t*,
                                               uint2*, uint2*, uint32_t*);
template __global__ void k_pdict_only<PD_RATE | PD_RATE_GENERIC>(const uint8_t*, const uint32_t*, uint32_t, uint32_t,
                                                                 double, uint32_t*, uint2*, uint2*, uint32_t*);
#endif
template __global__ void k_pdict_parse<false>(const uint8_t*, const uint32_t*, uint32_t, uint32_t, double, uint32_t*,
                                              uint2*, uint2*, uint32_t*);
template __global__ void k_pdict_parse<true>(const uint8_t*, const uint32_t*, uint32_t, uint32_t, double, uint32_t*,
                                             uint2*, uint2*, uint32_t*);

// ======================================================================================
// pod-status table + lookup tables
// ======================================================================================
KD_INLINE void pods_fill_one(const DevTopos& T, uint32_t slice, uint32_t rank_base, uint4* pods, uint32_t t);

__global__ void __launch_bounds__(BLOCK) k_pods_fill(DevTopos T, uint32_t slice, uint32_t rank_base,
                                                     uint4* pods) {
    pods_fill_one(T, slice, rank_base, pods, blockIdx.x * BLOCK + threadIdx.x);
}

// The epoch's first launch: zero the sync header and look-back area (n16 16-B words, blocks
// [0, nbz)) and fill this rank's pod-status rows (the other blocks; slice 0 = none).
__global__ void __launch_bounds__(BLOCK) k_epoch_begin(uint4* sync, uint32_t n16, uint32_t nbz, DevTopos T,
                                                       uint32_t slice, uint32_t rank_base, uint4* pods) {
    if (blockIdx.x < nbz) {
        for (uint32_t i = blockIdx.x * BLOCK + threadIdx.x; i < n16; i += nbz * BLOCK) sync[i] = make_uint4(0u, 0u, 0u, 0u);
        return;
    }
    pods_fill_one(T, slice, rank_base, pods, (blockIdx.x - nbz) * BLOCK + threadIdx.x);
}

KD_INLINE void pods_fill_one(const DevTopos& T, uint32_t slice, uint32_t rank_base, uint4* pods, uint32_t t) {
    if (t >= slice) return;
    uint4 e;
    if (t < T.n) {
        e.x = T.ns[t];
        e.y = T.name[t];
        e.z = T.src_ip[t];
        e.w = T.net_ns[t] | ((T.flags[t] & KDTN_TOPO_SPEC_NIL) ? 0x80000000u : 0u);
    } else {
        e = make_uint4(0xFFFFFFFFu, 0xFFFFFFFFu, 0u, 0u);   // padding: never inserted
    }
    pods[rank_base + t] = e;
}

// Pod lookup table (informer store, handler.go:27-41), direct-mapped by the kdict id of
// the pod's name: slot[name] = {ns, g<<2|physical<<1|spec_nil, src_ip|netns_empty<<31,
// stamp<<1|multi}. A peer lookup is ONE 16-B gather with no probing: the slot belongs to
// this epoch when its stamp matches, and answers (ns, name) when ns matches. Names shared
// by several pods (other namespaces, or duplicate keys) set `multi`; their lookups go to a
// small overflow table of pod indices keyed by (ns, name), which keeps the informer's
// first-wins (smallest index) with one CAS + atomicMin per colliding pod. The stamp (per
// context, incremented each epoch) makes clearing the table unnecessary.
KD_INLINE uint32_t pod_probe_slot(uint32_t home, uint32_t i, uint32_t mask) {
    const uint32_t b = (home >> 3) + (i >> 3);
    return ((b << 3) + ((home + i) & 7u)) & mask;
}
KD_INLINE uint32_t pod_home(uint32_t mask, uint32_t ns, uint32_t name) {
    return (uint32_t)hash64(((uint64_t)ns << 32) | name) & mask;
}
// Overflow slots are {stamp:32 | g:32} words: a slot of an older epoch reads as empty, so
// the table needs no clearing between epochs (the stamp is the direct table's).
KD_INLINE void ovf_insert(const uint4* pods, uint32_t g, uint32_t ns, uint32_t name, unsigned long long* ovf,
                          uint32_t mask, uint32_t stamp) {
    const uint32_t home = pod_home(mask, ns, name);
    const unsigned long long mine = ((unsigned long long)stamp << 32) | g;
    for (uint32_t i = 0;; ++i) {
        const uint32_t h = pod_probe_slot(home, i, mask);
        unsigned long long cur = __hip_atomic_load(ovf + h, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        while ((uint32_t)(cur >> 32) != stamp) {                 // stale: claim it
            const unsigned long long prev = atomicCAS(ovf + h, cur, mine);
            if (prev == cur) return;
            cur = prev;
        }
        const uint32_t og = (uint32_t)cur;
        if (og == g) return;
        const uint4 o = pods[og];
        if (o.x == ns && o.y == name) {
            atomicMin(ovf + h, mine);                           // first topology wins (same stamp)
            return;
        }
    }
}

// Thread t's pod in the gathered table of nr ranks (rank-major, total = slice * nr): rank
// t % nr, local index t / nr, so a wave's pods come from every rank at about the same informer
// position and their name slots lie close together (in rank-major order consecutive rows
// are ~nr informer positions apart: at N = 8 the slot stores and verify loads touched 2x the
// lines of N = 1).
// Rows past the gathered table (total) are the late pods of kdtn_epoch_late_pods, in order.
KD_INLINE uint32_t pod_order(uint32_t t, uint32_t total, uint32_t nr) {
    if (nr <= 1 || t >= total) return t;
    const uint32_t slice = total / nr;
    return (t % nr) * slice + t / nr;
}

// "physical/" prefix of key string `id` from its bytes (the KB_PHYSICAL predicate, without
// waiting for k_kdict_flags: the lookup build runs beside the dictionary parses)
KD_INLINE uint32_t name_physical(const uint8_t* kd_bytes, const uint32_t* kd_offs, uint32_t id) {
    const uint32_t ob = kd_offs[id], len = kd_offs[id + 1] - ob;
    if (len < 9) return 0u;
    const uint32_t* p = reinterpret_cast<const uint32_t*>(kd_bytes + (ob & ~3u));   // arena has 64 B slack
    const uint32_t d0 = p[0], d1 = p[1], d2 = p[2], d3 = p[3], sh = ob & 3u;
    const uint32_t w0 = __builtin_amdgcn_alignbyte(d1, d0, sh), w1 = __builtin_amdgcn_alignbyte(d2, d1, sh);
    const uint32_t w2 = __builtin_amdgcn_alignbyte(d3, d2, sh);
    return (w0 == 0x73796870u && w1 == 0x6C616369u && (w2 & 0xFFu) == '/') ? 1u : 0u;   // "phys" "ical" '/'
}

// phys_bits: the KB_PHYSICAL bitset of a finished key-string parse, or null (the PHYSICAL bit
// from the name's bytes: the lookup build beside the parses, A/B)
template <int PER>
__global__ void __launch_bounds__(BLOCK) k_pod_direct_scatter(const uint4* pods, uint32_t total,
                                                              const uint32_t* phys_bits, const uint8_t* kd_bytes,
                                                              const uint32_t* kd_offs, uint4* slots, uint32_t stamp,
                                                              uint32_t nd, uint32_t nr, uint32_t gathered) {
    // PER rows per thread, every row load issued before the first slot store (latency-bound)
    const uint32_t t0 = blockIdx.x * BLOCK * PER + threadIdx.x;
    uint32_t g[PER];
    uint4 e[PER];
#pragma unroll
    for (int q = 0; q < PER; ++q) {
        const uint32_t t = t0 + q * BLOCK;
        g[q] = t < total ? pod_order(t, gathered, nr) : 0u;
        e[q] = t < total ? pods[g[q]] : make_uint4(0xFFFFFFFFu, 0u, 0u, 0u);
    }
#pragma unroll
    for (int q = 0; q < PER; ++q) {
        if (e[q].x == 0xFFFFFFFFu || e[q].y >= nd) continue;   // padding row / name outside this dictionary
        const uint32_t y = e[q].y;
        const uint32_t phys = phys_bits ? (phys_bits[y >> 5] >> (y & 31)) & 1u : name_physical(kd_bytes, kd_offs, y);
        slots[y] = make_uint4(e[q].x, (g[q] << 2) | (phys << 1) | (e[q].w >> 31),
                              e[q].z | ((e[q].w & 0x7FFFFFFFu) == 0 ? 0x80000000u : 0u), stamp << 1);
    }
}
template __global__ void k_pod_direct_scatter<1>(const uint4*, uint32_t, const uint32_t*, const uint8_t*, const uint32_t*,
                                                 uint4*, uint32_t, uint32_t, uint32_t, uint32_t);
template __global__ void k_pod_direct_scatter<4>(const uint4*, uint32_t, const uint32_t*, const uint8_t*, const uint32_t*,
                                                 uint4*, uint32_t, uint32_t, uint32_t, uint32_t);
#if KDTN_PROFILING
template __global__ void k_pod_direct_scatter<2>(const uint4*, uint32_t, const uint32_t*, const uint8_t*, const uint32_t*,
                                                 uint4*, uint32_t, uint32_t, uint32_t, uint32_t);
#endif

// Pods whose name slot was won by another pod: mark the name `multi` and put both pods
// into the overflow table (duplicates are rare; the table then answers every lookup of
// that name).
KD_INLINE void pod_verify_one(const uint4* pods, uint32_t total, uint4* slots, uint32_t stamp,
                               unsigned long long* ovf, uint32_t mask, uint32_t nd, uint32_t g) {
    if (g >= total) return;
    const uint4 e = pods[g];
    if (e.x == 0xFFFFFFFFu || e.y >= nd) return;
    const uint4 w = slots[e.y];
    const uint32_t owner = w.y >> 2;
    if (owner == g) return;
    reinterpret_cast<uint32_t*>(slots + e.y)[3] = (stamp << 1) | 1u;
    ovf_insert(pods, g, e.x, e.y, ovf, mask, stamp);
    ovf_insert(pods, owner, pods[owner].x, e.y, ovf, mask, stamp);
}

__global__ void __launch_bounds__(BLOCK) k_pod_direct_verify(const uint4* pods, uint32_t total, uint4* slots,
                                                             uint32_t stamp, unsigned long long* ovf, uint32_t mask,
                                                             uint32_t nd) {
    pod_verify_one(pods, total, slots, stamp, ovf, mask, nd, blockIdx.x * BLOCK + threadIdx.x);
}

__global__ void __launch_bounds__(BLOCK) k_vni_pack(const uint32_t* node, const int32_t* vni,
                                                    const uint32_t* net_ns, uint32_t n, uint4* ents) {
    const uint32_t v = blockIdx.x * BLOCK + threadIdx.x;
    if (v < n) ents[v] = make_uint4(node[v], (uint32_t)vni[v], net_ns[v], 0u);
}

// Slot contents after the build: the entry itself (first wins), or node = ~0 (empty).
__global__ void __launch_bounds__(BLOCK) k_vni_fill(const uint4* ents, const uint32_t* slots, uint32_t nslots,
                                                    uint4* out) {
    const uint32_t h = blockIdx.x * BLOCK + threadIdx.x;
    if (h >= nslots) return;
    const uint32_t v = slots[h];
    out[h] = v == 0xFFFFFFFFu ? make_uint4(0xFFFFFFFFu, 0xFFFFFFFFu, 0xFFFFFFFFu, 0u) : ents[v];
}

// VxlanManager snapshot: slots hold the smallest entry index with key (node, vni).
__global__ void __launch_bounds__(BLOCK) k_vni_ht_build(const uint4* ents, uint32_t n, uint32_t* slots,
                                                        uint32_t mask) {
    const uint32_t v = blockIdx.x * BLOCK + threadIdx.x;
    if (v >= n) return;
    const uint4 e = ents[v];
    uint32_t h = (uint32_t)hash64(((uint64_t)e.x << 32) | e.y) & mask;
    for (;;) {
        const uint32_t prev = atomicCAS(&slots[h], 0xFFFFFFFFu, v);
        if (prev == 0xFFFFFFFFu) return;
        const uint4 o = ents[prev];
        if (o.x == e.x && o.y == e.y) {
            atomicMin(&slots[h], v);                 // first entry wins
            return;
        }
        h = (h + 1) & mask;
    }
}

// getPod(name, ns) (handler.go:27-41) → {g|POD_* flags, src_ip|netns_empty<<31}; x = 0xFFFFFFFF
// on a miss. Empty slots hold all-ones, which no (ns, name) key equals (ids < 2^31).
typedef unsigned int u32x2 __attribute__((ext_vector_type(2)));
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

template <bool NT>
KD_INLINE uint4 pod_slot(const DevTables& tb, uint32_t name) {
    if constexpr (NT) {           // little reuse: keep L2 for the parsed tables
        const u32x4 v = ldg_nt(reinterpret_cast<const u32x4*>(tb.pod_direct), name);
        return make_uint4(v.x, v.y, v.z, v.w);
    } else {
        return ldg(tb.pod_direct, name);
    }
}
// Resolve a lookup of (ns, name) whose direct slot already read as w.
// Returns {g | POD_SPEC_NIL | POD_PHYSICAL, src_ip | netns_empty<<31}; x = 0xFFFFFFFF on a miss.
KD_INLINE uint2 pod_resolve(const DevTables& tb, uint32_t ns, uint32_t name, uint4 w) {
    if (ns == 0xFFFFFFFFu || (w.w >> 1) != tb.pod_stamp) return make_uint2(0xFFFFFFFFu, 0u);
    if ((w.w & 1u) == 0) {
        if (w.x != ns) return make_uint2(0xFFFFFFFFu, 0u);
        return make_uint2((w.y >> 2) | ((w.y & 1u) << 31) | ((w.y & 2u) << 29), w.z);
    }
    // name shared by several pods: overflow table of pod indices (rare)
    const uint32_t home = pod_home(tb.ovf_mask, ns, name);
    for (uint32_t i = 0;; ++i) {
        const unsigned long long w8 = ldg(tb.pod_ovf, pod_probe_slot(home, i, tb.ovf_mask));
        if ((uint32_t)(w8 >> 32) != tb.pod_stamp) return make_uint2(0xFFFFFFFFu, 0u);   // empty this epoch
        const uint32_t g = (uint32_t)w8;
        const uint4 e = ldg(tb.pods, g);
        if (e.x == ns && e.y == name) {
            const uint32_t phys = (w.y >> 1) & 1u;          // a property of the name string
            return make_uint2(g | (e.w & POD_SPEC_NIL) | (phys ? POD_PHYSICAL : 0u),
                              e.z | ((e.w & 0x7FFFFFFFu) == 0 ? 0x80000000u : 0u));
        }
    }
}

// VxlanManager.Get(vni) on node `node`: net_ns id, or 0xFFFFFFFF when absent. The slots hold
// the entries themselves ({node, vni, net_ns}, node = ~0 when empty): one gather per probe.
KD_INLINE uint32_t vni_lookup(const DevTables& tb, uint32_t node, int32_t vni) {
    if (tb.vni_mask == 0) return 0xFFFFFFFFu;
    uint32_t h = (uint32_t)hash64(((uint64_t)node << 32) | (uint32_t)vni) & tb.vni_mask;
    for (;;) {
        const uint4 e = ldg(tb.vnis, h);
        if (e.x == 0xFFFFFFFFu) return 0xFFFFFFFFu;
        if (e.x == node && e.y == (uint32_t)vni) return e.z;
        h = (h + 1) & tb.vni_mask;
    }
}

// ======================================================================================
// per-entry outputs: MakeQdiscs, delLink / addLink / UpdateLinks pure prefix
// ======================================================================================
// Columns of one link record that the outputs need, loaded together (one round trip).
struct RecCols {
    uint32_t lip, lmac, pp, pip;      // local_ip, local_mac, peer_pod, peer_ip (kdict ids)
    uint32_t pmac;                    // peer_mac (VAR_GLDS bulk emission only: VAR_PMAC_COLS)
    uint32_t prop[KDTN_NPROP];        // pdict ids
    uint32_t gap;
    int64_t uid;
};

template <bool NTL>
KD_INLINE void load_cols(const DevLinks& L, uint32_t j, bool keys, bool props, RecCols& c) {
    const uint32_t* r = L.rec(j);
    if (keys) {
        c.lip = L.col<NTL>(r, COL_KEY0 + KDTN_K_LOCAL_IP);
        c.lmac = L.col<NTL>(r, COL_KEY0 + KDTN_K_LOCAL_MAC);
        c.pp = L.col<NTL>(r, COL_KEY0 + KDTN_K_PEER_POD);
        c.pip = L.col<NTL>(r, COL_KEY0 + KDTN_K_PEER_IP);
        c.uid = L.uid_at<NTL>(r, j);
    }
    if (props) {
#pragma unroll
        for (int k = 0; k < KDTN_NPROP; ++k) c.prop[k] = L.col<NTL>(r, COL_PROP0 + k);
        c.gap = L.col<NTL>(r, COL_GAP);
    }
}

// Parsed-table values of one record's properties (12 independent gathers, issued together).
// The property ids die once the gathers are issued: only `empty`, `gap` and the rate id
// (for the rare all-ones rate) stay live.
struct PropVals {
    uint2 lat, jit, rt;
    uint32_t pct[9];                  // latency_corr, loss, loss_corr, duplicate, duplicate_corr,
                                      // reorder_prob, reorder_corr, corrupt_prob, corrupt_corr
    uint32_t gap, rate_id;
    bool empty;                       // all 12 strings "" and gap 0 (proto.Size == 0, :24)
};
constexpr int PCT_FIELDS[9] = {KDTN_P_LATENCY_CORR, KDTN_P_LOSS, KDTN_P_LOSS_CORR, KDTN_P_DUPLICATE,
                               KDTN_P_DUPLICATE_CORR, KDTN_P_REORDER_PROB, KDTN_P_REORDER_CORR,
                               KDTN_P_CORRUPT_PROB, KDTN_P_CORRUPT_CORR};

template <int V>
KD_INLINE void gather_props(const RecCols& c, const DevTables& tb, PropVals& v) {
    if constexpr ((V & VAR_MASK_EMPTY) != 0) {
        // "" (id 0) parses to 0 in every table: only lanes with a string issue the gather
        const uint32_t il = c.prop[KDTN_P_LATENCY], ij = c.prop[KDTN_P_JITTER], ir = c.prop[KDTN_P_RATE];
        v.lat = il ? ldg(tb.pdur, il) : make_uint2(0u, 0u);
        v.jit = ij ? ldg(tb.pdur, ij) : make_uint2(0u, 0u);
        v.rt = ir ? ldg(tb.prate, ir) : make_uint2(0u, 0u);
    } else {
        v.lat = ldg(tb.pdur, c.prop[KDTN_P_LATENCY]);
        v.jit = ldg(tb.pdur, c.prop[KDTN_P_JITTER]);
        v.rt = ldg(tb.prate, c.prop[KDTN_P_RATE]);
    }
#pragma unroll
    for (int k = 0; k < 9; ++k) {
        const uint32_t id = c.prop[PCT_FIELDS[k]];
        // (VAR_SKIP_PCT: profiling only, wrong results) the id stands in for the parsed value
        if constexpr ((V & VAR_SKIP_PCT) != 0) v.pct[k] = id;
        else if constexpr ((V & VAR_MASK_EMPTY) != 0) v.pct[k] = id ? ldg(tb.ppct, id) : 0u;
        else v.pct[k] = ldg(tb.ppct, id);
    }
    uint32_t any = c.gap;
#pragma unroll
    for (int k = 0; k < KDTN_NPROP; ++k) any |= c.prop[k];   // id 0 == ""
    v.empty = any == 0;
    v.gap = c.gap;
    v.rate_id = c.prop[KDTN_P_RATE];
}

KD_INLINE bool dur_err(uint2 d) { return d.x == 0u && d.y == 1u; }
KD_INLINE bool rate_bad(const DevTables& tb, const PropVals& v) {
    if ((v.rt.x & v.rt.y) != 0xFFFFFFFFu) return false;          // rare: error or 2^64-1
    return (ldg(tb.rate_err, v.rate_id >> 5) >> (v.rate_id & 31)) & 1u;
}

// MakeQdiscs over parsed dictionary entries (common/qdisc.go:20-126 + netlink NewNetem)
KD_INLINE void qdisc_from(const DevTables& tb, const PropVals& v, uint32_t* q) {
#pragma unroll
    for (int w = 0; w < 18; ++w) q[w] = 0;
    if (v.empty) return;
    const uint32_t lco = v.pct[0], los = v.pct[1], lsc = v.pct[2], dup = v.pct[3], dpc = v.pct[4],
                   rop = v.pct[5], roc = v.pct[6], cop = v.pct[7], coc = v.pct[8];
    uint32_t err = 0;                            // first failing parse, reference order
    if (dur_err(v.lat)) err = KDTN_E_LATENCY;
    else if (lco == PCT_ERR) err = KDTN_E_LATENCY_CORR;
    else if (dur_err(v.jit)) err = KDTN_E_JITTER;
    else if (los == PCT_ERR) err = KDTN_E_LOSS;
    else if (lsc == PCT_ERR) err = KDTN_E_LOSS_CORR;
    else if (dup == PCT_ERR) err = KDTN_E_DUPLICATE;
    else if (dpc == PCT_ERR) err = KDTN_E_DUPLICATE_CORR;
    else if (rop == PCT_ERR) err = KDTN_E_REORDER_PROB;
    else if (roc == PCT_ERR) err = KDTN_E_REORDER_CORR;
    else if (cop == PCT_ERR) err = KDTN_E_CORRUPT_PROB;
    else if (coc == PCT_ERR) err = KDTN_E_CORRUPT_CORR;
    else if (rate_bad(tb, v)) err = KDTN_E_RATE;
    if (err) {
        q[17] = err << 16;                       // byte 70 = err
        return;
    }
    // NewNetem
    const uint32_t lat_us = v.lat.x, jit_us = v.jit.x, lat_t = v.lat.y;
    q[0] = lat_t;                                                   // latency
    q[1] = (lat_us > 0 && jit_us > 0) ? lco : 0u;                  // delay_corr
    q[2] = 1000u;                                                   // limit
    q[3] = los;                                                     // loss
    q[4] = los > 0 ? lsc : 0u;                                      // loss_corr
    q[5] = (rop > 0 && v.gap == 0) ? 1u : v.gap;                    // gap
    q[6] = dup;                                                     // duplicate
    q[7] = dup > 0 ? dpc : 0u;                                      // duplicate_corr
    q[8] = lat_t > 0 ? v.jit.y : jit_us;                            // jitter
    q[9] = rop;
    q[10] = roc;
    q[11] = cop;
    q[12] = coc;
    const uint64_t rate = ((uint64_t)v.rt.y << 32) | v.rt.x;
    uint32_t has_tbf = 0;
    if (rate != 0) {
        uint32_t burst = (uint32_t)(rate / 250ull);              // getTbfBurst
        if (burst < 5000u) burst = 5000u;
        q[13] = burst;
        q[14] = v.rt.x;
        q[15] = v.rt.y;
        q[16] = 1500u;
        has_tbf = 1;
    }
    q[17] = 1u | (has_tbf << 8);                 // has_netem, has_tbf, err = 0
}

template <int V>
KD_INLINE void store_qdisc(uint2* dst, const uint32_t* q) {
    if constexpr ((V & VAR_NO_QSTORE) != 0) {
#pragma unroll
        for (int w = 0; w < 18; ++w) asm volatile("" ::"v"(q[w]));   // keep the work alive
        return;
    }
    u32x2* d = reinterpret_cast<u32x2*>(dst);
#pragma unroll
    for (int w = 0; w < 9; ++w) {
        u32x2 v;
        v.x = q[2 * w];
        v.y = q[2 * w + 1];
        if constexpr ((V & VAR_NT_STORE) != 0) __builtin_nontemporal_store(v, d + w);
        else d[w] = v;
    }
}

template <int V>
KD_INLINE void store_q8(uint2* dst, uint2 v) {
    if constexpr ((V & VAR_NT_STORE) != 0) {
        u32x2 x;
        x.x = v.x;
        x.y = v.y;
        __builtin_nontemporal_store(x, reinterpret_cast<u32x2*>(dst));
    } else {
        *dst = v;
    }
}

template <int V>
KD_INLINE void store_res(uint4* dst, uint4 r) {
    if constexpr ((V & VAR_NT_STORE) != 0) {
        u32x4 v;
        v.x = r.x;
        v.y = r.y;
        v.z = r.z;
        v.w = r.w;
        __builtin_nontemporal_store(v, reinterpret_cast<u32x4*>(dst));
    } else {
        *dst = r;
    }
}

template <int V>
KD_INLINE void store_idx(uint32_t* dst, uint32_t v) {
    if constexpr ((V & VAR_NT_STORE) != 0) __builtin_nontemporal_store(v, dst);
    else *dst = v;
}

KD_INLINE uint4 pack_res(uint32_t peer, int32_t vni, uint32_t vtep, uint32_t kind, uint32_t err,
                         uint32_t hit, uint32_t remote_err = 0) {
    return make_uint4(peer, (uint32_t)vni, vtep, kind | (err << 8) | (hit << 16) | (remote_err << 24));
}

KD_INLINE bool kbit(const DevTables& tb, int set, uint32_t id) {
    return (ldg(tb.kbits + (size_t)set * tb.kb_words, id >> 5) >> (id & 31)) & 1u;
}

// MakeVeth(netns, intf, ip, mac) validity from key-string predicates (common/veth.go:21-36)
KD_INLINE uint32_t veth_err(const DevTables& tb, uint32_t ip, uint32_t mac, uint32_t ecidr,
                            uint32_t emac) {
    if (kbit(tb, KB_CIDR_BAD, ip)) return ecidr;
    if (kbit(tb, KB_MAC_BAD, mac)) return emac;
    return 0;
}

KD_INLINE int32_t vni_of(int32_t base, int64_t uid) {   // common/utils.go:29-31
    return (int32_t)(uint32_t)((uint64_t)(int64_t)base + (uint64_t)uid);
}

struct TopoCtx {       // the local pod of a batch (topology_controller.go:181-186)
    uint32_t ns, src, netns;
};

// delLink (handler.go:461-492) from loaded columns (keys). The *_calc forms compute an
// entry's outputs without storing them (the caller may not know its position yet).
KD_INLINE uint4 del_calc(const RecCols& c, const TopoCtx& tc, const DevTables& tb) {
    const int32_t vni = vni_of(tb.vxlan_base, c.uid);
    const uint32_t err = veth_err(tb, c.lip, c.lmac, KDTN_E_VETH_CIDR, KDTN_E_VETH_MAC);
    uint32_t hit = 0;
    if (!err) hit = vni_lookup(tb, tc.src, vni) == tc.netns;
    return pack_res(0xFFFFFFFFu, vni, 0, 0, err, hit);
}

template <int V>
KD_INLINE void emit_del(const RecCols& c, uint32_t i, const TopoCtx& tc, const DevTables& tb,
                        const RecOut& out, uint32_t e, bool res) {
    store_idx<V>(out.del_idx + e, i);
    if (res) store_res<V>(out.del_res + e, del_calc(c, tc, tb));
}

// UpdateLinks entry (handler.go:644-663): MakeVeth(local), then MakeQdiscs
template <int V>
KD_INLINE uint4 upd_calc(const RecCols& c, const DevTables& tb, bool res, uint32_t* q) {
    PropVals v;
    gather_props<V>(c, tb, v);
    uint32_t werr = 0;
    if (res) werr = veth_err(tb, c.lip, c.lmac, KDTN_E_VETH_CIDR, KDTN_E_VETH_MAC);
    qdisc_from(tb, v, q);
    const uint32_t err = werr ? werr : (q[17] >> 16) & 0xFF;
    return pack_res(0xFFFFFFFFu, vni_of(tb.vxlan_base, c.uid), 0, 0, err, 0);
}

template <int V>
KD_INLINE void emit_upd(const RecCols& c, uint32_t j, const DevTables& tb, const RecOut& out,
                        uint32_t e, bool res, bool qd, uint32_t* q) {
    store_idx<V>(out.upd_idx + e, j);
    if (!res && !qd) return;
    const uint4 r = upd_calc<V>(c, tb, res, q);
    if (res) store_res<V>(out.upd_res + e, r);
}

// addLink pure prefix (handler.go:316-459) + MakeQdiscs, from loaded columns, in two steps:
// add_gather issues every lookup the entry may need (parsed properties, key-string
// predicate words, the home slot of the peer's pod) without using any, so an entry costs one
// gather round trip and the caller can put the next records' column loads behind it;
// add_finish combines them in the reference's step order and stores the outputs.
struct AddGath {
    PropVals v;
    uint4 slot;                       // direct slot of peer_pod
    uint32_t lns, kb_ip, kb_mac, kb_pip;
};

template <int V>
KD_INLINE void add_gather(const RecCols& c, const TopoCtx& tc, const DevTables& tb, bool res, bool qd,
                          AddGath& g) {
    if (qd) gather_props<V>(c, tb, g.v);
    if (!res) return;
    g.lns = tc.ns == 0 ? tb.special[SPECIAL_DEFAULT] : tc.ns;                     // :29-31
    if constexpr ((V & VAR_SKIP_KB3) != 0) {             // profiling only, wrong results
        g.kb_ip = c.lip & 0x100u;
        g.kb_mac = c.lmac & 0x100u;
        g.kb_pip = c.pip & 0x100u;
    } else {
        g.kb_ip = ldg(tb.kbits + (size_t)KB_CIDR_BAD * tb.kb_words, c.lip >> 5);
        if constexpr ((V & VAR_SKIP_KB1) != 0) g.kb_mac = c.lmac & 0x100u;   // profiling only, wrong results
        else g.kb_mac = ldg(tb.kbits + (size_t)KB_MAC_BAD * tb.kb_words, c.lmac >> 5);
        g.kb_pip = ldg(tb.kbits + (size_t)KB_CIDR_BAD * tb.kb_words, c.pip >> 5);    // peer end (same / cross node)
    }
    if constexpr ((V & VAR_POD8) != 0) {              // profiling only: 8 B from the table's first half
        const u32x2 w = ldg(reinterpret_cast<const u32x2*>(tb.pod_direct), c.pp);
        g.slot = make_uint4(w.x, w.y, 0u, 0u);
    } else if constexpr ((V & VAR_SKIP_POD) == 0) {
        g.slot = pod_slot<(V & VAR_NT_POD) != 0>(tb, c.pp);
    }
}

template <int V>
KD_INLINE uint4 add_calc(const RecCols& c, const AddGath& g, const DevLinks& N, uint32_t j,
                         const TopoCtx& tc, const DevTables& tb, bool res, bool qd, uint32_t* q) {
    constexpr bool NTL = (V & VAR_NT_LOAD) != 0;
    if (qd) qdisc_from(tb, g.v, q);
    if (!res) return make_uint4(0u, 0u, 0u, 0u);
    const int32_t vni = vni_of(tb.vxlan_base, c.uid);
    uint32_t err = ((g.kb_ip >> (c.lip & 31)) & 1u) ? (uint32_t)KDTN_E_VETH_CIDR
                 : ((g.kb_mac >> (c.lmac & 31)) & 1u) ? (uint32_t)KDTN_E_VETH_MAC : 0u;   // :327
    uint32_t kind = 0, peer = 0xFFFFFFFFu, vtep = 0, hit = 0, rerr = 0;
    const bool pip_bad = (g.kb_pip >> (c.pip & 31)) & 1u;
    if (!err) {
        // Reference order: localhost (:333), "physical/" prefix (:348), getPod (:375). The
        // lookup is pure, so it was started first: a hit carries the PHYSICAL bit of the
        // pod's name, only a miss reads the key-string bitset.
        const bool lh = c.pp == tb.special[SPECIAL_LOCALHOST];
        uint2 p = make_uint2(0xFFFFFFFFu, 0u);
        if constexpr ((V & VAR_SKIP_POD) != 0) p = make_uint2(c.pp & POD_INDEX, g.lns);   // profiling only
        else if constexpr ((V & VAR_POD8) != 0) {                                          // profiling only
            asm volatile("" ::"v"(g.slot.x), "v"(g.slot.y));
            p = make_uint2(c.pp & POD_INDEX, g.lns);
        }
        else if (!lh) p = pod_resolve(tb, g.lns, c.pp, g.slot);
        const bool miss = p.x == 0xFFFFFFFFu;
        if (lh) {
            kind = KDTN_KIND_MACVLAN;                                                     // :333
        } else if (miss ? kbit(tb, KB_PHYSICAL, c.pp) : (p.x & POD_PHYSICAL) != 0) {
            kind = KDTN_KIND_PHYSICAL;                                                    // :348
            vtep = c.pp;
            const uint32_t nsx = vni_lookup(tb, tc.src, vni);                           // :177-179
            hit = (nsx != 0xFFFFFFFFu && nsx != tc.netns);
        } else if (miss) {
            err = KDTN_E_PEER_LOOKUP;                                                     // :375-379
        } else {
            peer = p.x & POD_INDEX;
            const uint32_t p_src = p.y & 0x7FFFFFFFu;
            if (p.x & POD_SPEC_NIL) {
                err = KDTN_E_PEER_NO_LINKS;                                               // :380-384
            } else if (p_src == 0 || (p.y & 0x80000000u)) {
                kind = KDTN_KIND_PEER_DEAD;                                               // :386-395
            } else if (p_src == tc.src) {
                kind = KDTN_KIND_SAME_NODE;                                               // :399-418
                err = pip_bad ? (uint32_t)KDTN_E_PEER_VETH_CIDR                         // MakeVeth(peer) :402
                    : kbit(tb, KB_MAC_BAD, (V & VAR_PMAC_COLS) ? c.pmac : N.key_s<NTL>(KDTN_K_PEER_MAC, j))
                        ? (uint32_t)KDTN_E_PEER_VETH_MAC : 0u;
            } else {
                kind = KDTN_KIND_CROSS_NODE;                                              // :419-453
                vtep = p_src;
                // the peer daemon's Update parses IntfIp = link.PeerIp (vxlan.go:80-83, utils.go:45)
                if (pip_bad) rerr = KDTN_E_REMOTE_CIDR;
                if (tb.vni_mask) {                                       // remote Update check
                    const uint32_t nsx = vni_lookup(tb, p_src, vni);
                    hit = (nsx != 0xFFFFFFFFu && nsx != (ldg(tb.pods, peer).w & 0x7FFFFFFFu));
                }
            }
        }
    }
    return pack_res(peer, vni, vtep, kind, err, hit, rerr);
}

template <int V>
KD_INLINE void add_finish(const RecCols& c, const AddGath& g, const DevLinks& N, uint32_t j,
                          const TopoCtx& tc, const DevTables& tb, const RecOut& out, uint32_t e,
                          bool res, bool qd, uint32_t* q) {
    store_idx<V>(out.add_idx + e, j);
    const uint4 r = add_calc<V>(c, g, N, j, tc, tb, res, qd, q);
    if (res) store_res<V>(out.add_res + e, r);
    if (res && qd) out.add_qerr[e] = (uint8_t)(q[17] >> 16);
}

template <int V>
KD_INLINE void emit_add(const RecCols& c, const DevLinks& N, uint32_t j, const TopoCtx& tc,
                        const DevTables& tb, const RecOut& out, uint32_t e, bool res, bool qd,
                        uint32_t* q) {
    AddGath g;
    add_gather<V>(c, tc, tb, res, qd, g);
    add_finish<V>(c, g, N, j, tc, tb, out, e, res, qd, q);
}

// Store the 72-B qdisc structs of this wave's active lanes. Active lanes' output positions
// are consecutive in lane order (every emission path assigns positions by an exclusive
// count in record order), so the wave stages 32 structs at a time in LDS and writes them
// as contiguous 512-B bursts instead of nine 8-B stores at a 72-B stride per lane.
template <int V>
__device__ __forceinline__ void wave_store_qdisc(uint2* outq, bool active, uint32_t e,
                                                 const uint32_t* q, uint2* stage) {
    const uint64_t m = __ballot(active);
    if (m == 0) return;
    if constexpr ((V & VAR_NO_QSTORE) != 0) {
        if (active)
#pragma unroll
            for (int w = 0; w < 18; ++w) asm volatile("" ::"v"(q[w]));
        return;
    }
    const int lane = threadIdx.x & 63;
    const uint32_t p0 = __shfl(e, __ffsll((long long)m) - 1, 64);
    const uint32_t rank = __popcll(m & lanemask_lt());
    const uint32_t lo = __popcll(m & 0xFFFFFFFFull), all = __popcll(m);
#pragma unroll
    for (int half = 0; half < 2; ++half) {
        const uint32_t r0 = half ? lo : 0u, cnt = half ? all - lo : lo;
        if (cnt == 0) continue;
        if (active && ((lane >= 32) == (half == 1))) {
            uint2* slot = stage + (rank - r0) * 9;
#pragma unroll
            for (int w = 0; w < 9; ++w) slot[w] = make_uint2(q[2 * w], q[2 * w + 1]);
        }
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        uint2* dst = outq + (size_t)(p0 + r0) * 9;
        const uint32_t nq = cnt * 9;
        for (uint32_t k = lane; k < nq; k += 64) {
            if constexpr ((V & VAR_NT_STORE) != 0) {
                u32x2 v;
                v.x = stage[k].x;
                v.y = stage[k].y;
                __builtin_nontemporal_store(v, reinterpret_cast<u32x2*>(dst + k));
            } else {
                dst[k] = stage[k];
            }
        }
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    }
}

// (VAR_Q16) the wave's 64 structs staged at once and stored as 16-B words: the destination
// range starts 8-B aligned, so at most one leading and one trailing 8-B word go alone
template <int V>
__device__ __forceinline__ void wave_store_qdisc16(uint2* outq, bool active, uint32_t e, const uint32_t* q,
                                                   uint2* stage) {
    const uint64_t m = __ballot(active);
    if (m == 0) return;
    const int lane = threadIdx.x & 63;
    const uint32_t p0 = __shfl(e, __ffsll((long long)m) - 1, 64);
    const uint32_t rank = __popcll(m & lanemask_lt()), cnt = __popcll(m);
    if (active) {
        uint2* slot = stage + rank * 9;
#pragma unroll
        for (int w = 0; w < 9; ++w) slot[w] = make_uint2(q[2 * w], q[2 * w + 1]);
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    const size_t base = (size_t)p0 * 9;
    uint2* dst = outq + base;
    const uint32_t nq = cnt * 9, head = (uint32_t)(base & 1u), n16 = (nq - head) >> 1;
    if (head && lane == 0) store_q8<V>(dst, stage[0]);
    u32x4* d16 = reinterpret_cast<u32x4*>(dst + head);
    for (uint32_t k = lane; k < n16; k += 64) {
        const uint2 a = stage[head + 2 * k], b = stage[head + 2 * k + 1];
        u32x4 v;
        v.x = a.x;
        v.y = a.y;
        v.z = b.x;
        v.w = b.y;
        if constexpr ((V & VAR_NT_STORE) != 0) __builtin_nontemporal_store(v, d16 + k);
        else d16[k] = v;
    }
    if (((nq - head) & 1u) && lane == 0) store_q8<V>(dst + nq - 1, stage[nq - 1]);
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// ======================================================================================
// k_reconcile: one workgroup = TPW consecutive topologies (dynamic ticket order).
// ======================================================================================
struct RecShared {
    uint32_t ooff[TPW + 1];
    uint32_t noff[TPW + 1];
    uint8_t tflag[TPW];
    uint8_t dirty[TPW];
    uint8_t act[TPW];
    uint32_t ns[TPW], src[TPW], netns[TPW];
    uint32_t tcnt[3][TPW];       // per-topology counts (del, upd, add) → exclusive offsets
    uint32_t wsum[BLOCK / 64][4];
    uint32_t wtot[3];
    uint32_t base[3];
    uint32_t ticket;
    uint32_t any_cmp;
    uint32_t n_dense;
    union {
        struct {                  // comparison windows (gate + CalcDiff, fast-path emission)
            uint16_t rank[CAP];  // entry position within the workgroup's list
            uint16_t dense[CAP]; // fast path: the flagged records, in record order
            uint16_t tgt[CAP];   // upd target, relative to the workgroup's first desired record
            uint8_t flag[CAP];
            uint8_t lt[CAP];
            union {               // CalcDiff hashes, then (emission) per-wave qdisc staging
                uint32_t hash[CAP];
                uint2 stage[BLOCK / 64][32 * 9];
            };
        };
        struct {                  // (VAR_GLDS, profiling build) bulk emission: one link tile per wave
            uint32_t tiles[BLOCK / 64][KDTN_PROFILING ? GL_UNITS * TILE_RECS : 1];
            uint2 bstage[BLOCK / 64][32 * 9];
        };
        uint2 stage64[BLOCK / 64][64 * 9];   // (VAR_Q16) bulk emission: a wave's 64 qdisc structs
    };
};

// need element comparisons: both lists non-nil and non-empty
KD_INLINE bool need_cmp(const RecShared& s, int tt) {
    return (s.tflag[tt] & (KDTN_TOPO_STATUS_NIL | KDTN_TOPO_SPEC_NIL)) == 0 &&
           s.ooff[tt + 1] > s.ooff[tt] && s.noff[tt + 1] > s.noff[tt];
}

// Action of topology tt (topology_controller.go:77-88)
KD_INLINE uint8_t topo_action(const RecShared& s, int tt) {
    const uint8_t tf = s.tflag[tt];
    const bool st_nil = tf & KDTN_TOPO_STATUS_NIL, sp_nil = tf & KDTN_TOPO_SPEC_NIL;
    const uint32_t ko = s.ooff[tt + 1] - s.ooff[tt], kn = s.noff[tt + 1] - s.noff[tt];
    if (st_nil || sp_nil) return (st_nil && sp_nil) ? KDTN_ACT_SKIP : (st_nil ? KDTN_ACT_CREATED : KDTN_ACT_DIFF);
    return (ko == kn && !s.dirty[tt]) ? KDTN_ACT_SKIP : KDTN_ACT_DIFF;
}

// CalcDiff over the topologies [tb, te) of this workgroup as one window (records of the
// window: old part [0, no) then new part [no, no+nn)). hsh/flg are LDS (lt != nullptr,
// tgt16 valid) or global scratch (single topology; targets go to wk.otarget). Leaves the
// MASKED flag of every window record in flg and accumulates per-topology counts.
// TR (profiling trace build): phase timestamps into tr[6] (A done) and tr[7] (B done).
__device__ __forceinline__ void diff_window_tail(RecShared& s, int tb, int te, const DevLinks& N, const uint32_t* hsh, uint8_t* flg,
                                 const uint8_t* lt, uint32_t no, uint32_t nn, uint32_t tot, uint32_t wn0);

template <bool TR>
__device__ void diff_window(RecShared& s, int tb, int te, const DevLinks& O, const DevLinks& N,
                            uint32_t* hsh, uint8_t* flg, uint8_t* lt, uint16_t* tgt16,
                            uint32_t* otarget, uint32_t wn_base, unsigned long long* tr = nullptr) {
    const uint32_t wo0 = s.ooff[tb], wo1 = s.ooff[te];
    const uint32_t wn0 = s.noff[tb], wn1 = s.noff[te];
    const uint32_t no = wo1 - wo0, nn = wn1 - wn0, tot = no + nn;
    const int tid = threadIdx.x;

    // A. segment of every record; key hashes of the new records where comparisons are
    //    needed (an old record hashes its own key in B); new records' marks cleared
    for (uint32_t r = tid; r < tot; r += BLOCK) {
        const bool old = r < no;
        const uint32_t idx = old ? wo0 + r : wn0 + (r - no);
        int tt = tb;
        if (lt) {
            tt = find_seg(old ? s.ooff : s.noff, tb, te, idx);
            lt[r] = (uint8_t)tt;
        }
        if (!old) {
            if (need_cmp(s, tt)) {
                uint32_t k[KEYW];
                load_key(N, idx, k);
                hsh[r] = key_hash_w(k);
            }
            flg[r] = 0;
        }
    }
    __syncthreads();
    if constexpr (TR) {
        if (tid == 0) tr[6] = __builtin_amdgcn_s_memrealtime();
    }

    // B. old side: first key-equal new record (CalcDiff :289-303) + positional DeepEqual (:77).
    //    The old record and the new record at the same position (the common first match of
    //    an unchanged or edited link) are loaded together in one round trip (both coalesced:
    //    consecutive threads, consecutive records); the LDS key hashes find the first match
    //    when the positional record is not it, and any earlier duplicate key when it is.
    for (uint32_t r = tid; r < no; r += BLOCK) {
        const int tt = lt ? lt[r] : tb;
        uint8_t f = RF_DEL;
        if (need_cmp(s, tt)) {
            const uint32_t i = wo0 + r;
            const uint32_t os_ = s.ooff[tt], ns_ = s.noff[tt], ne_ = s.noff[tt + 1];
            const uint32_t jp = ns_ + (i - os_);
            const bool have_p = jp < ne_;
            uint32_t ki[KEYW], pi[PROPW], kj[KEYW], pj[PROPW];
            load_key(O, i, ki);
            load_props(O, i, pi);
            if (have_p) {
                load_key(N, jp, kj);
                load_props(N, jp, pj);
            }
            const uint32_t h = key_hash_w(ki);
            const bool pos_key = have_p && words_eq<KEYW>(ki, kj);
            const bool pos_eq = pos_key && words_eq<PROPW>(pi, pj);
            uint32_t first = 0xFFFFFFFFu;
            bool same_props = false;
            const uint32_t jend = pos_key ? jp : ne_;       // before jp: an earlier duplicate only
            for (uint32_t j = ns_; j < jend; ++j) {
                if (j == jp || hsh[no + (j - wn0)] != h) continue;
                uint32_t kx[KEYW], px[PROPW];
                load_key(N, j, kx);
                load_props(N, j, px);
                if (words_eq<KEYW>(ki, kx)) {
                    first = j;
                    same_props = words_eq<PROPW>(pi, px);
                    break;
                }
            }
            if (first == 0xFFFFFFFFu && pos_key) {
                first = jp;
                same_props = pos_eq;
            }
            if (first != 0xFFFFFFFFu) {
                flg[no + (first - wn0)] = RF_MATCHED;        // j is some old record's first match
                if (!same_props) {
                    f = RF_UPD;
                    if (tgt16) tgt16[r] = (uint16_t)(first - wn0);
                    else otarget[i] = first;
                } else {
                    f = 0;
                }
            }
            if (s.ooff[tt + 1] - os_ == ne_ - ns_ && !pos_eq) s.dirty[tt] = 1;
        }
        flg[r] = f;
    }
    __syncthreads();
    if constexpr (TR) {
        if (tid == 0) tr[7] = __builtin_amdgcn_s_memrealtime();
    }

    diff_window_tail(s, tb, te, N, hsh, flg, lt, no, nn, tot, wn0);
}

// Phases C-E of a CalcDiff window (both forms)
__device__ __forceinline__ void diff_window_tail(RecShared& s, int tb, int te, const DevLinks& N, const uint32_t* hsh, uint8_t* flg,
                                 const uint8_t* lt, uint32_t no, uint32_t nn, uint32_t tot, uint32_t wn0) {
    const int tid = threadIdx.x;
    // C. new side: any key-equal old record (CalcDiff :305-316). Key equality is an
    //    equivalence: j has one iff it is some old record's first match (marked in B) or
    //    equals an earlier marked new record of its topology (a duplicate key in spec).
    for (uint32_t r = tid; r < nn; r += BLOCK) {
        const int tt = lt ? lt[no + r] : tb;
        uint8_t f = RF_ADD;
        if (need_cmp(s, tt)) {
            if (flg[no + r] & RF_MATCHED) {
                f = 0;
            } else {
                const uint32_t j = wn0 + r;
                const uint32_t h = hsh[no + r];
                bool have = false;
                for (uint32_t j2 = s.noff[tt]; j2 < j && !have; ++j2) {
                    if (hsh[no + (j2 - wn0)] != h || !(flg[no + (j2 - wn0)] & RF_MATCHED)) continue;
                    uint32_t ka[KEYW], kb[KEYW];
                    load_key(N, j, ka);
                    load_key(N, j2, kb);
                    have = words_eq<KEYW>(ka, kb);
                }
                if (have) f = 0;
            }
        }
        flg[no + r] = f | (flg[no + r] & RF_MATCHED);    // other threads still read the mark
    }
    __syncthreads();

    // D. action per topology
    for (int tt = tb + tid; tt < te; tt += BLOCK) s.act[tt] = topo_action(s, tt);
    __syncthreads();

    // E. mask by action; per-topology counts
    for (uint32_t r = tid; r < tot; r += BLOCK) {
        const int tt = lt ? lt[r] : tb;
        uint8_t f = flg[r] & (RF_DEL | RF_UPD | RF_ADD);
        if (s.act[tt] != KDTN_ACT_DIFF) f = 0;
        flg[r] = f;
        if (f & RF_DEL) atomicAdd(&s.tcnt[0][tt], 1u);
        if (f & RF_UPD) atomicAdd(&s.tcnt[1][tt], 1u);
        if (f & RF_ADD) atomicAdd(&s.tcnt[2][tt], 1u);
    }
    __syncthreads();
}

// (VAR_AB) the LDS window with its first two phases merged: every old record is loaded with
// the new record at its position in ONE round trip (both keys and properties), both key hashes
// go to LDS and the positional key / DeepEqual bits to the old record's flag byte; new records
// past their topology's old count hash their own key. The scan phase then reads only LDS,
// loading keys (and properties on a key match) for a hash hit off the positional record.
// Saves the new records' separate key pass (a round trip and 36 B per new record).
template <bool TR>
__device__ void diff_window_ab(RecShared& s, int tb, int te, const DevLinks& O, const DevLinks& N, uint32_t* hsh,
                               uint8_t* flg, uint8_t* lt, uint16_t* tgt16, unsigned long long* tr = nullptr) {
    const uint32_t wo0 = s.ooff[tb], wo1 = s.ooff[te];
    const uint32_t wn0 = s.noff[tb], wn1 = s.noff[te];
    const uint32_t no = wo1 - wo0, nn = wn1 - wn0, tot = no + nn;
    const int tid = threadIdx.x;
    constexpr uint8_t POS_KEY = 1, POS_EQ = 2;

    // A. loads and hashes
    for (uint32_t r = tid; r < tot; r += BLOCK) {
        const bool old = r < no;
        const uint32_t idx = old ? wo0 + r : wn0 + (r - no);
        const int tt = find_seg(old ? s.ooff : s.noff, tb, te, idx);
        lt[r] = (uint8_t)tt;
        uint8_t f = 0;
        if (need_cmp(s, tt)) {
            const uint32_t os_ = s.ooff[tt], ns_ = s.noff[tt], ne_ = s.noff[tt + 1];
            const uint32_t ko = s.ooff[tt + 1] - os_;
            if (old) {
                const uint32_t jp = ns_ + (idx - os_);
                const bool have_p = jp < ne_;
                uint32_t ki[KEYW], pi[PROPW], kj[KEYW], pj[PROPW];
                load_key(O, idx, ki);
                load_props(O, idx, pi);
                if (have_p) {
                    load_key(N, jp, kj);
                    load_props(N, jp, pj);
                }
                hsh[r] = key_hash_w(ki);
                if (have_p) hsh[no + (jp - wn0)] = key_hash_w(kj);
                const bool pos_key = have_p && words_eq<KEYW>(ki, kj);
                const bool pos_eq = pos_key && words_eq<PROPW>(pi, pj);
                f = (pos_key ? POS_KEY : 0) | (pos_eq ? POS_EQ : 0);
                if (ko == ne_ - ns_ && !pos_eq) s.dirty[tt] = 1;
            } else if (idx - ns_ >= ko) {                    // no old record at its position
                uint32_t k[KEYW];
                load_key(N, idx, k);
                hsh[r] = key_hash_w(k);
            }
        }
        flg[r] = f;
    }
    __syncthreads();
    if constexpr (TR) {
        if (tid == 0) tr[6] = __builtin_amdgcn_s_memrealtime();
    }

    // B. old side: first key-equal new record (CalcDiff :289-303), from the LDS hashes
    for (uint32_t r = tid; r < no; r += BLOCK) {
        const int tt = lt[r];
        uint8_t f = RF_DEL;
        if (need_cmp(s, tt)) {
            const uint32_t i = wo0 + r;
            const uint32_t os_ = s.ooff[tt], ns_ = s.noff[tt], ne_ = s.noff[tt + 1];
            const uint32_t jp = ns_ + (i - os_);
            const uint8_t pb = flg[r];
            const bool pos_key = pb & POS_KEY, pos_eq = pb & POS_EQ;
            const uint32_t h = hsh[r];
            uint32_t first = 0xFFFFFFFFu;
            bool same_props = false;
            const uint32_t jend = pos_key ? jp : ne_;        // before jp: an earlier duplicate only
            for (uint32_t j = ns_; j < jend; ++j) {
                if (j == jp || hsh[no + (j - wn0)] != h) continue;
                uint32_t ki[KEYW], kx[KEYW], pi[PROPW], px[PROPW];   // one round trip per candidate
                load_key(O, i, ki);
                load_key(N, j, kx);
                load_props(O, i, pi);
                load_props(N, j, px);
                if (words_eq<KEYW>(ki, kx)) {
                    first = j;
                    same_props = words_eq<PROPW>(pi, px);
                    break;
                }
            }
            if (first == 0xFFFFFFFFu && pos_key) {
                first = jp;
                same_props = pos_eq;
            }
            if (first != 0xFFFFFFFFu) {
                flg[no + (first - wn0)] = RF_MATCHED;
                if (!same_props) {
                    f = RF_UPD;
                    tgt16[r] = (uint16_t)(first - wn0);
                } else {
                    f = 0;
                }
            }
        }
        flg[r] = f;
    }
    __syncthreads();
    if constexpr (TR) {
        if (tid == 0) tr[7] = __builtin_amdgcn_s_memrealtime();
    }
    diff_window_tail(s, tb, te, N, hsh, flg, lt, no, nn, tot, wn0);
}

// (VAR_HB) the LDS window with both sides' key hashes in the first phase (each record's 9 key
// words, two records per thread in flight), so the old side knows its first candidate before it
// loads anything: one round trip for the old record and that candidate (keys and properties),
// where the positional form loads the positional record first and an off-position first match
// (every record after a deleted link of its Topology) takes a second round trip. A hash that
// matches a different key (a collision) or a positional record other than the first match with
// the same hash (duplicate keys in spec) load more, rarely.
template <bool TR>
__device__ void diff_window_hb(RecShared& s, int tb, int te, const DevLinks& O, const DevLinks& N, uint32_t* hsh,
                               uint8_t* flg, uint8_t* lt, uint16_t* tgt16, uint32_t* otarget,
                               unsigned long long* tr = nullptr) {
    const uint32_t wo0 = s.ooff[tb], wo1 = s.ooff[te];
    const uint32_t wn0 = s.noff[tb], wn1 = s.noff[te];
    const uint32_t no = wo1 - wo0, nn = wn1 - wn0, tot = no + nn;
    const int tid = threadIdx.x;

    // A. segment and key hash of every record (old and new), two records per thread per step
    for (uint32_t r0 = tid; r0 < tot; r0 += 2 * BLOCK) {
        uint32_t k0[KEYW], k1[KEYW];
        bool c0 = false, c1 = false;
        const uint32_t r1 = r0 + BLOCK;
#pragma unroll
        for (int q = 0; q < 2; ++q) {
            const uint32_t r = q ? r1 : r0;
            if (r >= tot) continue;
            const bool old = r < no;
            const uint32_t idx = old ? wo0 + r : wn0 + (r - no);
            const int tt = find_seg(old ? s.ooff : s.noff, tb, te, idx);
            lt[r] = (uint8_t)tt;
            if (!old) flg[r] = 0;
            if (need_cmp(s, tt)) {
                if (q) { load_key(old ? O : N, idx, k1); c1 = true; }
                else { load_key(old ? O : N, idx, k0); c0 = true; }
            }
        }
        if (c0) hsh[r0] = key_hash_w(k0);
        if (c1) hsh[r1] = key_hash_w(k1);
    }
    __syncthreads();
    if constexpr (TR) {
        if (tid == 0) tr[6] = __builtin_amdgcn_s_memrealtime();
    }

    // B. old side: the first key-equal new record (CalcDiff :289-303) and the positional
    //    DeepEqual (:77), from the first hash candidate
    for (uint32_t r = tid; r < no; r += BLOCK) {
        const int tt = lt[r];
        uint8_t f = RF_DEL;
        if (need_cmp(s, tt)) {
            const uint32_t i = wo0 + r;
            const uint32_t os_ = s.ooff[tt], ns_ = s.noff[tt], ne_ = s.noff[tt + 1];
            const uint32_t jp = ns_ + (i - os_);
            const uint32_t h = hsh[r];
            uint32_t cand = 0xFFFFFFFFu;
            for (uint32_t j = ns_; j < ne_; ++j)
                if (hsh[no + (j - wn0)] == h) { cand = j; break; }
            const bool p_hash = jp < ne_ && hsh[no + (jp - wn0)] == h;
            uint32_t first = 0xFFFFFFFFu;
            bool same_props = false, pos_eq = false;
            if (cand != 0xFFFFFFFFu) {
                uint32_t ki[KEYW], pi[PROPW], kx[KEYW], px[PROPW];
                load_key(O, i, ki);
                load_props(O, i, pi);
                load_key(N, cand, kx);
                load_props(N, cand, px);
                uint32_t j = cand;
                for (;;) {                                     // (a second pass only on a collision)
                    if (words_eq<KEYW>(ki, kx)) {
                        first = j;
                        same_props = words_eq<PROPW>(pi, px);
                        break;
                    }
                    while (++j < ne_ && hsh[no + (j - wn0)] != h) {
                    }
                    if (j >= ne_) break;
                    load_key(N, j, kx);
                    load_props(N, j, px);
                }
                if (first == jp) {
                    pos_eq = same_props;
                } else if (p_hash) {                           // the positional record shares the hash
                    load_key(N, jp, kx);
                    load_props(N, jp, px);
                    pos_eq = words_eq<KEYW>(ki, kx) && words_eq<PROPW>(pi, px);
                }
            }
            if (first != 0xFFFFFFFFu) {
                flg[no + (first - wn0)] = RF_MATCHED;
                if (!same_props) {
                    f = RF_UPD;
                    if (tgt16) tgt16[r] = (uint16_t)(first - wn0);
                    else otarget[i] = first;
                } else {
                    f = 0;
                }
            }
            if (s.ooff[tt + 1] - os_ == ne_ - ns_ && !pos_eq) s.dirty[tt] = 1;
        }
        flg[r] = f;
    }
    __syncthreads();
    if constexpr (TR) {
        if (tid == 0) tr[7] = __builtin_amdgcn_s_memrealtime();
    }
    diff_window_tail(s, tb, te, N, hsh, flg, lt, no, nn, tot, wn0);
}

// Decoupled look-back over the workgroups' list counts (3 lists), one wave, 64
// predecessors per round trip. Granules are 8-byte {state:32 | count:32} words written and
// read at agent scope (sc1); the data is its own flag, so no fences are needed
// (MI355X_MICROARCH.md, Valid forms / R2 granules). state 1 = aggregate, 2 = inclusive.
KD_INLINE uint32_t wave_sum(uint32_t v) {
#pragma unroll
    for (int d = 32; d >= 1; d >>= 1) v += __shfl_xor(v, d, 64);
    return v;
}

KD_INLINE void publish_aggregate(const RecShared& s, const RecWork& wk, uint32_t wg, int lane) {
    __hip_atomic_store(wk.status + (size_t)wg * 3 + lane, ((wg == 0 ? 2ull : 1ull) << 32) | s.wtot[lane],
                       __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

__device__ void lookback(RecShared& s, const RecWork& wk, uint32_t wg) {
    const int tid = threadIdx.x;
    if (tid < 64) {
        const int lane = tid;
        unsigned long long* st = wk.status;
        if (lane < 3) publish_aggregate(s, wk, wg, lane);
        uint32_t pre[3] = {0u, 0u, 0u};
        if (wg > 0) {
            bool done[3] = {false, false, false};
            int64_t whi = (int64_t)wg - 1;
            uint32_t spins = 0;
            while (!(done[0] && done[1] && done[2])) {
                const int64_t w = whi - lane;
                uint64_t g[3] = {0, 0, 0};
                if (w >= 0) {
#pragma unroll
                    for (int c = 0; c < 3; ++c)
                        if (!done[c])
                            g[c] = __hip_atomic_load(st + (size_t)w * 3 + c, __ATOMIC_RELAXED,
                                                     __HIP_MEMORY_SCOPE_AGENT);
                }
                bool ready = true;
                int fi[3];
#pragma unroll
                for (int c = 0; c < 3; ++c) {
                    fi[c] = 64;
                    if (done[c]) continue;
                    const uint32_t state = (uint32_t)(g[c] >> 32);
                    const uint64_t inc = __ballot(w >= 0 && state == 2);
                    const uint64_t nrd = __ballot(w >= 0 && state == 0);
                    fi[c] = inc ? (__ffsll((long long)inc) - 1) : 64;
                    const uint64_t upto = fi[c] >= 63 ? ~0ull : ((2ull << fi[c]) - 1);   // lanes 0..fi
                    if (nrd & upto) ready = false;
                }
                if (!ready) {
                    if (++spins > (1u << 24)) {              // bounded spin: report, never hang
                        if (lane == 0) {
                            atomicOr(&wk.sync[SYNC_ERR], 1u);
                            if (wk.herr) *wk.herr = 1u;
                        }
                        break;
                    }
                    __builtin_amdgcn_s_sleep(2);
                    continue;
                }
#pragma unroll
                for (int c = 0; c < 3; ++c) {
                    if (done[c]) continue;
                    const uint32_t v = (w >= 0 && lane <= fi[c]) ? (uint32_t)g[c] : 0u;
                    pre[c] += wave_sum(v);
                    if (fi[c] < 64) done[c] = true;
                }
                whi -= 64;
            }
        }
        if (lane < 3) {
            const uint32_t p = lane == 0 ? pre[0] : (lane == 1 ? pre[1] : pre[2]);
            if (wg > 0)
                __hip_atomic_store(st + (size_t)wg * 3 + lane, (2ull << 32) | (p + s.wtot[lane]),
                                   __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            s.base[lane] = p;
        }
    }
    __syncthreads();
}

// First chunk (TPW topologies = one k_reconcile workgroup) holding a topology that does NOT
// emit every one of its records as an entry. A topology without element comparisons
// (a nil or empty side) emits all records when its action is DIFF (all old → DelLinks,
// all new → AddLinks) and none otherwise, so it is "full" iff DIFF or both lists are
// empty; a topology needing comparisons is conservatively not full. Chunks up to and
// including the first partial one know their batch bases from the record offsets alone.
KD_INLINE bool topo_partial(uint8_t tf, uint32_t ko, uint32_t kn) {
    const bool st_nil = tf & KDTN_TOPO_STATUS_NIL, sp_nil = tf & KDTN_TOPO_SPEC_NIL;
    const bool cmp = !st_nil && !sp_nil && ko > 0 && kn > 0;
    const bool empty = ko == 0 && kn == 0;
    // action (topology_controller.go:77-88) of a topology without comparisons
    const bool diff = (st_nil || sp_nil) ? (!st_nil && sp_nil) : !empty;
    return cmp || !(diff || empty);
}

// Four topologies per thread (16-B offset loads), grid-stride over the role's nb blocks of
// NT threads, one global atomicMax per block: an epoch of partial topologies (config 3) sent
// every wave's atomic to one address (133 µs). The result is stored inverted (atomicMax of
// ~chunk) so the zeroed sync header means "none".
template <int NT>
KD_INLINE void full_prefix_blocks(const DevTopos& T, uint32_t* first_partial_inv, uint32_t bid, uint32_t nb,
                                  uint32_t* bmin) {
    if (threadIdx.x == 0) *bmin = 0xFFFFFFFFu;
    __syncthreads();
    const uint32_t stride = nb * NT * 4;
    for (uint32_t base = bid * NT * 4; base < T.n; base += stride) {
        const uint32_t t0 = base + threadIdx.x * 4;
        uint32_t first = 0xFFFFFFFFu;                  // first partial topology of the four
        if (t0 + 4 <= T.n) {
            const uint4 ro = *reinterpret_cast<const uint4*>(T.real_off + t0);
            const uint4 dn = *reinterpret_cast<const uint4*>(T.des_off + t0);
            const uint32_t ro4 = T.real_off[t0 + 4], dn4 = T.des_off[t0 + 4];
            const uint32_t fl = *reinterpret_cast<const uint32_t*>(T.flags + t0);
            if (topo_partial(fl >> 24, ro4 - ro.w, dn4 - dn.w)) first = t0 + 3;
            if (topo_partial((fl >> 16) & 0xFF, ro.w - ro.z, dn.w - dn.z)) first = t0 + 2;
            if (topo_partial((fl >> 8) & 0xFF, ro.z - ro.y, dn.z - dn.y)) first = t0 + 1;
            if (topo_partial(fl & 0xFF, ro.y - ro.x, dn.y - dn.x)) first = t0;
        } else {
            for (uint32_t t = t0 + 3; t + 1 > t0; --t)
                if (t < T.n && topo_partial(T.flags[t], T.real_off[t + 1] - T.real_off[t],
                                            T.des_off[t + 1] - T.des_off[t]))
                    first = t;
        }
        const bool partial = first != 0xFFFFFFFFu;
        const uint64_t m = __ballot(partial);
        if (partial && (threadIdx.x & 63) == (uint32_t)(__ffsll((long long)m) - 1))
            atomicMin(bmin, first / TPW);               // lanes hold increasing topologies
        if (__syncthreads_or(m != 0)) break;         // later iterations only hold later chunks
    }
    if (threadIdx.x == 0 && *bmin != 0xFFFFFFFFu) atomicMax(first_partial_inv, ~*bmin);
}

__global__ void __launch_bounds__(FP_BLOCK) k_full_prefix(DevTopos T, uint32_t* first_partial_inv) {
    __shared__ uint32_t bmin;
    full_prefix_blocks<FP_BLOCK>(T, first_partial_inv, blockIdx.x, gridDim.x, &bmin);
}

// k_pod_direct_verify and k_full_prefix in one launch (independent work; one kernel boundary
// less per epoch): blocks [0, nbv) verify pods, the rest scan topologies.
template <int PER>
__global__ void __launch_bounds__(BLOCK) k_pod_verify_prefix(const uint4* pods, uint32_t total, uint4* slots,
                                                             uint32_t stamp, unsigned long long* ovf, uint32_t mask,
                                                             uint32_t nd, DevTopos T, uint32_t* first_partial_inv,
                                                             uint32_t nbv, uint32_t nr, uint32_t gathered) {
    __shared__ uint32_t bmin;
    if (blockIdx.x < nbv) {
        if constexpr (PER == 1) {
            const uint32_t t = blockIdx.x * BLOCK + threadIdx.x;
            if (t < total) pod_verify_one(pods, total, slots, stamp, ovf, mask, nd, pod_order(t, gathered, nr));
        } else {                                  // PER rows per thread: row loads, then slot owner words
            const uint32_t t0 = blockIdx.x * BLOCK * PER + threadIdx.x;
            uint32_t g[PER], own[PER];
            uint4 e[PER];
#pragma unroll
            for (int q = 0; q < PER; ++q) {
                const uint32_t t = t0 + q * BLOCK;
                g[q] = t < total ? pod_order(t, gathered, nr) : 0u;
                e[q] = t < total ? pods[g[q]] : make_uint4(0xFFFFFFFFu, 0u, 0u, 0u);
            }
#pragma unroll
            for (int q = 0; q < PER; ++q)
                own[q] = (e[q].x == 0xFFFFFFFFu || e[q].y >= nd) ? g[q] << 2
                         : reinterpret_cast<const uint32_t*>(slots + e[q].y)[1];
#pragma unroll
            for (int q = 0; q < PER; ++q)
                if ((own[q] >> 2) != g[q]) pod_verify_one(pods, total, slots, stamp, ovf, mask, nd, g[q]);
        }
        return;
    }
    full_prefix_blocks<BLOCK>(T, first_partial_inv, blockIdx.x - nbv, gridDim.x - nbv, &bmin);
}

template __global__ void k_pod_verify_prefix<1>(const uint4*, uint32_t, uint4*, uint32_t, unsigned long long*, uint32_t,
                                                uint32_t, DevTopos, uint32_t*, uint32_t, uint32_t, uint32_t);
template __global__ void k_pod_verify_prefix<4>(const uint4*, uint32_t, uint4*, uint32_t, unsigned long long*, uint32_t,
                                                uint32_t, DevTopos, uint32_t*, uint32_t, uint32_t, uint32_t);
#if KDTN_PROFILING
template __global__ void k_pod_verify_prefix<2>(const uint4*, uint32_t, uint4*, uint32_t, unsigned long long*, uint32_t,
                                                uint32_t, DevTopos, uint32_t*, uint32_t, uint32_t, uint32_t);
#endif
// ---- fused epoch front (one local rank: no exchange) -------------------------------------
// Two launches instead of five when the key-string parse is short (kdtn_epoch_run's rule):
// the pod tables' memory-bound work shares launches with the dictionary parses. With a long
// VALU-bound key parse (config 2, 12M strings) the sequence is faster (0.793 vs 0.804 ms); with
// a short one the launches were the cost (config-3 churn epochs 0.762 -> 0.741 ms, config 4
// 0.246 -> 0.240, config 1 0.223 -> 0.206; profiles/r06ad_fuse_churn.json, r06ae_fuse_ab.json).
// k_epoch_front: blocks [0, nbz) zero the sync header and look-back area; [nbz, nbz + nbs)
// fill this rank's pod-status rows and scatter each into its direct lookup slot (the row is
// computed from the topology table here, the "physical/" prefix of the name read from its
// bytes, so nothing waits for the parse); the rest parse the key strings (k_kdict_flags).
// Memory-bound blocks come first, so they are dispatched before the parse's.
__global__ void __launch_bounds__(BLOCK) k_epoch_front(uint4* sync, uint32_t n16, uint32_t nbz, uint32_t nbs,
                                                       DevTopos T, uint32_t slice, uint4* pods, uint4* slots,
                                                       uint32_t stamp, const uint8_t* kd_bytes,
                                                       const uint32_t* kd_offs, uint32_t k0, uint32_t D,
                                                       uint32_t* kbits, uint32_t kb_words, uint32_t* special) {
    const uint32_t b = blockIdx.x;
    if (b < nbz) {
        for (uint32_t i = b * BLOCK + threadIdx.x; i < n16; i += nbz * BLOCK) sync[i] = make_uint4(0u, 0u, 0u, 0u);
        return;
    }
    if (b < nbz + nbs) {
        const uint32_t t = (b - nbz) * BLOCK + threadIdx.x;
        if (t >= slice) return;
        pods_fill_one(T, slice, 0u, pods, t);
        if (t >= T.n) return;                                   // padding row
        const uint32_t name = T.name[t];
        if (name >= D) return;
        const uint32_t ob = kd_offs[name], len = kd_offs[name + 1] - ob;
        const uint32_t* p = reinterpret_cast<const uint32_t*>(kd_bytes + (ob & ~3u));
        const uint32_t d0 = p[0], d1 = p[1], d2 = p[2], d3 = p[3], sh = ob & 3u;
        const uint32_t w0 = __builtin_amdgcn_alignbyte(d1, d0, sh), w1 = __builtin_amdgcn_alignbyte(d2, d1, sh);
        const uint32_t w2 = __builtin_amdgcn_alignbyte(d3, d2, sh);
        const uint32_t phys = (len >= 9 && w0 == 0x73796870u && w1 == 0x6C616369u && (w2 & 0xFFu) == '/') ? 1u : 0u;
        const uint32_t netns = T.net_ns[t];
        const uint32_t nil = (T.flags[t] & KDTN_TOPO_SPEC_NIL) ? 1u : 0u;
        slots[name] = make_uint4(T.ns[t], (t << 2) | (phys << 1) | nil, T.src_ip[t] | (netns == 0 ? 0x80000000u : 0u),
                                 stamp << 1);
        return;
    }
    kdict_block(kd_bytes, kd_offs, k0 + (b - nbz - nbs) * BLOCK, D, kbits, kb_words, special);
}

// k_pdict_verify: blocks [0, nbv) verify the lookup slots (names shared by several pods →
// overflow table), [nbv, nbv + nbp) scan the topologies for the first partial chunk
// (k_full_prefix), the rest parse the property strings, interpretation (b - nbv - nbp) / nbd.
__global__ void __launch_bounds__(BLOCK) k_pdict_verify(const uint4* pods, uint32_t total, uint4* slots, uint32_t stamp,
                                                        unsigned long long* ovf, uint32_t mask, uint32_t nd,
                                                        DevTopos T, uint32_t* first_partial_inv, uint32_t nbv,
                                                        uint32_t nbp, const uint8_t* pbytes, const uint32_t* poffs,
                                                        uint32_t p0, uint32_t np, uint32_t nbd, double tick,
                                                        uint32_t* ppct, uint2* pdur, uint2* prate, uint32_t* rate_err) {
    __shared__ uint4 buf[STAGE / 16];
    const uint32_t b = blockIdx.x;
    if (b < nbv) {
        const uint32_t t = b * BLOCK + threadIdx.x;
        if (t < total) pod_verify_one(pods, total, slots, stamp, ovf, mask, nd, t);
        return;
    }
    if (b < nbv + nbp) {
        full_prefix_blocks<BLOCK>(T, first_partial_inv, b - nbv, nbp, reinterpret_cast<uint32_t*>(buf));
        return;
    }
    const uint32_t q = b - nbv - nbp, y = q / nbd, s0 = p0 + (q - y * nbd) * BLOCK;
    if (y == 0) pdict_parse_block<PD_PCT>(pbytes, poffs, s0, np, tick, ppct, pdur, prate, rate_err, buf);
    else if (y == 1) pdict_parse_block<PD_DUR>(pbytes, poffs, s0, np, tick, ppct, pdur, prate, rate_err, buf);
    else pdict_parse_block<PD_RATE>(pbytes, poffs, s0, np, tick, ppct, pdur, prate, rate_err, buf);
}

// (VAR_TRACE) phase timestamp of this workgroup: 100 MHz chip-wide clock
template <int V>
KD_INLINE void trace_mark(const RecWork& wk, uint32_t wg, int k, unsigned long long t0 = 0) {
    if constexpr ((V & VAR_TRACE) != 0) {
        if (threadIdx.x == 0) wk.trace[(size_t)wg * TRACE_WORDS + k] = t0 ? t0 : __builtin_amdgcn_s_memrealtime();
    }
}

// ---- VAR_GLDS: bulk emission from LDS-DMA'd link tiles ----------------------------------
// The records [rlo, rhi) of a bulk chunk (old part [0, no) then new part) as whole 64-record
// tiles of the two link stores: tile g of the list is old tile to0 + g (g < nto), else new tile
// tn0 + g - nto. A wave takes tiles wave, wave + 4, ...; lane l handles record 64 t + l.
struct GlPlan {
    uint32_t oa, ob, na, nb;          // old / new record ranges
    uint32_t to0, nto, tn0, nt;       // first tiles, old tile count, all tiles
};
KD_INLINE GlPlan gl_plan(uint32_t rlo, uint32_t rhi, uint32_t no, uint32_t o0, uint32_t n0) {
    GlPlan p;
    p.oa = o0 + min(rlo, no);
    p.ob = o0 + min(rhi, no);
    p.na = n0 + (max(rlo, no) - no);
    p.nb = n0 + (max(rhi, no) - no);
    p.to0 = p.oa >> 6;
    p.nto = p.ob > p.oa ? ((p.ob - 1) >> 6) - p.to0 + 1 : 0u;
    p.tn0 = p.na >> 6;
    p.nt = p.nto + (p.nb > p.na ? ((p.nb - 1) >> 6) - p.tn0 + 1 : 0u);
    return p;
}

// One 16-B piece per lane into this wave's LDS slot: lane l of the instruction writes bytes
// [16 l, 16 l + 16) after `dst` (wave-uniform); the source address is the lane's own.
template <bool NT>
KD_INLINE void glds16(const void* src, uint32_t* dst) {
    __builtin_amdgcn_global_load_lds((__attribute__((address_space(1))) void*)src,
                                     (__attribute__((address_space(3))) void*)dst, 16, 0, NT ? 2 : 0);
}

// Copy tile g of the plan into `slot`: an add tile as GL_UNITS column units (5 instructions of
// 64 pieces), a delete tile as 4 (local_ip, local_mac, uid; one instruction). A piece whose
// records all lie outside the plan's range (the chunk's edge tiles) is not copied.
template <bool NT>
KD_INLINE void gl_issue(const GlPlan& p, uint32_t g, const DevLinks& O, const DevLinks& N, uint32_t* slot,
                        int lane) {
    if (g >= p.nt) return;
    const bool old = g < p.nto;
    const uint32_t t = old ? p.to0 + g : p.tn0 + (g - p.nto);
    const uint32_t lo = old ? p.oa : p.na, hi = old ? p.ob : p.nb, t64 = t * 64u;
    const uint32_t rlo = lo > t64 ? lo - t64 : 0u, rhi = min(hi - t64, 64u);
    const uint8_t* tile = reinterpret_cast<const uint8_t*>((old ? O.base : N.base) + (size_t)t * TILE_WORDS);
    const int k = lane & 15;
    if (old) {
        const int u = lane >> 4;
        const uint32_t r0 = u < 2 ? k * 4 : (u - 2) * 32 + k * 2, r1 = r0 + (u < 2 ? 4 : 2);
        if (r0 < rhi && r1 > rlo) glds16<NT>(tile + gl_col_del(u) * 256 + k * 16, slot);
        return;
    }
#pragma unroll
    for (int i = 0; i < GL_UNITS / 4; ++i) {
        const int u = i * 4 + (lane >> 4);
        const uint32_t r0 = u < 18 ? k * 4 : (u - 18) * 32 + k * 2, r1 = r0 + (u < 18 ? 4 : 2);
        if (r0 < rhi && r1 > rlo) glds16<NT>(tile + gl_col(u) * 256 + k * 16, slot + i * 256);
    }
}

// This lane's record columns from the wave's tile slot
KD_INLINE void gl_cols(const uint32_t* slot, int lane, bool old, RecCols& c) {
    c.lip = slot[lane];
    c.lmac = slot[64 + lane];
    if (old) {
        c.uid = reinterpret_cast<const int64_t*>(slot + 2 * 64)[lane];
        return;
    }
    c.pip = slot[2 * 64 + lane];
    c.pmac = slot[3 * 64 + lane];
    c.pp = slot[4 * 64 + lane];
#pragma unroll
    for (int k = 0; k < KDTN_NPROP; ++k) c.prop[k] = slot[(5 + k) * 64 + lane];
    c.gap = slot[17 * 64 + lane];
    c.uid = reinterpret_cast<const int64_t*>(slot + 18 * 64)[lane];
}

template <int V>
__global__ void __launch_bounds__(BLOCK) __attribute__((amdgpu_waves_per_eu(var_waves(V))))
k_reconcile(DevTopos T, DevLinks O, DevLinks N, DevTables tb, RecOut out, RecWork wk) {
    __shared__ RecShared s;
    const int tid = threadIdx.x;
    unsigned long long t_entry = 0;
    if constexpr ((V & VAR_TRACE) != 0) t_entry = __builtin_amdgcn_s_memrealtime();
    constexpr bool kDefer = (V & VAR_DIFF) != 0;
    const uint32_t fpi = *wk.first_partial_inv;          // ~first partial chunk (0: none)
    // The chunk's topology rows, loaded for chunk blockIdx.x / split while fpi is in flight
    // (reloaded below in the rare ticket case).
    struct TopoRow { uint32_t ro, no, ns, src, netns; uint8_t fl; };
    auto load_rows = [&](uint32_t w, TopoRow& r) {
        const uint32_t t0_ = w * TPW;
        const int nt_ = (int)min((uint32_t)TPW, T.n - t0_);
        if (tid <= nt_) {
            r.ro = T.real_off[t0_ + tid];
            r.no = T.des_off[t0_ + tid];
        }
        if (tid < nt_) {
            r.fl = T.flags[t0_ + tid];
            r.ns = T.ns[t0_ + tid];
            r.src = T.src_ip[t0_ + tid];
            r.netns = T.net_ns[t0_ + tid];
        }
    };
    TopoRow row{};
    load_rows(blockIdx.x / wk.split, row);
    // A dynamic ticket (dispatch order) orders look-backs after scheduled predecessors. Without
    // look-backs — every chunk in the full prefix, or the comparison build, whose chunks past
    // it are deferred — the workgroup index serves and the single-address atomic (one per
    // workgroup) stays off every workgroup's critical path.
    const bool need_ticket = (V & VAR_NO_PREFIX) != 0 || (!kDefer && fpi != 0u);
    if (need_ticket) {
        if (tid == 0) s.ticket = atomicAdd(&wk.sync[SYNC_TICKET], 1u);
        __syncthreads();
    }
    const uint32_t tk = need_ticket ? s.ticket : blockIdx.x;
    // wk.split workgroups per chunk: part 0 does the chunk's work; in a bulk chunk of the full
    // prefix (bases known without predecessors) the parts share its records, so a small epoch
    // whose chunks hold many records does not leave most of the chip idle in a second round
    const uint32_t wg = tk / wk.split, part = tk - wg * wk.split;
    if (need_ticket && wg != blockIdx.x / wk.split) load_rows(wg, row);
    if constexpr ((V & VAR_TRACE) != 0) {
        trace_mark<V>(wk, wg, 0, t_entry);
        uint32_t xcc, hw;
        asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
        asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(hw));
        if (tid == 0) wk.trace[(size_t)wg * TRACE_WORDS + 5] = ((unsigned long long)xcc << 32) | hw;
    }
    const uint32_t t0 = wg * TPW;
    const int nt = (int)min((uint32_t)TPW, T.n - t0);
    if (tid <= nt) {
        s.ooff[tid] = row.ro;
        s.noff[tid] = row.no;
    }
    if (tid < nt) {
        s.tflag[tid] = row.fl;
        s.dirty[tid] = 0;
        s.ns[tid] = row.ns;
        s.src[tid] = row.src;
        s.netns[tid] = row.netns;
    }
    if (tid < TPW) {
        s.tcnt[0][tid] = 0;
        s.tcnt[1][tid] = 0;
        s.tcnt[2][tid] = 0;
    }
    __syncthreads();
    trace_mark<V>(wk, wg, 1);
    const uint32_t o0 = s.ooff[0], o1 = s.ooff[nt], n0 = s.noff[0], n1 = s.noff[nt];
    const uint32_t no = o1 - o0, nn = n1 - n0, tot = no + nn;
    const bool fast = tot <= (uint32_t)CAP;
    const bool do_res = out.stages & KDTN_STAGE_RESOLVE;
    const bool do_q = out.stages & KDTN_STAGE_QDISC;
    // (VAR_PREFETCH) the thread's first bulk record's columns, issued before the gate, count
    // and base phases (speculatively: the records a shared bulk chunk gives this part)
    RecCols pre;
    uint32_t pre_r = 0xFFFFFFFFu;
    if constexpr ((V & VAR_PREFETCH) != 0 && !kDefer) {
        const uint32_t per_s = (tot + wk.split - 1) / wk.split;
        const uint32_t lo_s = min(tot, part * per_s), r = lo_s + tid;
        if (r < min(tot, lo_s + per_s)) {
            const bool old = r < no;
            load_cols<(V & VAR_NT_LOAD) != 0>(old ? O : N, old ? o0 + r : n0 + (r - no), do_res, !old && do_q, pre);
            pre_r = r;
        }
    }
    if (tid < 64) {
        const uint64_t b = __ballot(tid < nt && need_cmp(s, tid));
        if (tid == 0) s.any_cmp = b != 0ull;
    }
    __syncthreads();
    // bulk: no topology of this workgroup has both lists non-empty (new pods: status empty;
    // deleted pods: spec nil) → every record of a DIFF topology is an entry, in order
    const bool bulk = s.any_cmp == 0;
    const bool prefix = (V & VAR_NO_PREFIX) == 0 && wg <= ~fpi;
    const bool shared = bulk && prefix;                  // the parts split the records
    if (part != 0 && !shared) return;                    // (block-uniform)
    const bool lead = part == 0;
    const uint32_t per = shared ? (tot + wk.split - 1) / wk.split : tot;
    const uint32_t rlo = min(tot, part * per), rhi = min(tot, rlo + per);

    // ---- 1. Reconcile gate + CalcDiff ------------------------------------------------
    if (bulk) {
        if (tid < nt) {
            const uint8_t a = topo_action(s, tid);
            s.act[tid] = a;
            const bool d = a == KDTN_ACT_DIFF;
            s.tcnt[0][tid] = d ? s.ooff[tid + 1] - s.ooff[tid] : 0u;
            s.tcnt[2][tid] = d ? s.noff[tid + 1] - s.noff[tid] : 0u;
        }
        __syncthreads();
    } else if (fast) {
        if constexpr ((V & VAR_HB) != 0) {
            if constexpr ((V & VAR_TRACE) != 0)
                diff_window_hb<true>(s, 0, nt, O, N, s.hash, s.flag, s.lt, s.tgt, wk.otarget,
                                     wk.trace + (size_t)wg * TRACE_WORDS);
            else
                diff_window_hb<false>(s, 0, nt, O, N, s.hash, s.flag, s.lt, s.tgt, wk.otarget);
        } else if constexpr ((V & VAR_AB) != 0) {
            if constexpr ((V & VAR_TRACE) != 0)
                diff_window_ab<true>(s, 0, nt, O, N, s.hash, s.flag, s.lt, s.tgt, wk.trace + (size_t)wg * TRACE_WORDS);
            else
                diff_window_ab<false>(s, 0, nt, O, N, s.hash, s.flag, s.lt, s.tgt);
        } else if constexpr ((V & VAR_TRACE) != 0) {
            diff_window<true>(s, 0, nt, O, N, s.hash, s.flag, s.lt, s.tgt, wk.otarget, n0, wk.trace + (size_t)wg * TRACE_WORDS);
        } else {
            diff_window<false>(s, 0, nt, O, N, s.hash, s.flag, s.lt, s.tgt, wk.otarget, n0);
        }
    } else {
        // the chunk's records exceed one window: consecutive topologies are grouped into LDS
        // windows of up to CAP records (a chunk of 64 fat-tree spines of ~100 records takes 4
        // windows, not 64); a topology larger than CAP alone uses global scratch
        auto recs = [&](int t) { return (s.ooff[t + 1] - s.ooff[t]) + (s.noff[t + 1] - s.noff[t]); };
        int tt = 0;
        while (tt < nt) {                                   // (workgroup-uniform)
            uint32_t k = recs(tt);
            if (k > (uint32_t)CAP) {
                const uint32_t gofs = s.ooff[tt] + s.noff[tt];
                diff_window<false>(s, tt, tt + 1, O, N, wk.hscratch + gofs, wk.fscratch + gofs, nullptr,
                            nullptr, wk.otarget, 0);
                ++tt;
                continue;
            }
            int te = tt + 1;
            while (te < nt && k + recs(te) <= (uint32_t)CAP) k += recs(te++);
            if constexpr ((V & VAR_HB) != 0)
                diff_window_hb<false>(s, tt, te, O, N, s.hash, s.flag, s.lt, nullptr, wk.otarget);
            else
                diff_window<false>(s, tt, te, O, N, s.hash, s.flag, s.lt, nullptr, wk.otarget, 0);
            // spill the window's masked flags to each topology's global scratch slots (the
            // slow-path emission reads them: old records, then new records, per topology)
            const uint32_t wo0 = s.ooff[tt], wn0 = s.noff[tt], no_w = s.ooff[te] - wo0;
            for (uint32_t r = tid; r < k; r += BLOCK) {
                const int t2 = s.lt[r];
                const uint32_t pos = r < no_w ? wo0 + r - s.ooff[t2]
                                              : (s.ooff[t2 + 1] - s.ooff[t2]) + (wn0 + (r - no_w) - s.noff[t2]);
                wk.fscratch[s.ooff[t2] + s.noff[t2] + pos] = s.flag[r];
            }
            __syncthreads();
            tt = te;
        }
    }

    // ---- 2. per-topology exclusive offsets within the workgroup, list totals -----------
    if (tid < 64) {
        const int tt = tid;
        for (int c = 0; c < 3; ++c) {
            const uint32_t x = (tt < nt) ? s.tcnt[c][tt] : 0u;
            uint32_t v = x;
            for (int d = 1; d < 64; d <<= 1) {
                const uint32_t o = __shfl_up(v, d, 64);
                if (tt >= d) v += o;
            }
            s.tcnt[c][tt] = v - x;                   // exclusive
            if (tt == 63) s.wtot[c] = v;
        }
    }
    // ranks of flagged records within the workgroup's lists (fast path)
    if (fast && !bulk) {
        const uint32_t per = (tot + BLOCK - 1) / BLOCK;
        const uint32_t r0 = min(tot, tid * per), r1 = min(tot, r0 + per);
        uint32_t c[4] = {0, 0, 0, 0};                 // del, upd, add, any (dense list)
        for (uint32_t r = r0; r < r1; ++r) {
            const uint8_t f = s.flag[r];
            c[0] += (f & RF_DEL) ? 1u : 0u;
            c[1] += (f & RF_UPD) ? 1u : 0u;
            c[2] += (f & RF_ADD) ? 1u : 0u;
            c[3] += f ? 1u : 0u;
        }
        const int lane = tid & 63, wave = tid >> 6;
        uint32_t ex[4];
        for (int k = 0; k < 4; ++k) {
            uint32_t v = c[k];
            for (int d = 1; d < 64; d <<= 1) {
                const uint32_t o = __shfl_up(v, d, 64);
                if (lane >= d) v += o;
            }
            ex[k] = v - c[k];
            if (lane == 63) s.wsum[wave][k] = v;
        }
        __syncthreads();
        for (int k = 0; k < 4; ++k)
            for (int w = 0; w < wave; ++w) ex[k] += s.wsum[w][k];
        if (tid == BLOCK - 1) s.n_dense = ex[3] + c[3];
        for (uint32_t r = r0; r < r1; ++r) {
            const uint8_t f = s.flag[r];
            if (f) s.dense[ex[3]++] = (uint16_t)r;
            if (f & RF_DEL) s.rank[r] = (uint16_t)ex[0]++;
            else if (f & RF_UPD) s.rank[r] = (uint16_t)ex[1]++;
            else if (f & RF_ADD) s.rank[r] = (uint16_t)ex[2]++;
        }
    }
    __syncthreads();

    // ---- 3. batch bases: decoupled look-back -------------------------------------------
    trace_mark<V>(wk, wg, 2);
    constexpr bool NTL = (V & VAR_NT_LOAD) != 0;
    // Every topology before this workgroup's chunk emits all of its records (bulk DIFF:
    // k_full_prefix found no earlier exception): the batch bases are the record offsets of
    // the chunk, known without waiting on the predecessors. The inclusive prefix is
    // published at once so that later workgroups' look-backs stop here.
    // Comparison build: a chunk behind the full prefix does not wait for its predecessors'
    // windows. It emits at record-offset bases into the upper halves of the output arrays
    // (every list of a chunk holds at most as many entries as its records), and k_place moves
    // the entries down once k_place_scan has summed the workgroup counts.
    const bool deferred = kDefer && !prefix;
    if constexpr (kDefer) {
        if (lead && tid < 3) wk.wcount[(size_t)wg * 3 + tid] = s.wtot[tid];
    }
    if (prefix) {
        if (lead && tid < 3) {
            const uint32_t p = tid == 0 ? s.ooff[0] : (tid == 1 ? 0u : s.noff[0]);
            __hip_atomic_store(wk.status + (size_t)wg * 3 + tid, (2ull << 32) | (p + s.wtot[tid]),
                               __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
        if (tid < 3) s.base[tid] = tid == 0 ? s.ooff[0] : (tid == 1 ? 0u : s.noff[0]);
        __syncthreads();
    } else if (deferred) {
        if (tid < 3) s.base[tid] = tid == 2 ? wk.n_cap + s.noff[0] : wk.m_cap + s.ooff[0];
        __syncthreads();
    } else {
        lookback(s, wk, wg);
    }
    trace_mark<V>(wk, wg, 3);
    const uint32_t bd = s.base[0], bu = s.base[1], ba = s.base[2];
    if (!kDefer && lead && wg == wk.nwg - 1 && tid < 3) {             // comparison build: k_place_scan
        const uint32_t total = s.base[tid] + s.wtot[tid];
        out.totals[tid] = total;
        if (out.htotals) out.htotals[tid] = total;
        (tid == 0 ? out.del_off : tid == 1 ? out.upd_off : out.add_off)[T.n] = total;
    }
    if (lead && tid < nt) {
        out.action[t0 + tid] = s.act[tid];
        out.del_off[t0 + tid] = (deferred ? 0u : bd) + s.tcnt[0][tid];   // k_place adds the base
        out.upd_off[t0 + tid] = (deferred ? 0u : bu) + s.tcnt[1][tid];
        out.add_off[t0 + tid] = (deferred ? 0u : ba) + s.tcnt[2][tid];
    }

    // ---- 4. emission -------------------------------------------------------------------
    uint2* stage = s.stage[tid >> 6];
    if constexpr ((V & VAR_GLDS) != 0 && !kDefer) {
        if (bulk) {
            // Bulk emission from LDS-DMA'd tiles: the wave's tile is read from its slot, the
            // record's gathers are issued, then the wave's next tile is copied into the slot
            // (its reads have retired) while the gathers are in flight.
            const int wave = tid >> 6, lane = tid & 63;
            GlPlan pl = gl_plan(rlo, rhi, no, o0, n0);
            // the plan in VGPRs: the emission's scalar registers hold the table bases
            asm volatile("" : "+v"(pl.oa), "+v"(pl.ob), "+v"(pl.na), "+v"(pl.nb), "+v"(pl.to0), "+v"(pl.tn0));
            uint32_t* slot = s.tiles[wave];
            uint2* bst = s.bstage[wave];
            gl_issue<NTL>(pl, (uint32_t)wave, O, N, slot, lane);
            for (uint32_t g = wave; g < pl.nt; g += BLOCK / 64) {
                asm volatile("s_waitcnt vmcnt(0)" ::: "memory");            // the tile has landed
                const bool old = g < pl.nto;
                const uint32_t t = old ? pl.to0 + g : pl.tn0 + (g - pl.nto);
                const uint32_t x = t * 64u + lane;
                const bool in = old ? (x >= pl.oa && x < pl.ob) : (x >= pl.na && x < pl.nb);
                int tt = 0;
                bool on = false;
                if (in) {
                    tt = find_seg(old ? s.ooff : s.noff, 0, nt, x);
                    on = s.act[tt] == KDTN_ACT_DIFF;
                }
                RecCols cc;
                if (on) gl_cols(slot, lane, old, cc);
                asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");          // slot reads retired
                bool qa = false;
                uint32_t e = 0, q[18];
                const TopoCtx tc{s.ns[tt], s.src[tt], s.netns[tt]};
                if (old) {
                    gl_issue<NTL>(pl, g + BLOCK / 64, O, N, slot, lane);
                    if (on) emit_del<V>(cc, x, tc, tb, out, bd + s.tcnt[0][tt] + (x - s.ooff[tt]), do_res);
                } else {
                    AddGath ga;
                    if (on) add_gather<V>(cc, tc, tb, do_res, do_q, ga);
                    gl_issue<NTL>(pl, g + BLOCK / 64, O, N, slot, lane);
                    if (on) {
                        e = ba + s.tcnt[2][tt] + (x - s.noff[tt]);
                        add_finish<V | VAR_PMAC_COLS>(cc, ga, N, x, tc, tb, out, e, do_res, do_q, q);
                        qa = do_q;
                    }
                }
                wave_store_qdisc<V>(out.add_qdisc, qa, e, q, bst);
            }
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            trace_mark<V>(wk, wg, 4);
            return;
        }
    }
    if (bulk) {
        // Every record of a DIFF topology is an entry at topology offset + index. Software
        // pipelined: a thread's next record's columns are loaded right after this record's
        // gathers are issued, so a wave has both in flight.
        struct Slot { uint32_t x; int tt; bool old, on; };
        auto decode = [&](uint32_t r) {
            Slot sl{0u, 0, false, false};
            if (r < rhi) {
                sl.old = r < no;
                sl.x = sl.old ? o0 + r : n0 + (r - no);
                sl.tt = find_seg(sl.old ? s.ooff : s.noff, 0, nt, sl.x);
                sl.on = s.act[sl.tt] == KDTN_ACT_DIFF;
            }
            return sl;
        };
        auto fetch = [&](const Slot& sl, RecCols& c) {
            if (sl.on) load_cols<NTL>(sl.old ? O : N, sl.x, do_res, !sl.old && do_q, c);
        };
        if constexpr ((V & VAR_DIFF) != 0) {
            // comparison-heavy build: one record at a time (fewer registers, more waves)
            for (uint32_t b = rlo; b < rhi; b += BLOCK) {
                const Slot cs = decode(b + tid);
                bool qa = false;
                uint32_t e = 0, q[18];
                if (cs.on) {
                    const int tt = cs.tt;
                    const TopoCtx tc{s.ns[tt], s.src[tt], s.netns[tt]};
                    RecCols cc;
                    fetch(cs, cc);
                    if (cs.old) {
                        emit_del<V>(cc, cs.x, tc, tb, out, bd + s.tcnt[0][tt] + (cs.x - s.ooff[tt]), do_res);
                    } else {
                        e = ba + s.tcnt[2][tt] + (cs.x - s.noff[tt]);
                        emit_add<V>(cc, N, cs.x, tc, tb, out, e, do_res, do_q, q);
                        qa = do_q;
                    }
                }
                wave_store_qdisc<V>(out.add_qdisc, qa, e, q, stage);
            }
            trace_mark<V>(wk, wg, 4);
            return;
        }
        Slot cs = decode(rlo + tid);
        RecCols cc;
        if (pre_r == rlo + tid && cs.on) cc = pre;
        else fetch(cs, cc);
        for (uint32_t b = rlo; b < rhi; b += BLOCK) {
            // the next record's segment search (LDS) runs after this record's gathers issue
            Slot nx;
            if constexpr ((V & VAR_DECODE_FIRST) != 0) nx = decode(b + BLOCK + tid);
            auto next = [&]() {
                if constexpr ((V & VAR_DECODE_FIRST) == 0) nx = decode(b + BLOCK + tid);
            };
            RecCols nc;
            bool qa = false;
            uint32_t e = 0, q[18];
            if (cs.on) {
                const int tt = cs.tt;
                const TopoCtx tc{s.ns[tt], s.src[tt], s.netns[tt]};
                if (cs.old) {
                    next();
                    fetch(nx, nc);
                    emit_del<V>(cc, cs.x, tc, tb, out, bd + s.tcnt[0][tt] + (cs.x - s.ooff[tt]), do_res);
                } else {
                    e = ba + s.tcnt[2][tt] + (cs.x - s.noff[tt]);
                    AddGath g;
                    add_gather<V>(cc, tc, tb, do_res, do_q, g);
                    next();
                    fetch(nx, nc);
                    add_finish<V>(cc, g, N, cs.x, tc, tb, out, e, do_res, do_q, q);
                    qa = do_q;
                }
            } else {
                next();
                fetch(nx, nc);
            }
            if constexpr ((V & VAR_Q16) != 0) wave_store_qdisc16<V>(out.add_qdisc, qa, e, q, s.stage64[tid >> 6]);
            else wave_store_qdisc<V>(out.add_qdisc, qa, e, q, stage);
            cs = nx;
            cc = nc;
        }
        trace_mark<V>(wk, wg, 4);
        return;
    }
    if (fast) {
        // only the flagged records, densely (a churn epoch flags a few % of them): one pass
        // of dependent loads per BLOCK flagged records instead of per BLOCK records
        const uint32_t nd = s.n_dense;
        for (uint32_t b = 0; b < nd; b += BLOCK) {           // no workgroup barriers
            const uint32_t r = b + tid < nd ? s.dense[b + tid] : 0u;
            bool qa = false, qu = false;
            uint32_t e = 0, q[18];
            const uint8_t f = b + tid < nd ? s.flag[r] : 0;
            if (f) {
                const int tt = s.lt[r];
                const TopoCtx tc{s.ns[tt], s.src[tt], s.netns[tt]};
                RecCols c;
                if (f & RF_DEL) {
                    load_cols<NTL>(O, o0 + r, do_res, false, c);
                    emit_del<V>(c, o0 + r, tc, tb, out, bd + s.rank[r], do_res);
                } else if (f & RF_UPD) {
                    e = bu + s.rank[r];
                    const uint32_t j = n0 + s.tgt[r];
                    load_cols<NTL>(N, j, do_res, do_q || do_res, c);
                    emit_upd<V>(c, j, tb, out, e, do_res, do_q, q);
                    qu = do_q;
                } else {
                    e = ba + s.rank[r];
                    const uint32_t j = n0 + (r - no);
                    load_cols<NTL>(N, j, do_res, do_q, c);
                    emit_add<V>(c, N, j, tc, tb, out, e, do_res, do_q, q);
                    qa = do_q;
                }
            }
            wave_store_qdisc<V>(out.add_qdisc, qa, e, q, stage);
            wave_store_qdisc<V>(out.upd_qdisc, qu, e, q, stage);
        }
        trace_mark<V>(wk, wg, 4);
        return;
    }
    // slow path: chunked, order-preserving compaction of the flags in global scratch
    uint32_t cd = 0, cu = 0, ca = 0;
    const int lane = tid & 63, wave = tid >> 6;
    for (int side = 0; side < 2; ++side) {
        const uint32_t lo = side ? n0 : o0, hi = side ? n1 : o1;
        for (uint32_t c = lo; c < hi; c += BLOCK) {
            const uint32_t x = c + tid;
            uint8_t f = 0;
            if (x < hi) {
                const uint32_t tt_ = find_seg(side ? s.noff : s.ooff, 0, nt, x);
                const uint32_t gofs = s.ooff[tt_] + s.noff[tt_];
                const uint32_t pos = side ? (s.ooff[tt_ + 1] - s.ooff[tt_]) + (x - s.noff[tt_]) : (x - s.ooff[tt_]);
                f = wk.fscratch[gofs + pos];
            }
            const uint64_t b0 = __ballot(f & RF_DEL), b1 = __ballot(f & RF_UPD), b2 = __ballot(f & RF_ADD);
            if (lane == 0) {
                s.wsum[wave][0] = __popcll(b0);
                s.wsum[wave][1] = __popcll(b1);
                s.wsum[wave][2] = __popcll(b2);
            }
            __syncthreads();
            uint32_t p0 = 0, p1 = 0, p2 = 0, t0_ = 0, t1_ = 0, t2_ = 0;
            for (int w = 0; w < BLOCK / 64; ++w) {
                if (w < wave) { p0 += s.wsum[w][0]; p1 += s.wsum[w][1]; p2 += s.wsum[w][2]; }
                t0_ += s.wsum[w][0];
                t1_ += s.wsum[w][1];
                t2_ += s.wsum[w][2];
            }
            const uint64_t lt = lanemask_lt();
            if (f) {
                const int tt = find_seg(side ? s.noff : s.ooff, 0, nt, x);
                const TopoCtx tc{s.ns[tt], s.src[tt], s.netns[tt]};
                uint32_t q[18];
                RecCols c;
                if (f & RF_DEL) {
                    load_cols<NTL>(O, x, do_res, false, c);
                    emit_del<V>(c, x, tc, tb, out, bd + cd + p0 + __popcll(b0 & lt), do_res);
                } else if (f & RF_UPD) {
                    const uint32_t e = bu + cu + p1 + __popcll(b1 & lt);
                    const uint32_t j = wk.otarget[x];
                    load_cols<NTL>(N, j, do_res, do_q || do_res, c);
                    emit_upd<V>(c, j, tb, out, e, do_res, do_q, q);
                    if (do_q) store_qdisc<V>(out.upd_qdisc + (size_t)e * 9, q);
                } else {
                    const uint32_t e = ba + ca + p2 + __popcll(b2 & lt);
                    load_cols<NTL>(N, x, do_res, do_q, c);
                    emit_add<V>(c, N, x, tc, tb, out, e, do_res, do_q, q);
                    if (do_q) store_qdisc<V>(out.add_qdisc + (size_t)e * 9, q);
                }
            }
            cd += t0_;
            cu += t1_;
            ca += t2_;
            __syncthreads();
        }
    }
    trace_mark<V>(wk, wg, 4);
}

// ---- VAR_DIFF placement -------------------------------------------------------------
// Exclusive bases of every workgroup's three lists (one block; nwg × 3 counts), the list
// totals and the closing offsets [T]. Tiles of PLACE_SCAN_BLOCK × PLACE_PER workgroups:
// each thread loads its PLACE_PER consecutive count triples with independent 16-B loads
// (one memory round trip per tile), scans them in registers, block-scans the thread sums.
__global__ void __launch_bounds__(PLACE_SCAN_BLOCK) k_place_scan(const uint32_t* wcount, uint32_t nwg,
                                                                 uint32_t* wbase, RecOut out, uint32_t T) {
    __shared__ uint32_t wsum[PLACE_SCAN_BLOCK / 64][3];
    __shared__ uint32_t carry[3];
    const uint32_t tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    if (tid < 3) carry[tid] = 0;
    constexpr uint32_t TILE = PLACE_SCAN_BLOCK * PLACE_PER;
    for (uint32_t t0 = 0; t0 < nwg; t0 += TILE) {
        const uint32_t w0 = t0 + tid * PLACE_PER;
        uint32_t v[PLACE_PER * 3];
        if (w0 + PLACE_PER <= nwg) {
            const uint4* src = reinterpret_cast<const uint4*>(wcount + (size_t)w0 * 3);
#pragma unroll
            for (int k = 0; k < PLACE_PER * 3 / 4; ++k) {
                const uint4 x = src[k];
                v[4 * k] = x.x;
                v[4 * k + 1] = x.y;
                v[4 * k + 2] = x.z;
                v[4 * k + 3] = x.w;
            }
        } else {
#pragma unroll
            for (int k = 0; k < PLACE_PER * 3; ++k)
                v[k] = w0 + k / 3 < nwg ? wcount[(size_t)w0 * 3 + k] : 0u;
        }
        uint32_t ex[3];
#pragma unroll
        for (int c = 0; c < 3; ++c) {
            uint32_t x = 0;
#pragma unroll
            for (int k = 0; k < PLACE_PER; ++k) x += v[3 * k + c];
            uint32_t sc = x;
            for (int d = 1; d < 64; d <<= 1) {
                const uint32_t o = __shfl_up(sc, d, 64);
                if (lane >= (uint32_t)d) sc += o;
            }
            ex[c] = sc - x;
            if (lane == 63) wsum[wave][c] = sc;
        }
        __syncthreads();
        uint32_t tot[3];
#pragma unroll
        for (int c = 0; c < 3; ++c) {
            uint32_t add = carry[c], all = 0;
            for (uint32_t w = 0; w < PLACE_SCAN_BLOCK / 64; ++w) {
                if (w < wave) add += wsum[w][c];
                all += wsum[w][c];
            }
            tot[c] = all;
            uint32_t run = ex[c] + add;
#pragma unroll
            for (int k = 0; k < PLACE_PER; ++k) {
                const uint32_t x = v[3 * k + c];
                v[3 * k + c] = run;                       // exclusive base, in place
                run += x;
            }
        }
        if (w0 + PLACE_PER <= nwg) {
            uint4* dst = reinterpret_cast<uint4*>(wbase + (size_t)w0 * 3);
#pragma unroll
            for (int k = 0; k < PLACE_PER * 3 / 4; ++k) dst[k] = make_uint4(v[4 * k], v[4 * k + 1], v[4 * k + 2], v[4 * k + 3]);
        } else {
#pragma unroll
            for (int k = 0; k < PLACE_PER * 3; ++k)
                if (w0 + k / 3 < nwg) wbase[(size_t)w0 * 3 + k] = v[k];
        }
        __syncthreads();                                  // wsum / carry reads done
        if (tid < 3) carry[tid] += tot[tid];
        __syncthreads();
    }
    if (tid < 3) {
        out.totals[tid] = carry[tid];
        if (out.htotals) out.htotals[tid] = carry[tid];
        (tid == 0 ? out.del_off : tid == 1 ? out.upd_off : out.add_off)[T] = carry[tid];
    }
}

// Deferred chunks: per-topology offsets += the chunk's bases, entries moved from [cap + record
// offset, +count) to [base, +count) of the same arrays (never overlapping), PLACE_U elements per
// thread loaded before any is stored (element by element, each store waited for its load). One
// wave per chunk when the chunks fill the chip (config 3: 15,625 chunks of ~32 entries), else
// `parts` workgroups per chunk (config 1: 157 chunks, a chunk of fat-tree spines moves 3,200
// 72-B records).
constexpr int PLACE_U = 4;
template <typename T>
KD_INLINE void place_move(T* dst, const T* src, uint32_t n, uint32_t me, uint32_t g) {
    for (uint32_t b = 0; b < n; b += g * PLACE_U) {
        T v[PLACE_U];
#pragma unroll
        for (int u = 0; u < PLACE_U; ++u) {
            const uint32_t k = b + u * g + me;
            if (k < n) v[u] = src[k];
        }
#pragma unroll
        for (int u = 0; u < PLACE_U; ++u) {
            const uint32_t k = b + u * g + me;
            if (k < n) __builtin_nontemporal_store(v[u], dst + k);
        }
    }
}
template <bool WAVE>
__global__ void __launch_bounds__(BLOCK) k_place(DevTopos T, const uint32_t* wcount, const uint32_t* wbase,
                                                 const uint32_t* first_partial_inv, RecOut out, uint32_t m_cap,
                                                 uint32_t n_cap, uint32_t nwg, uint32_t parts) {
    const uint32_t G = WAVE ? 64u : BLOCK * parts;                // threads per chunk
    const uint32_t wg = WAVE ? blockIdx.x * (BLOCK / 64) + (threadIdx.x >> 6) : blockIdx.x / parts;
    const uint32_t me = WAVE ? threadIdx.x & 63u : (blockIdx.x % parts) * BLOCK + threadIdx.x;
    if (wg >= nwg || wg <= ~*first_partial_inv) return;          // prefix chunks wrote final positions
    const uint32_t t0 = wg * TPW, nt = min((uint32_t)TPW, T.n - t0);
    const uint32_t cd = wcount[(size_t)wg * 3], cu = wcount[(size_t)wg * 3 + 1], ca = wcount[(size_t)wg * 3 + 2];
    const uint32_t bd = wbase[(size_t)wg * 3], bu = wbase[(size_t)wg * 3 + 1], ba = wbase[(size_t)wg * 3 + 2];
    if (me < nt) {
        out.del_off[t0 + me] += bd;
        out.upd_off[t0 + me] += bu;
        out.add_off[t0 + me] += ba;
    }
    const uint32_t sd = m_cap + T.real_off[t0], sa = n_cap + T.des_off[t0];
    const bool res = out.stages & KDTN_STAGE_RESOLVE, qd = out.stages & KDTN_STAGE_QDISC;
    typedef unsigned int u32x4v __attribute__((ext_vector_type(4)));
    typedef unsigned int u32x2v __attribute__((ext_vector_type(2)));
    place_move(out.del_idx + bd, out.del_idx + sd, cd, me, G);
    place_move(out.upd_idx + bu, out.upd_idx + sd, cu, me, G);
    place_move(out.add_idx + ba, out.add_idx + sa, ca, me, G);
    if (res) {
        place_move(reinterpret_cast<u32x4v*>(out.del_res + bd), reinterpret_cast<const u32x4v*>(out.del_res + sd), cd, me, G);
        place_move(reinterpret_cast<u32x4v*>(out.upd_res + bu), reinterpret_cast<const u32x4v*>(out.upd_res + sd), cu, me, G);
        place_move(reinterpret_cast<u32x4v*>(out.add_res + ba), reinterpret_cast<const u32x4v*>(out.add_res + sa), ca, me, G);
        if (qd) place_move(out.add_qerr + ba, out.add_qerr + sa, ca, me, G);
    }
    if (qd) {
        place_move(reinterpret_cast<u32x2v*>(out.upd_qdisc + (size_t)bu * 9),
                      reinterpret_cast<const u32x2v*>(out.upd_qdisc + (size_t)sd * 9), cu * 9, me, G);
        place_move(reinterpret_cast<u32x2v*>(out.add_qdisc + (size_t)ba * 9),
                      reinterpret_cast<const u32x2v*>(out.add_qdisc + (size_t)sa * 9), ca * 9, me, G);
    }
}
template __global__ void k_place<true>(DevTopos, const uint32_t*, const uint32_t*, const uint32_t*, RecOut, uint32_t,
                                       uint32_t, uint32_t, uint32_t);
template __global__ void k_place<false>(DevTopos, const uint32_t*, const uint32_t*, const uint32_t*, RecOut, uint32_t,
                                        uint32_t, uint32_t, uint32_t);

// Standalone MakeQdiscs over a batch of property sets (kdtn_make_qdiscs).
__global__ void __launch_bounds__(BLOCK) k_qdisc_batch(DevLinks props, DevTables tb, uint2* out) {
    const uint32_t j = blockIdx.x * BLOCK + threadIdx.x;
    if (j >= props.n) return;
    uint32_t q[18];
    RecCols c;
    load_cols<false>(props, j, false, true, c);
    PropVals v;
    gather_props<0>(c, tb, v);
    qdisc_from(tb, v, q);
    store_qdisc<0>(out + (size_t)j * 9, q);
}

template __global__ void k_reconcile<DEFAULT_VARIANT>(DevTopos, DevLinks, DevLinks, DevTables, RecOut, RecWork);
template __global__ void k_reconcile<DIFF_VARIANT>(DevTopos, DevLinks, DevLinks, DevTables, RecOut, RecWork);
#if KDTN_PROFILING
#define KDTN_VARIANT_INST(V) template __global__ void k_reconcile<V>(DevTopos, DevLinks, DevLinks, DevTables, RecOut, RecWork);
KDTN_PROFILING_VARIANTS(KDTN_VARIANT_INST)
#undef KDTN_VARIANT_INST
#endif

}  // namespace kdtn
