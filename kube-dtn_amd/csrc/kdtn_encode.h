// kdtn_encode.h — device helpers of the output stages (wire encoding, RemotePod messages,
// tc argv, fan-out, VXLAN ops): the wave-cooperative entry -> topology search, the
// dword-assembling byte writer and the wave-image stores. Kept apart from kdtn_kernels.h so the
// k_reconcile sources (whose hash tags its PMC profiles) do not change with them.
#pragma once
#include "kdtn_kernels.h"

namespace kdtn {

// entry_topo for every lane of a wave at once (all lanes must call it; on = the lane has an
// entry). The topologies of the wave's smallest and largest entry are found together by a
// 32-ary search (lanes 0-31 for one, 32-63 for the other; each step one load per lane and a
// ballot, so about log32(T) dependent loads instead of log2(T)); when the wave's entries span
// fewer than 64 topologies, one more load gives every lane the boundaries between them and a
// register search (shuffles) finds its own. A wave's entries are usually neighbours.
KD_INLINE uint32_t entry_topo_wave(const uint32_t* offs, uint32_t T, uint32_t e, bool on) {
    const int lane = threadIdx.x & 63;
    uint32_t lo_e = on ? e : 0xFFFFFFFFu, hi_e = on ? e : 0u;
#pragma unroll
    for (int d = 32; d >= 1; d >>= 1) {
        const uint32_t a = __shfl_xor(lo_e, d, 64), b = __shfl_xor(hi_e, d, 64);
        lo_e = a < lo_e ? a : lo_e;
        hi_e = b > hi_e ? b : hi_e;
    }
    if (lo_e > hi_e) return 0;                         // no lane has an entry (wave-uniform)
    // offs[lo] <= key < offs[hi] for key = lo_e (lanes 0-31) / hi_e (lanes 32-63)
    const uint32_t key = lane < 32 ? lo_e : hi_e, j = (uint32_t)lane & 31u;
    uint32_t lo = 0, hi = T;
    for (;;) {
        const bool open = hi - lo > 1;
        if (!__ballot(open)) break;                    // both searches done (wave-uniform)
        const uint32_t step = (hi - lo + 31u) >> 5;
        const uint32_t probe = lo + j * step;
        const bool ok = open && probe < hi && offs[probe] <= key;
        const uint64_t b = __ballot(ok);
        const uint32_t bh = (uint32_t)(lane < 32 ? b : (b >> 32));   // this half's probes, monotone
        if (open) {
            const uint32_t jj = 31u - (uint32_t)__clz((int)bh);       // last probe <= key (j = 0 always is)
            lo = lo + jj * step;
            hi = min(hi, lo + step);
        }
    }
    const uint32_t tlo = __shfl(lo, 0, 64), thi = __shfl(lo, 32, 64);   // topologies of lo_e, hi_e
    if (thi - tlo < 64u) {
        // boundary l: the first entry of topology tlo + 1 + l (lanes past thi: never <= e)
        const uint32_t bnd = tlo + 1u + (uint32_t)lane <= thi ? offs[tlo + 1u + lane] : 0xFFFFFFFFu;
        uint32_t c = 0;                                // boundaries <= e (a prefix of the lanes)
#pragma unroll
        for (int s = 32; s >= 1; s >>= 1) {
            const uint32_t v = __shfl(bnd, (int)(c + (uint32_t)s - 1u), 64);
            if (c + (uint32_t)s <= 64u && v <= e) c += (uint32_t)s;
        }
        return tlo + c;
    }
    lo = tlo;
    hi = thi + 1;                                      // offs[lo] <= e < offs[hi]
    while (hi - lo > 1) {
        const uint32_t mid = (lo + hi) >> 1;
        if (offs[mid] <= e) lo = mid;
        else hi = mid;
    }
    return lo;
}

// entry_topo_wave with a coarse index of the list (k_list_coarse: coarse[w] = topology of entry
// 64 w): the wave starts from the topology of its first entry's 64-entry group and finds every
// lane's topology with one load of the next 64 boundaries — two dependent loads instead of the
// search's four or five. Falls back to the search when the wave's entries reach past those 64
// topologies (empty topologies of the list in between).
KD_INLINE uint32_t entry_topo_wave_c(const uint32_t* offs, const uint32_t* coarse, uint32_t T, uint32_t e, bool on) {
    if (!coarse) return entry_topo_wave(offs, T, e, on);
    const int lane = threadIdx.x & 63;
    uint32_t lo_e = on ? e : 0xFFFFFFFFu, hi_e = on ? e : 0u;
#pragma unroll
    for (int d = 32; d >= 1; d >>= 1) {
        const uint32_t a = __shfl_xor(lo_e, d, 64), b = __shfl_xor(hi_e, d, 64);
        lo_e = a < lo_e ? a : lo_e;
        hi_e = b > hi_e ? b : hi_e;
    }
    if (lo_e > hi_e) return 0;                         // no lane has an entry (wave-uniform)
    const uint32_t tlo = coarse[lo_e >> 6];            // <= the topology of lo_e
    // boundary l: the first entry of topology tlo + 1 + l (past T: never <= e)
    const uint32_t bnd = tlo + 1u + (uint32_t)lane <= T ? offs[tlo + 1u + lane] : 0xFFFFFFFFu;
    if (hi_e >= __shfl(bnd, 63, 64)) return entry_topo_wave(offs, T, e, on);   // wave-uniform
    uint32_t c = 0;                                    // boundaries <= e (a prefix of the lanes)
#pragma unroll
    for (int s = 32; s >= 1; s >>= 1) {
        const uint32_t v = __shfl(bnd, (int)(c + (uint32_t)s - 1u), 64);
        if (c + (uint32_t)s <= 64u && v <= e) c += (uint32_t)s;
    }
    return tlo + c;
}

// ---- byte-stream writer of the encoders (wire, RemotePod, tc argv) ---------------------------
// Bytes are appended 1-4 at a time into a 64-bit register and stored as whole dwords; only the
// first and the last dword of a writer's range — shared with the neighbouring writers — take
// byte stores. (One dword store per 4 output bytes instead of one byte store per byte.)
struct WSink {
    uint32_t* d;                 // the dword acc's byte 0 belongs to
    uint32_t* d0;                // the writer's first dword
    uint64_t acc;                // pending bytes, little-endian
    uint32_t fill;               // bytes in acc, counting the `head` bytes of d0 that are not ours
    uint32_t head;               // bytes [0, head) of d0 belong to the previous writer
    uint32_t first;              // d0's bytes, stored by finish() when head != 0
    bool hp;                     // d0 not flushed yet and shared (head != 0)
    KD_INLINE void init(uint8_t* p) {
        const uint32_t mis = (uint32_t)(reinterpret_cast<uintptr_t>(p) & 3u);
        d = d0 = reinterpret_cast<uint32_t*>(p - mis);     // pointer arithmetic keeps the address space
        head = fill = mis;
        hp = mis != 0;
        acc = 0;
        first = 0;
    }
    // bytes [lo, hi) of v into dword q, one byte store each
    KD_INLINE static void part(uint32_t* q, uint32_t v, uint32_t lo, uint32_t hi) {
        uint8_t* b = reinterpret_cast<uint8_t*>(q);
#pragma unroll
        for (uint32_t k = 0; k < 4; ++k)
            if (k >= lo && k < hi) b[k] = (uint8_t)(v >> (8u * k));
    }
    // the low n (1..4) bytes of v
    KD_INLINE void put(uint32_t v, uint32_t n) {
        if (n < 4u) v &= (1u << (8u * n)) - 1u;
        acc |= (uint64_t)v << (8u * fill);
        fill += n;
        if (fill >= 4u) {
            if (hp) {
                first = (uint32_t)acc;
                hp = false;
            } else {
                *d = (uint32_t)acc;
            }
            ++d;
            acc >>= 32;
            fill -= 4u;
        }
    }
    KD_INLINE void finish() {
        if (head && !hp) part(d0, first, head, 4u);     // shared first dword, flushed
        if (fill) part(d, (uint32_t)acc, hp ? head : 0u, fill);
    }
    // bytes [b, b + len) of an arena with >= 40 B of readable slack past its end, 32 per round
    // (two 16-B loads and a dword, realigned by alignbyte)
    KD_INLINE void copy(const uint8_t* arena, uint64_t b, uint32_t len) {
        typedef uint32_t u32x4a __attribute__((ext_vector_type(4), aligned(4)));
        const uint32_t* a32 = reinterpret_cast<const uint32_t*>(arena + (b & ~3ull));
        const uint32_t sh = (uint32_t)b & 3u;
        for (uint32_t o = 0; o < len; o += 32u, a32 += 8) {
            const u32x4a A = *reinterpret_cast<const u32x4a*>(a32);
            const u32x4a B = *reinterpret_cast<const u32x4a*>(a32 + 4);
            const uint32_t w[9] = {A.x, A.y, A.z, A.w, B.x, B.y, B.z, B.w, a32[8]};
#pragma unroll
            for (uint32_t q = 0; q < 8; ++q) {
                if (o + 4u * q < len) {
                    const uint32_t r = len - o - 4u * q;
                    put(__builtin_amdgcn_alignbyte(w[q + 1], w[q], sh), r < 4u ? r : 4u);
                }
            }
        }
    }
    // owned mode: the writer owns every byte of its dwords (a private LDS slot); `lead` zero
    // bytes put the output at the alignment of its destination
    KD_INLINE void init_owned(uint32_t* slot, uint32_t lead) {
        d = d0 = slot;
        head = 0;
        fill = lead;
        hp = false;
        acc = 0;
        first = 0;
    }
    KD_INLINE void finish_owned() {
        if (fill) *d = (uint32_t)acc;
    }
    KD_INLINE void byte(uint32_t v) { put(v, 1u); }
    // protobuf base-128 varint: four 7-bit groups per put
    KD_INLINE void varint(uint64_t v) {
        while (v >= (1ull << 28)) {
            const uint32_t x = (uint32_t)v;
            put((x & 0x7Fu) | 0x80u | (((x >> 7) & 0x7Fu) | 0x80u) << 8 | (((x >> 14) & 0x7Fu) | 0x80u) << 16 |
                    (((x >> 21) & 0x7Fu) | 0x80u) << 24, 4u);
            v >>= 28;
        }
        const uint32_t x = (uint32_t)v;
        uint32_t w = x & 0x7Fu, n = 1;
        if (x >= 0x80u) { w |= 0x80u | ((x >> 7) & 0x7Fu) << 8; n = 2; }
        if (x >= 0x4000u) { w |= 0x8000u | ((x >> 14) & 0x7Fu) << 16; n = 3; }
        if (x >= 0x200000u) { w |= 0x800000u | ((x >> 21) & 0x7Fu) << 24; n = 4; }
        put(w, n);
    }
    // bytes [b, b + len) of an arena with >= 40 B of readable slack past its end: the string's
    // dwords come from one or two 16-B loads (+ one dword) issued together, the bytes past 32
    // one at a time
    KD_INLINE void str(const uint8_t* arena, uint32_t b, uint32_t len) {
        if (!len) return;
        typedef uint32_t u32x4a __attribute__((ext_vector_type(4), aligned(4)));
        const uint32_t* a32 = reinterpret_cast<const uint32_t*>(arena) + (b >> 2);
        const uint32_t sh = b & 3u, nw = (sh + len + 3u) >> 2;
        const u32x4a A = *reinterpret_cast<const u32x4a*>(a32);
        u32x4a B = {0u, 0u, 0u, 0u};
        if (nw > 4u) B = *reinterpret_cast<const u32x4a*>(a32 + 4);
        const uint32_t c8 = nw > 8u ? a32[8] : 0u;
        const uint32_t w[9] = {A.x, A.y, A.z, A.w, B.x, B.y, B.z, B.w, c8};
#pragma unroll
        for (uint32_t q = 0; q < 8; ++q) {
            if (4u * q < len) {
                const uint32_t r = len - 4u * q;
                put(__builtin_amdgcn_alignbyte(w[q + 1], w[q], sh), r < 4u ? r : 4u);
            }
        }
        for (uint32_t k = 32; k < len; ++k) put(arena[b + k], 1u);
    }
};

// ---- inline string tables (StrTab, kdtn_kernels.h) ------------------------------------------
template <int W>
struct SIE {
    uint32_t w[W];
};
// length of string id (id 0 = ""), from the byte table (a long or invalid string: its entry);
// bad |= 1 when the string is not valid UTF-8
template <int W>
KD_INLINE uint32_t si_len(const StrTab& t, uint32_t id, uint32_t& bad) {
    if (!id) return 0u;
    const uint32_t l = t.len1[id];
    if (l != 255u) return l;
    const uint32_t* e = t.inl + (size_t)id * W;
    if (e[0] & SI_BAD) bad = 1u;
    return e[2];
}
// entry of string id (id 0: zero, no gather). A key entry (W = 6) loads its last 8 bytes only
// for an inline string of more than 15 bytes (its first 16 bytes and the rest share a line
// three times in four).
template <int W>
KD_INLINE SIE<W> si_load(const StrTab& t, uint32_t id) {
    SIE<W> e;
#pragma unroll
    for (int k = 0; k < W; ++k) e.w[k] = 0u;
    if (!id) return e;
    typedef uint32_t u32x4a __attribute__((ext_vector_type(4), aligned(4)));
    const uint32_t* p = t.inl + (size_t)id * W;
    const u32x4a a = *reinterpret_cast<const u32x4a*>(p);
    e.w[0] = a.x;
    e.w[1] = a.y;
    e.w[2] = a.z;
    e.w[3] = a.w;
    if constexpr (W > 4) {
        const uint32_t b0 = a.x & 0xFFu;
        if (b0 > 15u && b0 < SI_LONG) {
            const uint2 b = *reinterpret_cast<const uint2*>(p + 4);
            e.w[4] = b.x;
            e.w[5] = b.y;
        }
    }
    return e;
}
// length of a loaded entry's string (an invalid one's too); its SI_BAD bit
template <int W>
KD_INLINE uint32_t si_elen(const SIE<W>& e) {
    const uint32_t b0 = e.w[0] & 0xFFu;
    return b0 < SI_LONG ? b0 : e.w[2];
}
template <int W>
KD_INLINE uint32_t si_ebad(const SIE<W>& e) { return e.w[0] & SI_BAD; }

// protobuf string field `field` (nothing for ""): the tag, then bytes 0..len of an inline entry
// (byte 0 is the string's one-byte length varint), or the tag, the length varint and the arena
// bytes of a long string
template <int W>
KD_INLINE void si_field(WSink& o, uint32_t field, const SIE<W>& e, const uint8_t* arena) {
    const uint32_t b0 = e.w[0] & 0xFFu;
    if (b0 == 0u) return;
    if (b0 < SI_LONG) {
        o.byte(field << 3 | 2u);
        const uint32_t n = b0 + 1u;
        o.put(e.w[0], n < 4u ? n : 4u);
#pragma unroll
        for (int q = 1; q < W; ++q) {
            if (!__ballot(4u * q < n)) break;              // the wave's longest string written
            if (4u * q < n) o.put(e.w[q], n - 4u * q < 4u ? n - 4u * q : 4u);
        }
        return;
    }
    const uint32_t len = e.w[2];
    if (len < 0x80u) {
        o.put((field << 3 | 2u) | (len << 8), 2u);
    } else {
        o.byte(field << 3 | 2u);
        o.varint(len);
    }
    o.str(arena, e.w[1], len);
}
// the string's bytes alone (an argv element)
template <int W>
KD_INLINE void si_bytes(WSink& o, const SIE<W>& e, const uint8_t* arena) {
    const uint32_t b0 = e.w[0] & 0xFFu;
    if (b0 >= SI_LONG) {
        o.str(arena, e.w[1], e.w[2]);
        return;
    }
#pragma unroll
    for (int q = 0; q < W; ++q) {
        if (!__ballot(4u * q < b0)) break;
        if (4u * q < b0)
            o.put(__builtin_amdgcn_alignbyte(q + 1 < W ? e.w[q + 1] : 0u, e.w[q], 1u), b0 - 4u * q < 4u ? b0 - 4u * q : 4u);
    }
}

// One wave writes the bytes of its active lanes, which are consecutive ranges [s0, s1) of one
// arena (in lane order, empty lanes between them): each lane's body(WSink&) writes into the
// wave's LDS image (`img`, WIRE_IMG bytes), then the wave stores the image with coalesced
// dword stores — byte stores only at the two dwords shared with the neighbouring waves. A
// range larger than the image is written straight to global memory. Every lane of the wave
// must call it.
template <typename F>
KD_INLINE void wave_image_write(uint32_t* img, bool on, uint64_t s0, uint64_t s1, uint8_t* arena, F&& body) {
    const int lane = threadIdx.x & 63;
    uint64_t r0 = on ? s0 : ~0ull, r1 = on ? s1 : 0ull;
#pragma unroll
    for (int d = 32; d >= 1; d >>= 1) {
        const uint64_t a = __shfl_xor(r0, d, 64), b = __shfl_xor(r1, d, 64);
        r0 = a < r0 ? a : r0;
        r1 = b > r1 ? b : r1;
    }
    if (r1 <= r0) return;                                 // no active lane (wave-uniform)
    const uint32_t lead = (uint32_t)(r0 & 3u);
    WSink o;
    if (r1 - r0 + lead > (uint64_t)WIRE_IMG) {            // too large: straight to global memory
        if (on) {
            o.init(arena + s0);
            body(o);
            o.finish();
        }
        return;
    }
    if (on) {
        o.init(reinterpret_cast<uint8_t*>(img) + lead + (uint32_t)(s0 - r0));
        body(o);
        o.finish();
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    const uint64_t a0 = r0 - lead;                        // dword-aligned global start
    const uint32_t nw = (uint32_t)((r1 - a0 + 3) >> 2);
    for (uint32_t q = lane; q < nw; q += 64) {
        const uint64_t ga = a0 + 4ull * q;
        const uint32_t v = img[q];
        if (ga >= r0 && ga + 4 <= r1) {
            *reinterpret_cast<uint32_t*>(arena + ga) = v;
        } else {
            for (uint32_t k = 0; k < 4; ++k)
                if (ga + k >= r0 && ga + k < r1) arena[ga + k] = (uint8_t)(v >> (8 * k));
        }
    }
}

// One wave writes its lanes' byte ranges [s0, s1) when they are NOT one contiguous range (the
// RemotePod messages of consecutive add entries go to their daemons' runs): every lane writes
// its range into a private dword slot of the wave's LDS image (IMGB bytes) at the alignment of
// its destination (owned WSink), then the wave copies the slots out dword by dword — lane q
// takes image dword q, finds its slot by binary search, and stores it whole, or by bytes where
// the dword is shared with a neighbouring range. Consecutive lanes thus store consecutive
// dwords of each range instead of every lane storing its own range alone. All 64 lanes build
// their ranges in one round when the wave's slots fit the image; otherwise in two rounds of 32
// lanes (the range assembly then runs twice at half the lanes: round 2 measured 2x the VALU
// instructions of a one-round wave), and a round larger than the image goes straight to global
// memory. Every lane must call it.
template <int NL> constexpr int seg_meta() { return 4 * NL; }   // dwords of slot metadata (a uint4 per slot)
template <int NL, int R, int IMGB, typename F>
KD_INLINE void wave_segments_round(uint32_t* img, bool on, uint64_t s0, uint32_t len, uint32_t ndw, uint8_t* arena,
                                   F& body) {
    const int lane = threadIdx.x & 63;
    constexpr int META = seg_meta<NL>();
    uint4* ms = reinterpret_cast<uint4*>(img + IMGB / 4 - META);   // per slot {start dword, dst lo, hi, lead | len << 2}
    constexpr uint32_t budget = IMGB / 4 - META;
    const uint32_t lead = (uint32_t)s0 & 3u;
    const bool mine = NL == 64 || (lane >> 5) == R;
    const uint32_t x = mine ? ndw : 0u;
    uint32_t inc = x;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        const uint32_t o = __shfl_up(inc, d, 64);
        if (lane >= d) inc += o;
    }
    const uint32_t q0 = NL == 64 ? 0u : __shfl(inc - x, 32 * R, 64);         // the round's first slot start
    const uint32_t total = __shfl(inc, NL == 64 ? 63 : 32 * R + 31, 64) - q0;
    const uint32_t qi = inc - x - q0;
    if (total == 0) return;                                      // wave-uniform
    const bool direct = total > budget;                          // too large: straight to global memory
    const int sl = NL == 64 ? lane : lane - 32 * R;
    if (mine && !direct) ms[sl] = make_uint4(qi, (uint32_t)(s0 & ~3ull), (uint32_t)(s0 >> 32), lead | (len << 2));
    if (mine && on) {                                            // one call site of the body
        WSink o;
        if (direct) o.init(arena + s0);
        else o.init_owned(img + qi, lead);
        body(o);
        if (direct) o.finish();
        else o.finish_owned();
    }
    if (direct) return;
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    // whole dwords: lanes 0-31 copy slot 2k, lanes 32-63 slot 2k + 1, 32 consecutive dwords a
    // step (a slot of ~31 dwords takes one step; per dword a binary search over the slot starts
    // cost six LDS reads) ...
    const uint32_t half = (uint32_t)lane >> 5, hl = (uint32_t)lane & 31u;
    for (int k = 0; k < NL; k += 2) {
        const uint4 m = ms[k + half];
        const uint32_t ld = m.w & 3u, end = ld + (m.w >> 2), nd = (end + 3u) >> 2;   // bytes [ld, end)
        uint8_t* base = arena + ((((uint64_t)m.z) << 32) | m.y);
        for (uint32_t kk = hl; kk < nd; kk += 32u) {
            if ((kk == 0 && ld != 0) || 4u * kk + 4u > end) continue;   // an edge dword: below
            *reinterpret_cast<uint32_t*>(base + 4ull * kk) = img[m.x + kk];
        }
    }
    // ... then every lane its own slot's partial first and last dwords, by bytes (the dwords it
    // shares with the neighbouring ranges): at most eight byte stores per lane, instead of four
    // byte-store instructions in every round of the loop above
    if (mine && len) {
        const uint32_t end = lead + len, kl = (end - 1u) >> 2;
        uint8_t* dst = arena + (s0 & ~3ull);
        const uint32_t v0 = img[qi], v1 = img[qi + kl];
        const uint32_t h0 = kl == 0 ? end : 4u;                  // first dword: bytes [lead, h0)
        if (lead != 0 || h0 < 4u) {
#pragma unroll
            for (uint32_t c = 0; c < 4; ++c)
                if (c >= lead && c < h0) dst[c] = (uint8_t)(v0 >> (8 * c));
        }
        const uint32_t h1 = end - 4u * kl;                       // last dword (kl > 0): bytes [0, h1)
        if (kl > 0 && h1 < 4u) {
#pragma unroll
            for (uint32_t c = 0; c < 3; ++c)
                if (c < h1) dst[4u * kl + c] = (uint8_t)(v1 >> (8 * c));
        }
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}
template <int IMGB = WIRE_IMG, typename F>
KD_INLINE void wave_segments_write(uint32_t* img, bool on, uint64_t s0, uint64_t s1, uint8_t* arena, F&& body) {
    const uint32_t len = on ? (uint32_t)(s1 - s0) : 0u;
    const uint32_t ndw = on ? (((uint32_t)s0 & 3u) + len + 3u) >> 2 : 0u;
    uint32_t sum = ndw;                                          // the wave's slot dwords
#pragma unroll
    for (int d = 32; d >= 1; d >>= 1) sum += __shfl_xor(sum, d, 64);
    if (sum <= (uint32_t)(IMGB / 4 - seg_meta<64>())) {          // wave-uniform: one round
        wave_segments_round<64, 0, IMGB>(img, on, s0, len, ndw, arena, body);
        return;
    }
    wave_segments_round<32, 0, IMGB>(img, on, s0, len, ndw, arena, body);   // lanes 0-31, then 32-63
    wave_segments_round<32, 1, IMGB>(img, on, s0, len, ndw, arena, body);
}

// ---- tc argv (kdtn_tc.hip: kdtn_epoch_tc; kdtn_wire.hip: the receiving daemons' commands) ----
// decimal digits of v: compares against the powers of ten, no division (a u64 division loop
// per digit was most of the tc kernels' VALU)
KD_INLINE uint32_t ndigits(uint64_t v) {
    uint32_t n = 1;
    uint64_t p = 10u;
#pragma unroll
    for (int k = 1; k < 20; ++k) {
        n += v >= p ? 1u : 0u;
        p *= 10u;
    }
    return n;
}
KD_INLINE uint32_t ndigits32(uint32_t v) {
    return 1u + (v >= 10u) + (v >= 100u) + (v >= 1000u) + (v >= 10000u) + (v >= 100000u) + (v >= 1000000u) +
           (v >= 10000000u) + (v >= 100000000u) + (v >= 1000000000u);
}
// fixed argument bytes: "qdisc add dev " + " parent 1:1 handle 10:0 tbf rate " + " burst " +
// " latency 50ms minburst " + final NUL (every separator is a NUL)
constexpr uint32_t TC_FIXED = 14 + 1 + 32 + 1 + 6 + 1 + 22 + 1;

struct TcEntry {
    uint32_t intf;      // kdict id of LocalIntf
    uint64_t rate;
    uint32_t buffer, minburst;
    bool on;
};

// bytes of a TBF command's argv (0 when it runs none)
KD_INLINE uint32_t tc_size(const StrTab& kd, const TcEntry& t) {
    uint32_t bad = 0;                                      // argv bytes need no UTF-8
    return t.on ? TC_FIXED + si_len<SI_KW>(kd, t.intf, bad) + ndigits(t.rate) + ndigits32(t.buffer) +
                      ndigits32(t.minburst)
                : 0u;
}

// one argv element + its NUL separator: a literal, packed 4 bytes per put (constant-folded)
template <int N>
KD_INLINE void lit(WSink& o, const char (&s)[N]) {
#pragma unroll
    for (int k = 0; k < N; k += 4) {
        uint32_t w = 0;
#pragma unroll
        for (int c = 0; c < 4; ++c)
            if (k + c < N) w |= (uint32_t)(uint8_t)s[k + c] << (8 * c);
        o.put(w, (uint32_t)(N - k < 4 ? N - k : 4));
    }
}
// four ASCII digits of l < 10000, most significant first
KD_INLINE uint32_t dig4(uint32_t l) {
    return (0x30u + l / 1000u) | (0x30u + (l / 100u) % 10u) << 8 | (0x30u + (l / 10u) % 10u) << 16 |
           (0x30u + l % 10u) << 24;
}
// fmt.Sprint of an unsigned integer + NUL: base-10000 limbs, the top one without leading zeros
KD_INLINE void num(WSink& o, uint64_t v) {
    uint32_t l0, l1, l2, l3, l4;
    if (v >> 32) {                                      // u64 divisions only above 2^32
        l0 = (uint32_t)(v % 10000u);
        v /= 10000u;
        l1 = (uint32_t)(v % 10000u);
        v /= 10000u;
        l2 = (uint32_t)(v % 10000u);
        v /= 10000u;
        l3 = (uint32_t)(v % 10000u);
        l4 = (uint32_t)(v / 10000u);                    // < 1845 (2^64 < 10^20)
    } else {                                            // u32: divisions by constants are multiplies
        uint32_t x = (uint32_t)v;
        l0 = x % 10000u;
        x /= 10000u;
        l1 = x % 10000u;
        l2 = x / 10000u;                                // < 43
        l3 = l4 = 0u;
    }
    const int k = l4 ? 4 : l3 ? 3 : l2 ? 2 : l1 ? 1 : 0;
    const uint32_t top = k == 4 ? l4 : k == 3 ? l3 : k == 2 ? l2 : k == 1 ? l1 : l0;
    const uint32_t nd = ndigits32(top);
    o.put(dig4(top) >> (8u * (4u - nd)), nd);
    if (k >= 4) o.put(dig4(l3), 4u);
    if (k >= 3) o.put(dig4(l2), 4u);
    if (k >= 2) o.put(dig4(l1), 4u);
    if (k >= 1) o.put(dig4(l0), 4u);
    o.byte(0u);
}

KD_INLINE void write_tbf_argv(WSink& o, const StrTab& kd, const TcEntry& t) {
    const SIE<SI_KW> dev = si_load<SI_KW>(kd, t.intf);    // the interface name: one gather
    lit(o, "qdisc");
    lit(o, "add");
    lit(o, "dev");
    si_bytes(o, dev, kd.bytes);
    o.byte(0u);
    lit(o, "parent");
    lit(o, "1:1");
    lit(o, "handle");
    lit(o, "10:0");
    lit(o, "tbf");
    lit(o, "rate");
    num(o, t.rate);
    lit(o, "burst");
    num(o, t.buffer);
    lit(o, "latency");
    lit(o, "50ms");
    lit(o, "minburst");
    num(o, t.minburst);
}

}  // namespace kdtn
