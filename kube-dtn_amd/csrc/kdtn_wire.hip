// kdtn_wire.hip — protobuf wire encoding of the epoch's batches on the GPU (SURVEY §8(f)
// rank 1): for every Topology and list (DelLinks, AddLinks, UpdateLinks) the bytes of
//
//   proto.Marshal(&pb.LinksBatchQuery{LocalPod: &pb.Pod{Name, SrcIp, NetNs, KubeNs},
//                                     Links: common.Map(links, v1.Link.ToProto)})
//
// that Reconcile sends (controllers/topology_controller.go:180-188, 223-231, 266-274;
// api/v1/topology_types.go:97-109,178-194; proto/v1/kube_dtn.proto:8-53,65-68), so the Go
// side can hand them to the gRPC stream without ToProto + Marshal per link.
//
// Layout: one byte arena, regions del | add | upd, each in topology order; batch (l, t)
// occupies [off[l*T+t], off[l*T+t+1]) (empty when the list is empty — no RPC — or when a
// string is not valid UTF-8, which makes Marshal fail; err[t] bit l marks the latter).
//
// Kernels (launch order, kdtn_epoch_encode):
//   k_str_inline     per dictionary string its inline table entry and its length byte
//                    (StrTab, kdtn_kernels.h; unicode/utf8.ValidString decides SI_BAD)
//   k_wire_entry_sizes  one thread per entry: its topology and encoded size (its Link, plus
//                    the LocalPod header for a batch's first entry) from the length bytes; a
//                    string that is not valid UTF-8 fails its batch (err bit)
//   k_wire_scan_*    exclusive scan of the sizes of entries whose batch marshals → u64 arena
//                    offset of every entry; k_wire_batch_off: batch offsets [3T+1]
//   k_wire_write     one thread per entry: one gather per string field (the inline entry),
//                    its bytes assembled into the wave's LDS image (dwords built in registers,
//                    WSink), which the wave then stores with coalesced dword stores
#include "kdtn_encode.h"

namespace kdtn {


// ---- dictionary UTF-8 validity (Go unicode/utf8.ValidString) ---------------------------
KD_INLINE bool utf8_ok(const uint8_t* s, uint32_t n) {
    uint32_t i = 0;
    while (i < n) {
        const uint32_t c = s[i];
        if (c < 0x80u) { ++i; continue; }
        uint32_t need, lo = 0x80u, hi = 0xBFu;
        if (c >= 0xC2u && c <= 0xDFu) need = 1;
        else if (c == 0xE0u) { need = 2; lo = 0xA0u; }
        else if (c >= 0xE1u && c <= 0xECu) need = 2;
        else if (c == 0xEDu) { need = 2; hi = 0x9Fu; }
        else if (c >= 0xEEu && c <= 0xEFu) need = 2;
        else if (c == 0xF0u) { need = 3; lo = 0x90u; }
        else if (c >= 0xF1u && c <= 0xF3u) need = 3;
        else if (c == 0xF4u) { need = 3; hi = 0x8Fu; }
        else return false;
        if (i + need >= n) return false;
        const uint32_t c1 = s[i + 1];
        if (c1 < lo || c1 > hi) return false;
        for (uint32_t k = 2; k <= need; ++k)
            if (s[i + k] < 0x80u || s[i + k] > 0xBFu) return false;
        i += need + 1;
    }
    return true;
}

// One thread per dictionary string: its inline entry (W dwords; StrTab) and its length byte.
// The string's first 32 bytes come from one 16-B load pair (+ a dword); only strings with a
// byte >= 0x80 run the UTF-8 automaton. Bytes of an inline entry past the string are zero.
template <int W>
__global__ void __launch_bounds__(BLOCK) k_str_inline(const uint8_t* bytes, const uint32_t* offs, uint32_t n,
                                                      uint32_t* inl, uint8_t* len1) {
    const uint32_t i = blockIdx.x * BLOCK + threadIdx.x;
    if (i >= n) return;
    const uint32_t b = offs[i], len = offs[i + 1] - b;
    uint32_t hi = 0, s[8] = {0u, 0u, 0u, 0u, 0u, 0u, 0u, 0u};   // the string's dwords, zero past len
    if (len) {
        typedef uint32_t u32x4a __attribute__((ext_vector_type(4), aligned(4)));
        const uint32_t* a32 = reinterpret_cast<const uint32_t*>(bytes) + (b >> 2);
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
                const uint32_t m = r >= 4u ? 0xFFFFFFFFu : ((1u << (8u * r)) - 1u);
                s[q] = __builtin_amdgcn_alignbyte(w[q + 1], w[q], sh) & m;
                hi |= s[q] & 0x80808080u;
            }
        }
        for (uint32_t k = 32; k < len; ++k) hi |= bytes[b + k] & 0x80u;
    }
    const bool bad = hi != 0 && !utf8_ok(bytes + b, len);
    uint32_t e[W];
    if (!bad && len <= 4u * W - 1u) {                      // inline: byte 0 = len, bytes 1..len
        e[0] = len | (s[0] << 8);
#pragma unroll
        for (int q = 1; q < W; ++q) e[q] = (s[q - 1] >> 24) | (s[q] << 8);
    } else {                                               // long or not valid UTF-8: the range
#pragma unroll
        for (int q = 0; q < W; ++q) e[q] = 0u;
        e[0] = SI_LONG | (bad ? SI_BAD : 0u);
        e[1] = b;
        e[2] = len;
    }
    uint32_t* o = inl + (size_t)i * W;
    if constexpr (W == 4) {
        *reinterpret_cast<uint4*>(o) = make_uint4(e[0], e[1], e[2], e[3]);
    } else {
#pragma unroll
        for (int q = 0; q < W; q += 2) *reinterpret_cast<uint2*>(o + q) = make_uint2(e[q], e[q + 1]);
    }
    len1[i] = (uint8_t)((!bad && len <= 254u) ? len : 255u);
}
template __global__ void k_str_inline<SI_KW>(const uint8_t*, const uint32_t*, uint32_t, uint32_t*, uint8_t*);
template __global__ void k_str_inline<SI_PW>(const uint8_t*, const uint32_t*, uint32_t, uint32_t*, uint8_t*);

// ---- sizes ---------------------------------------------------------------------------------
KD_INLINE uint32_t vlen(uint64_t v) {
    uint32_t n = 1;
    while (v >= 0x80u) { v >>= 7; ++n; }
    return n;
}
KD_INLINE uint32_t str_field(uint32_t len) { return len ? 1u + vlen(len) + len : 0u; }

// pb.LinkProperties size (psz) and pb.Link size (lsz) of record j from the length bytes, and the
// bytes of the Link's fields before its properties (pre: fields 1-6); false if a string is not
// valid UTF-8
KD_INLINE bool link_sizes(const WireIn& w, const DevLinks& L, uint32_t j, uint32_t* psz, uint32_t* lsz,
                          uint32_t* pre) {
    uint32_t kid[KDTN_NKEY], pid[KDTN_NPROP];
#pragma unroll
    for (int k = 0; k < KDTN_NKEY; ++k) kid[k] = L.key(k, j);
#pragma unroll
    for (int k = 0; k < KDTN_NPROP; ++k) pid[k] = L.prop(k, j);
    const uint32_t gap = L.gap(j);
    const int64_t uid = L.uid(j);
    uint32_t bad = 0, p = 0, l = 0;
#pragma unroll
    for (int k = 0; k < KDTN_NPROP; ++k) p += str_field(si_len<SI_PW>(w.pd, pid[k], bad));
    if (gap) p += 1u + vlen(gap);
    uint32_t macs = 0;
#pragma unroll
    for (int k = 0; k < KDTN_NKEY; ++k) {
        const uint32_t f = str_field(si_len<SI_KW>(w.kd, kid[k], bad));
        if (k == KDTN_K_LOCAL_MAC || k == KDTN_K_PEER_MAC) macs += f;
        else l += f;
    }
    if (uid) l += 1u + vlen((uint64_t)uid);
    *pre = l;
    l += 1u + vlen(p) + p + macs;
    *psz = p;
    *lsz = l;
    return bad == 0;
}

// pb.Pod LocalPod of topology t: {Name, SrcIp, NetNs, KubeNs}
KD_INLINE uint32_t pod_size(const WireIn& w, uint32_t t, bool* ok) {
    const uint32_t ids[4] = {w.t_name[t], w.t_src[t], w.t_netns[t], w.t_ns[t]};
    uint32_t s = 0, bad = 0;
#pragma unroll
    for (int k = 0; k < 4; ++k) s += str_field(si_len<SI_KW>(w.kd, ids[k], bad));
    *ok = bad == 0;
    return s;
}

// list of global entry g (entries of the del, add, upd lists in that order)
KD_INLINE uint32_t wire_list(const WireIn& w, uint32_t g) {
    return g < w.list_base[1] ? 0u : (g < w.list_base[2] ? 1u : 2u);
}

// One thread per entry (all three lists): its topology (a wave-cooperative search per list the
// wave holds) and its encoded size — the Link field (tag + length varint + message), plus the
// LinksBatchQuery.local_pod field for the first entry of a batch. A string that is not valid
// UTF-8 makes the batch's Marshal fail: err[t] bit l, and the size does not count.
__global__ void __launch_bounds__(BLOCK) k_wire_entry_sizes(WireIn w, DevLinks O, DevLinks N, WireWork wk) {
    const uint32_t g = blockIdx.x * BLOCK + threadIdx.x;
    const bool on = g < w.n_entries;
    const uint32_t lst = on ? wire_list(w, g) : 3u;
    const uint32_t e = on ? g - w.list_base[lst] : 0u;
    uint32_t t = 0;
#pragma unroll
    for (uint32_t l = 0; l < 3; ++l)
        if (__ballot(lst == l)) {                          // wave-uniform
            const uint32_t tl = entry_topo_wave_c(w.list_off[l], w.coarse[l], w.T, e, lst == l);
            if (lst == l) t = tl;
        }
    if (!on) return;
    uint32_t psz, lsz, pre;
    bool ok = link_sizes(w, lst == 0 ? O : N, w.list_idx[lst][e], &psz, &lsz, &pre);
    uint32_t size = 1u + vlen(lsz) + lsz, hdr = 0;
    if (e == w.list_off[lst][t]) {                         // the batch's first entry carries the header
        bool pok;
        const uint32_t ps = pod_size(w, t, &pok);
        ok = ok && pok;
        hdr = 1u + vlen(ps) + ps;
        size += hdr;
    }
    if (lst == 1 && wk.pinfo)                              // the AddLinks entry's properties field
        wk.pinfo[e] = ((uint64_t)(hdr + 1u + vlen(lsz) + pre) << 32) | (1u + vlen(psz) + psz);
    wk.size[g] = ok ? size : 0u;
    wk.topo[g] = t;
    if (!ok) atomicOr(wk.err + t, 1u << lst);
}

// size of entry g as the arena lays it out: 0 when its batch does not marshal
KD_INLINE uint32_t wire_masked_size(const WireIn& w, const WireWork& wk, uint32_t g) {
    if (g >= w.n_entries) return 0u;
    return ((wk.err[wk.topo[g]] >> wire_list(w, g)) & 1u) ? 0u : wk.size[g];
}

// ---- exclusive scan of the entry sizes into u64 arena offsets ----------------------------
__global__ void __launch_bounds__(BLOCK) k_wire_scan_partial(WireIn w, WireWork wk, uint64_t* part) {
    __shared__ uint64_t sh[BLOCK / 64];
    const uint32_t b0 = blockIdx.x * SCAN_CHUNK + threadIdx.x * 4;
    uint64_t v = 0;
#pragma unroll
    for (int k = 0; k < 4; ++k) v += wire_masked_size(w, wk, b0 + k);
    uint64_t tot;
    block_exclusive(v, sh, &tot);
    if (threadIdx.x == 0) part[blockIdx.x] = tot;
}

__global__ void __launch_bounds__(BLOCK) k_wire_scan_final(WireIn w, WireWork wk, const uint64_t* part) {
    __shared__ uint64_t sh[BLOCK / 64];
    const uint32_t b0 = blockIdx.x * SCAN_CHUNK + threadIdx.x * 4;
    uint32_t v[4];
    uint64_t sum = 0;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        v[k] = wire_masked_size(w, wk, b0 + k);
        sum += v[k];
    }
    uint64_t tot;
    uint64_t x = part[blockIdx.x] + block_exclusive(sum, sh, &tot);
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        if (b0 + k <= w.n_entries) wk.pos[b0 + k] = x;     // pos[n] = grand total
        x += v[k];
    }
}

// batch (l, t) starts where its first entry does (an empty or failed batch: where the next
// batch starts); off[3T] = total. A batch of more than 4 GiB is flagged in err[T].
__global__ void __launch_bounds__(BLOCK) k_wire_batch_off(WireIn w, WireWork wk) {
    const uint32_t i = blockIdx.x * BLOCK + threadIdx.x;
    if (i > 3u * w.T) return;
    if (i == 3u * w.T) {
        wk.off[i] = wk.pos[w.n_entries];
        return;
    }
    const uint32_t l = i / w.T, t = i - l * w.T;
    const uint64_t a = wk.pos[w.list_base[l] + w.list_off[l][t]], b = wk.pos[w.list_base[l] + w.list_off[l][t + 1]];
    wk.off[i] = a;
    if (b - a > 0xFFFFFFFFull) atomicOr(wk.err + w.T, 1u);
}

// ---- exclusive scan of u32 sizes into u64 offsets (fan-out, RemotePod, tc) ---------------
__global__ void __launch_bounds__(BLOCK) k_scan_partial(const uint32_t* size, uint32_t n, uint64_t* part) {
    __shared__ uint64_t sh[BLOCK / 64];
    const uint32_t b0 = blockIdx.x * SCAN_CHUNK + threadIdx.x * 4;
    uint64_t v = 0;
#pragma unroll
    for (int k = 0; k < 4; ++k) v += b0 + k < n ? size[b0 + k] : 0u;
    uint64_t tot;
    block_exclusive(v, sh, &tot);
    if (threadIdx.x == 0) part[blockIdx.x] = tot;
}

// single block: exclusive scan of the block totals in place. 1024 threads x 16 consecutive
// totals each per pass, so the usual few-thousand totals take one pass (a 256-thread loop of
// one total per thread took ~40 dependent passes, ~0.1 ms, for 10M entries)
__global__ void __launch_bounds__(SCAN_TOP_BLOCK) k_scan_top(uint64_t* part, uint32_t nb) {
    __shared__ uint64_t wsum[SCAN_TOP_BLOCK / 64];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    uint64_t carry = 0;
    for (uint32_t c0 = 0; c0 < nb; c0 += SCAN_TOP_BLOCK * SCAN_TOP_PER) {
        const uint32_t b = c0 + (uint32_t)tid * SCAN_TOP_PER;
        uint64_t v[SCAN_TOP_PER], sum = 0;
#pragma unroll
        for (int k = 0; k < SCAN_TOP_PER; ++k) {
            v[k] = b + k < nb ? part[b + k] : 0ull;
            sum += v[k];
        }
        uint64_t x = sum;
#pragma unroll
        for (int d = 1; d < 64; d <<= 1) {
            const uint64_t o = __shfl_up(x, d, 64);
            if (lane >= d) x += o;
        }
        if (lane == 63) wsum[wave] = x;
        __syncthreads();
        uint64_t base = carry, tot = 0;
#pragma unroll
        for (int w = 0; w < SCAN_TOP_BLOCK / 64; ++w) {
            if (w < wave) base += wsum[w];
            tot += wsum[w];
        }
        __syncthreads();
        uint64_t run = base + x - sum;
#pragma unroll
        for (int k = 0; k < SCAN_TOP_PER; ++k) {
            if (b + k < nb) part[b + k] = run;
            run += v[k];
        }
        carry += tot;
    }
}

__global__ void __launch_bounds__(BLOCK) k_scan_final(const uint32_t* size, uint32_t n, const uint64_t* part,
                                                      uint64_t* off) {
    __shared__ uint64_t sh[BLOCK / 64];
    const uint32_t b0 = blockIdx.x * SCAN_CHUNK + threadIdx.x * 4;
    uint32_t v[4];
    uint64_t sum = 0;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        v[k] = b0 + k < n ? size[b0 + k] : 0u;
        sum += v[k];
    }
    uint64_t tot;
    uint64_t x = part[blockIdx.x] + block_exclusive(sum, sh, &tot);
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        if (b0 + k <= n) off[b0 + k] = x;     // off[n] = grand total
        x += v[k];
    }
}

// ---- writer --------------------------------------------------------------------------------
// One entry's bytes: the key strings' inline entries and the property strings' length bytes
// gathered at once (the sizes come from them), then the fields in number order, the property
// entries gathered after the key fields are written (registers: 7 key entries + 12 property
// entries held together cost the writer a wave per SIMD).
KD_INLINE void write_entry(WSink& o, const WireIn& w, const DevLinks& L, uint32_t j, bool header, uint32_t t) {
    SIE<SI_KW> k[KDTN_NKEY];
#pragma unroll
    for (int q = 0; q < KDTN_NKEY; ++q) k[q] = si_load<SI_KW>(w.kd, L.key(q, j));
    uint32_t pid[KDTN_NPROP];
#pragma unroll
    for (int q = 0; q < KDTN_NPROP; ++q) pid[q] = L.prop(q, j);
    const uint32_t gap = L.gap(j);
    const int64_t uid = L.uid(j);
    uint32_t psz = 0, lsz = 0, bad = 0;
#pragma unroll
    for (int q = 0; q < KDTN_NPROP; ++q) psz += str_field(si_len<SI_PW>(w.pd, pid[q], bad));
    if (gap) psz += 1u + vlen(gap);
#pragma unroll
    for (int q = 0; q < KDTN_NKEY; ++q) lsz += str_field(si_elen(k[q]));
    if (uid) lsz += 1u + vlen((uint64_t)uid);
    lsz += 1u + vlen(psz) + psz;
    if (header) {                                         // LinksBatchQuery.local_pod
        const uint32_t ids[4] = {w.t_name[t], w.t_src[t], w.t_netns[t], w.t_ns[t]};
        SIE<SI_KW> h[4];
        uint32_t hs = 0;
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            h[q] = si_load<SI_KW>(w.kd, ids[q]);
            hs += str_field(si_elen(h[q]));
        }
        o.byte(1u << 3 | 2u);
        o.varint(hs);
#pragma unroll
        for (int q = 0; q < 4; ++q) si_field(o, (uint32_t)q + 1u, h[q], w.kd.bytes);
    }
    o.byte(2u << 3 | 2u);                                 // LinksBatchQuery.links
    o.varint(lsz);
    // pb.Link fields in number order: peer_pod 1, local_intf 2, peer_intf 3, local_ip 4,
    // peer_ip 5, uid 6, properties 7, local_mac 8, peer_mac 9
    si_field(o, 1, k[KDTN_K_PEER_POD], w.kd.bytes);
    si_field(o, 2, k[KDTN_K_LOCAL_INTF], w.kd.bytes);
    si_field(o, 3, k[KDTN_K_PEER_INTF], w.kd.bytes);
    si_field(o, 4, k[KDTN_K_LOCAL_IP], w.kd.bytes);
    si_field(o, 5, k[KDTN_K_PEER_IP], w.kd.bytes);
    if (uid) {
        o.byte(6u << 3);
        o.varint((uint64_t)uid);
    }
    o.byte(7u << 3 | 2u);
    o.varint(psz);
    SIE<SI_PW> p[KDTN_NPROP];
#pragma unroll
    for (int q = 0; q < KDTN_NPROP; ++q) p[q] = si_load<SI_PW>(w.pd, pid[q]);
    // pb.LinkProperties: latency 1 .. rate 6, gap 7, duplicate 8 .. corrupt_corr 13 (KDTN_P_* order)
#pragma unroll
    for (int q = 0; q < KDTN_NPROP; ++q) {
        if (q == KDTN_P_DUPLICATE && gap) {
            o.byte(7u << 3);
            o.varint(gap);
        }
        si_field(o, (uint32_t)(q < KDTN_P_DUPLICATE ? q + 1 : q + 2), p[q], w.pd.bytes);
    }
    si_field(o, 8, k[KDTN_K_LOCAL_MAC], w.kd.bytes);
    si_field(o, 9, k[KDTN_K_PEER_MAC], w.kd.bytes);
}

// One thread per entry of the three lists (global entry index g). Consecutive entries
// write consecutive arena bytes (failed batches occupy none), so a wave's output is one
// contiguous range, assembled in the wave's LDS image (wave_image_write).
__global__ void __launch_bounds__(BLOCK) k_wire_write(WireIn w, DevLinks O, DevLinks N, WireWork wk,
                                                      uint8_t* arena) {
    __shared__ uint32_t img[BLOCK / 64][WIRE_IMG / 4];
    const uint32_t g = blockIdx.x * BLOCK + threadIdx.x;
    bool on = g < w.n_entries;
    uint32_t lst = 0, t = 0, e = 0;
    uint64_t s0 = 0, s1 = 0;
    if (on) {
        lst = wire_list(w, g);
        e = g - w.list_base[lst];
        t = wk.topo[g];
        on = ((wk.err[t] >> lst) & 1u) == 0;
        s0 = wk.pos[g];
        s1 = wk.pos[g + 1];
    }
    wave_image_write(img[threadIdx.x >> 6], on, s0, s1, arena, [&](WSink& o) __attribute__((always_inline)) {
        write_entry(o, w, lst == 0 ? O : N, w.list_idx[lst][e], e == w.list_off[lst][t], t);
    });
}

// ==========================================================================================
// RemotePod messages (proto/v1/kube_dtn.proto:65-79): the UpdateRemote payload of every
// add entry the fan-out groups (common/utils.go:42-51), in fan-out order, then the physical
// peers' local Update payloads (daemon/kubedtn/handler.go:353-362) in add-list order. Each
// message is preceded by its varint length; a message with a string that is not valid UTF-8
// fails to marshal and is empty. Fields: net_ns 1, intf_name 2, intf_ip 3, peer_vtep 4,
// kube_ns 5, int32 vni 6 (10-byte varint when negative), properties 7 (always present:
// Link.ToProto sets it), name 8.
// ==========================================================================================
__global__ void __launch_bounds__(BLOCK) k_remote_phys_flags(const uint8_t* reach_add, const uint4* add_res,
                                                             uint32_t na, uint32_t* flag) {
    const uint32_t e = blockIdx.x * BLOCK + threadIdx.x;
    if (e >= na) return;
    const uint32_t w = add_res[e].w;
    flag[e] = ((reach_add[e] & REACH_ON) && (w & 0xFFu) == KDTN_KIND_PHYSICAL && ((w >> 8) & 0xFFu) == 0) ? 1u : 0u;
}

__global__ void __launch_bounds__(BLOCK) k_remote_phys_scatter(const uint32_t* flag, const uint64_t* pos, uint32_t na,
                                                               uint32_t* phys_idx) {
    const uint32_t e = blockIdx.x * BLOCK + threadIdx.x;
    if (e < na && flag[e]) phys_idx[pos[e]] = e;
}

// the string ids of add entry e's message (remote: the UpdateRemote payload, else the physical
// peer's local Update payload; t = the entry's topology) in field order net_ns, intf_name,
// intf_ip, peer_vtep, kube_ns, name, and the link's property ids
struct RemoteMsg {
    uint32_t s[6], p[KDTN_NPROP];
    uint32_t gap;
    int32_t vni;
    bool phys;                      // peer_vtep = TrimPrefix(PeerPod, "physical/")
    uint32_t plen;                  // > 0: the properties field's bytes are the wire encoding's, at
    uint64_t psrc;                  // w_arena + psrc (its batch marshalled: every string valid)
};

KD_INLINE RemoteMsg remote_msg(const RemoteIn& r, uint32_t e, uint32_t t, bool remote) {
    RemoteMsg q;
    const uint32_t j = r.add_idx[e];
    const uint4 res = r.add_res[e];
    const uint32_t peer_pod = r.N.key(KDTN_K_PEER_POD, j);
    if (remote) {                                   // UpdateRemote: the peer daemon's side
        q.s[0] = r.pods[res.x].w & 0x7FFFFFFFu;     // peerPod.NetNs
        q.s[1] = r.N.key(KDTN_K_PEER_INTF, j);
        q.s[2] = r.N.key(KDTN_K_PEER_IP, j);
        q.s[3] = r.t_src[t];                        // localPod.SrcIp
    } else {                                        // physical: the local pod's side
        q.s[0] = r.t_netns[t];
        q.s[1] = r.N.key(KDTN_K_LOCAL_INTF, j);
        q.s[2] = r.N.key(KDTN_K_LOCAL_IP, j);
        q.s[3] = peer_pod;                          // TrimPrefix(PeerPod, "physical/")
    }
    q.s[4] = r.t_ns[t];                             // localPod.KubeNs
    q.s[5] = peer_pod;
    q.vni = (int32_t)res.y;
    q.phys = !remote;
    q.plen = 0;
    q.psrc = 0;
    if (r.w_pinfo && !((r.w_err[t] >> 1) & 1u)) {   // the run's AddLinks batch of t marshalled
        const uint64_t pi = r.w_pinfo[e];
        q.psrc = r.w_pos[r.w_nd + e] + (pi >> 32);
        q.plen = (uint32_t)pi;
    }
    q.gap = 0;
#pragma unroll
    for (int k = 0; k < KDTN_NPROP; ++k) q.p[k] = 0;
    if (!q.plen) {                                  // the property strings themselves
#pragma unroll
        for (int k = 0; k < KDTN_NPROP; ++k) q.p[k] = r.N.prop(k, j);
        q.gap = r.N.gap(j);
    }
    return q;
}

// message body size from the string lengths (the trimmed peer_vtep of a physical message is 9
// bytes shorter; "physical/" is ASCII, so it is valid UTF-8 iff the whole name is); false if a
// string is not valid UTF-8 (Marshal fails)
KD_INLINE bool remote_sizes(const RemoteIn& r, const RemoteMsg& q, uint32_t* body) {
    uint32_t n = 0, bad = 0;
#pragma unroll
    for (int k = 0; k < 6; ++k) {
        uint32_t l = si_len<SI_KW>(r.kd, q.s[k], bad);
        if (k == 3 && q.phys) l -= 9u;
        n += str_field(l);
    }
    if (q.vni) n += 1u + vlen((uint64_t)(int64_t)q.vni);
    if (q.plen) {                                   // the wire encoding's properties field
        n += q.plen;
    } else {
        uint32_t p = 0;
#pragma unroll
        for (int k = 0; k < KDTN_NPROP; ++k) p += str_field(si_len<SI_PW>(r.pd, q.p[k], bad));
        if (q.gap) p += 1u + vlen(q.gap);
        n += 1u + vlen(p) + p;
    }
    *body = n;
    return bad == 0;
}

// The receiving daemon's TBF command for RemotePod message m (m < n_remote): the peer
// daemon's Update runs SetupVxLan on link.PeerIntf → MakeQdiscs (the same properties, which
// built on the sending side) → SetVethQdiscs (daemon/vxlan/vxlan.go:31-51), unless its
// CreateOrUpdate rejects IntfIp (kdtn_resolved.remote_err). Physical messages have none here
// (their tc runs on LocalIntf: kdtn_epoch_tc slot 2e).
KD_INLINE TcEntry tc_remote_entry(const RemoteIn& r, uint32_t e) {
    TcEntry t{0, 0, 0, 0, false};
    if (!(r.send[e] & REACH_SEND)) return t;
    const uint2* q = r.add_qdisc + (size_t)e * 9;
    const uint32_t flags = q[8].y;
    if (((flags >> 8) & 0xFFu) == 0 || (r.add_res[e].w >> 24) != 0) return t;
    t.intf = r.N.key(KDTN_K_PEER_INTF, r.add_idx[e]);
    t.buffer = q[6].y;
    t.rate = ((uint64_t)q[7].y << 32) | q[7].x;
    t.minburst = q[8].x;
    t.on = true;
    return t;
}

// One thread per add entry (add-list order: the entry's columns are read coalesced): the size
// of its message, if it has one (0 when a string is not valid UTF-8), and for an UpdateRemote
// the receiving daemon's tc argv size, both stored at the message's index (every message has
// exactly one entry, so the arrays need no clearing)
__global__ void __launch_bounds__(BLOCK) k_remote_sizes(RemoteIn r, uint32_t* msz, uint32_t* tsz) {
    const uint32_t e = blockIdx.x * BLOCK + threadIdx.x;
    const uint32_t kind = e < r.n_add ? remote_kind(r, e) : 0u;
    if (__ballot(kind != 0) == 0) return;           // wave-uniform
    const uint32_t t = entry_topo_wave_c(r.add_off, r.add_coarse, r.T, e, kind != 0);
    if (!kind) return;
    const RemoteMsg q = remote_msg(r, e, t, kind == 1);
    const uint32_t ts = kind == 1 ? tc_size(r.kd, tc_remote_entry(r, e)) : 0u;   // (its loads before the stores)
    uint32_t body;
    const bool ok = remote_sizes(r, q, &body);
    const uint32_t m = remote_msg_index(r, e, kind);
    msz[m] = ok ? vlen(body) + body : 0u;
    tsz[m] = ts;
}

// a string field from arena bytes [b, b + len) (nothing for "")
KD_INLINE void arena_field(WSink& o, uint32_t field, const uint8_t* arena, uint32_t b, uint32_t len) {
    if (!len) return;
    if (len < 0x80u) {
        o.put((field << 3 | 2u) | (len << 8), 2u);
    } else {
        o.byte(field << 3 | 2u);
        o.varint(len);
    }
    o.str(arena, b, len);
}

// the message's bytes: the key strings' entries gathered at once, then the fields in number
// order; the properties field copied from the wire encoding when the run has one for the entry
// (q.plen), else from the property strings' length bytes and entries (gathered after the key
// fields are written, as in write_entry)
KD_INLINE void write_remote(WSink& o, const RemoteIn& r, const RemoteMsg& q) {
    SIE<SI_KW> s[6];
#pragma unroll
    for (int k = 0; k < 6; ++k) s[k] = si_load<SI_KW>(r.kd, (k == 3 && q.phys) ? 0u : q.s[k]);
    uint32_t vb = 0, vl = 0;                        // physical: the trimmed name's arena range
    if (q.phys) {
        vb = r.kd_offs[q.s[3]] + 9u;
        vl = r.kd_offs[q.s[3] + 1] - vb;
    }
    uint32_t n = 0, psz = 0, bad = 0;
#pragma unroll
    for (int k = 0; k < 6; ++k) n += str_field(k == 3 && q.phys ? vl : si_elen(s[k]));
    if (q.vni) n += 1u + vlen((uint64_t)(int64_t)q.vni);
    if (q.plen) {
        n += q.plen;
    } else {
#pragma unroll
        for (int k = 0; k < KDTN_NPROP; ++k) psz += str_field(si_len<SI_PW>(r.pd, q.p[k], bad));
        if (q.gap) psz += 1u + vlen(q.gap);
        n += 1u + vlen(psz) + psz;
    }
    o.varint(n);
#pragma unroll
    for (int k = 0; k < 5; ++k) {
        if (k == 3 && q.phys) arena_field(o, 4u, r.kd.bytes, vb, vl);
        else si_field(o, (uint32_t)k + 1, s[k], r.kd.bytes);
    }
    if (q.vni) {
        o.byte(6u << 3);
        o.varint((uint64_t)(int64_t)q.vni);
    }
    if (q.plen) {
        o.copy(r.w_arena, q.psrc, q.plen);
    } else {
        o.byte(7u << 3 | 2u);
        o.varint(psz);
        SIE<SI_PW> p[KDTN_NPROP];
#pragma unroll
        for (int k = 0; k < KDTN_NPROP; ++k) p[k] = si_load<SI_PW>(r.pd, q.p[k]);
#pragma unroll
        for (int k = 0; k < KDTN_NPROP; ++k) {
            if (k == KDTN_P_DUPLICATE && q.gap) {
                o.byte(7u << 3);
                o.varint(q.gap);
            }
            si_field(o, (uint32_t)(k < KDTN_P_DUPLICATE ? k + 1 : k + 2), p[k], r.pd.bytes);
        }
    }
    si_field(o, 8, s[5], r.kd.bytes);
}

// One thread per add entry with a message, in add-list order (its columns read coalesced),
// writing the message at its fan-out position. A wave's messages for one daemon are one
// contiguous run of the arena (fan-out order keeps add-list order within a daemon), so the
// wave stores them through its LDS image dword by dword (wave_segments_write).
__global__ void __launch_bounds__(BLOCK, 4) k_remote_write(RemoteIn r, const uint64_t* off, uint8_t* arena) {
    __shared__ uint32_t img[BLOCK / 64][REMOTE_IMG / 4];
    const uint32_t e = blockIdx.x * BLOCK + threadIdx.x;
    const uint32_t kind = e < r.n_add ? remote_kind(r, e) : 0u;
    if (__ballot(kind != 0) == 0) return;           // wave-uniform
    const uint32_t t = entry_topo_wave_c(r.add_off, r.add_coarse, r.T, e, kind != 0);
    uint64_t s0 = 0, s1 = 0;
    if (kind) {
        const uint32_t m = remote_msg_index(r, e, kind);
        s0 = off[m];
        s1 = off[m + 1];
    }
    const bool on = s1 > s0;                        // empty: no message or a Marshal error
    RemoteMsg q{};
    if (on) q = remote_msg(r, e, t, kind == 1);
    wave_segments_write<REMOTE_IMG>(img[threadIdx.x >> 6], on, s0, s1, arena,
                                    [&](WSink& o) __attribute__((always_inline)) { write_remote(o, r, q); });
}

// The receiving daemons' tc argv, one thread per add entry with an UpdateRemote (add-list
// order), written at its message's index of the tc arena through the wave's LDS image (a
// separate launch: with the messages in one kernel the writer held 138 VGPRs, 3 waves per SIMD)
__global__ void __launch_bounds__(BLOCK) k_tc_remote_write(RemoteIn r, const uint64_t* off, uint8_t* arena) {
    __shared__ uint32_t img[BLOCK / 64][WIRE_IMG / 4];
    const uint32_t e = blockIdx.x * BLOCK + threadIdx.x;
    TcEntry te{0, 0, 0, 0, false};
    uint64_t s0 = 0, s1 = 0;
    if (e < r.n_add && (r.send[e] & REACH_SEND)) {
        te = tc_remote_entry(r, e);
        if (te.on) {
            const uint32_t m = r.rem_inv[e];
            s0 = off[m];
            s1 = off[m + 1];
        }
    }
    if (__ballot(s1 > s0) == 0) return;             // wave-uniform
    wave_segments_write(img[threadIdx.x >> 6], s1 > s0, s0, s1, arena,
                        [&](WSink& o) __attribute__((always_inline)) { write_tbf_argv(o, r.kd, te); });
}

}  // namespace kdtn
