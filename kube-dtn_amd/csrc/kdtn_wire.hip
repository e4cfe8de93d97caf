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
//   k_utf8_bits      unicode/utf8.ValidString per dictionary string → bitset (1 = invalid)
//   k_str_table      {offset, length | STR_BAD} per dictionary string (STR_BAD: not valid
//                    UTF-8, unicode/utf8.ValidString)
//   k_wire_entry_sizes  one thread per entry: its topology and encoded size (its Link, plus
//                    the LocalPod header for a batch's first entry); a string that is not
//                    valid UTF-8 fails its batch (err bit)
//   k_wire_scan_*    exclusive scan of the sizes of entries whose batch marshals → u64 arena
//                    offset of every entry; k_wire_batch_off: batch offsets [3T+1]
//   k_wire_write     one thread per entry: writes its bytes into the wave's LDS image (dwords
//                    assembled in registers, WSink), which the wave then stores with
//                    coalesced dword stores
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

__global__ void __launch_bounds__(BLOCK) k_utf8_bits(const uint8_t* bytes, const uint32_t* offs,
                                                     uint32_t n, uint32_t* bits) {
    const uint32_t i = blockIdx.x * BLOCK + threadIdx.x;
    bool bad = false;
    if (i < n) {
        const uint32_t b = offs[i], len = offs[i + 1] - b;
        bool ascii = true;
        for (uint32_t k = 0; k < len && ascii; ++k) ascii = bytes[b + k] < 0x80u;
        if (!ascii) bad = !utf8_ok(bytes + b, len);
    }
    const uint64_t m = __ballot(bad);
    const int lane = threadIdx.x & 63;
    if (lane == 0 || lane == 32) bits[((i - lane) >> 5) + (lane >> 5)] = lane ? (uint32_t)(m >> 32) : (uint32_t)m;
}

// {offset, length | STR_BAD} per dictionary string (the encoders' one gather per string field).
// The high-bit test reads the string's first 32 bytes as one 16-B load pair (+ a dword)
// instead of byte by byte; only strings with a byte >= 0x80 run the UTF-8 automaton. (16-B
// entries holding strings of <= 12 bytes inline measured slower: wire_write 1.83 vs 1.77 ms,
// sizes 0.72 vs 0.63 ms — the table doubles and the writer loses a wave per SIMD,
// profiles/r03k_stages.json.)
__global__ void __launch_bounds__(BLOCK) k_str_table(const uint8_t* bytes, const uint32_t* offs, uint32_t n,
                                                     uint2* tab) {
    const uint32_t i = blockIdx.x * BLOCK + threadIdx.x;
    if (i >= n) return;
    const uint32_t b = offs[i], len = offs[i + 1] - b;
    uint32_t hi = 0;
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
                const uint32_t m = r >= 4u ? 0x80808080u : (0x80808080u & ((1u << (8u * r)) - 1u));
                hi |= __builtin_amdgcn_alignbyte(w[q + 1], w[q], sh) & m;
            }
        }
        for (uint32_t k = 32; k < len; ++k) hi |= bytes[b + k] & 0x80u;
    }
    const bool bad = hi != 0 && !utf8_ok(bytes + b, len);
    tab[i] = make_uint2(b, len | (bad ? STR_BAD : 0u));
}

// ---- sizes ---------------------------------------------------------------------------------
KD_INLINE uint32_t vlen(uint64_t v) {
    uint32_t n = 1;
    while (v >= 0x80u) { v >>= 7; ++n; }
    return n;
}
KD_INLINE uint32_t str_field(uint32_t len) { return len ? 1u + vlen(len) + len : 0u; }
KD_INLINE bool bit(const uint32_t* bits, uint32_t id) { return (bits[id >> 5] >> (id & 31)) & 1u; }
KD_INLINE uint32_t slen(SRef r) { return r.y & ~STR_BAD; }
// string-table entry of id (id 0 = "": no gather); FULL = false: the length word only (sizes)
template <bool FULL = true>
KD_INLINE SRef sref(const SRef* tab, uint32_t id) {
    if (!id) return make_uint2(0u, 0u);
    if constexpr (FULL) return tab[id];
    else return make_uint2(0u, reinterpret_cast<const uint32_t*>(tab)[2 * (size_t)id + 1]);
}

// the table entries of one Link record's 7 key and 12 property strings, gathered at once
struct LinkRefs {
    SRef k[KDTN_NKEY], p[KDTN_NPROP];
    uint32_t gap;
    int64_t uid;
};
template <bool FULL = true>
KD_INLINE LinkRefs link_refs(const SRef* kd_tab, const SRef* pd_tab, const DevLinks& L, uint32_t j) {
    LinkRefs r;
#pragma unroll
    for (int k = 0; k < KDTN_NKEY; ++k) r.k[k] = sref<FULL>(kd_tab, L.key(k, j));
#pragma unroll
    for (int k = 0; k < KDTN_NPROP; ++k) r.p[k] = sref<FULL>(pd_tab, L.prop(k, j));
    r.gap = L.gap(j);
    r.uid = L.uid(j);
    return r;
}
// pb.LinkProperties size (psz) and pb.Link size (lsz); false if a string is invalid UTF-8
KD_INLINE bool link_sizes(const LinkRefs& r, uint32_t* psz, uint32_t* lsz) {
    uint32_t bad = 0, p = 0, l = 0;
#pragma unroll
    for (int k = 0; k < KDTN_NPROP; ++k) {
        p += str_field(slen(r.p[k]));
        bad |= r.p[k].y;
    }
    if (r.gap) p += 1u + vlen(r.gap);
#pragma unroll
    for (int k = 0; k < KDTN_NKEY; ++k) {
        l += str_field(slen(r.k[k]));
        bad |= r.k[k].y;
    }
    if (r.uid) l += 1u + vlen((uint64_t)r.uid);
    l += 1u + vlen(p) + p;
    *psz = p;
    *lsz = l;
    return (bad & STR_BAD) == 0;
}

KD_INLINE uint32_t pod_size(const WireIn& w, uint32_t t, bool* ok) {
    const uint32_t ids[4] = {w.t_name[t], w.t_src[t], w.t_netns[t], w.t_ns[t]};
    uint32_t s = 0, bad = 0;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        const SRef r = sref<false>(w.kd_tab, ids[k]);
        s += str_field(slen(r));
        bad |= r.y;
    }
    *ok = (bad & STR_BAD) == 0;
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
            const uint32_t tl = entry_topo_wave(w.list_off[l], w.T, e, lst == l);
            if (lst == l) t = tl;
        }
    if (!on) return;
    uint32_t psz, lsz;
    bool ok = link_sizes(link_refs<false>(w.kd_tab, w.pd_tab, lst == 0 ? O : N, w.list_idx[lst][e]), &psz, &lsz);
    uint32_t size = 1u + vlen(lsz) + lsz;
    if (e == w.list_off[lst][t]) {                         // the batch's first entry carries the header
        bool pok;
        const uint32_t ps = pod_size(w, t, &pok);
        ok = ok && pok;
        size += 1u + vlen(ps) + ps;
    }
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
// string field: tag, length, bytes
KD_INLINE void str_field_out(WSink& o, uint32_t field, const uint8_t* arena, SRef r) {
    const uint32_t len = slen(r);
    if (!len) return;
    if (len < 0x80u) {
        o.put((field << 3 | 2u) | (len << 8), 2u);
    } else {
        o.byte(field << 3 | 2u);
        o.varint(len);
    }
    o.str(arena, r.x, len);
}

// one entry's bytes from its gathered string ranges r (and sizes psz / lsz)
KD_INLINE void write_entry_refs(WSink& o, const WireIn& w, const LinkRefs& r, uint32_t psz, uint32_t lsz, bool header,
                                uint32_t t) {
    if (header) {                                         // LinksBatchQuery.local_pod
        bool ok;
        o.byte(1u << 3 | 2u);
        o.varint(pod_size(w, t, &ok));
        str_field_out(o, 1, w.kd_bytes, sref(w.kd_tab, w.t_name[t]));
        str_field_out(o, 2, w.kd_bytes, sref(w.kd_tab, w.t_src[t]));
        str_field_out(o, 3, w.kd_bytes, sref(w.kd_tab, w.t_netns[t]));
        str_field_out(o, 4, w.kd_bytes, sref(w.kd_tab, w.t_ns[t]));
    }
    o.byte(2u << 3 | 2u);                                 // LinksBatchQuery.links
    o.varint(lsz);
    // pb.Link fields in number order: peer_pod 1, local_intf 2, peer_intf 3, local_ip 4,
    // peer_ip 5, uid 6, properties 7, local_mac 8, peer_mac 9
    str_field_out(o, 1, w.kd_bytes, r.k[KDTN_K_PEER_POD]);
    str_field_out(o, 2, w.kd_bytes, r.k[KDTN_K_LOCAL_INTF]);
    str_field_out(o, 3, w.kd_bytes, r.k[KDTN_K_PEER_INTF]);
    str_field_out(o, 4, w.kd_bytes, r.k[KDTN_K_LOCAL_IP]);
    str_field_out(o, 5, w.kd_bytes, r.k[KDTN_K_PEER_IP]);
    if (r.uid) {
        o.byte(6u << 3);
        o.varint((uint64_t)r.uid);
    }
    o.byte(7u << 3 | 2u);
    o.varint(psz);
    // pb.LinkProperties: latency 1 .. rate 6, gap 7, duplicate 8 .. corrupt_corr 13 (KDTN_P_* order)
#pragma unroll
    for (int k = 0; k < KDTN_NPROP; ++k) {
        if (k == KDTN_P_DUPLICATE && r.gap) {
            o.byte(7u << 3);
            o.varint(r.gap);
        }
        str_field_out(o, (uint32_t)(k < KDTN_P_DUPLICATE ? k + 1 : k + 2), w.pd_bytes, r.p[k]);
    }
    str_field_out(o, 8, w.kd_bytes, r.k[KDTN_K_LOCAL_MAC]);
    str_field_out(o, 9, w.kd_bytes, r.k[KDTN_K_PEER_MAC]);
}

KD_INLINE void write_entry(WSink& o, const WireIn& w, const DevLinks& L, uint32_t j, bool header, uint32_t t) {
    const LinkRefs r = link_refs(w.kd_tab, w.pd_tab, L, j);   // every string's range: one round trip
    uint32_t psz, lsz;
    link_sizes(r, &psz, &lsz);
    write_entry_refs(o, w, r, psz, lsz, header, t);
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

// the strings of message m as arena ranges, in field order net_ns, intf_name, intf_ip,
// peer_vtep, kube_ns, name, and the link's properties
struct RemoteMsg {
    SRef s[6], p[KDTN_NPROP];
    uint32_t gap;
    int32_t vni;
    bool ok;                        // every string valid UTF-8
};

// the strings of add entry e's message (remote: the UpdateRemote payload, else the physical
// peer's local Update payload); t = the entry's topology
template <bool FULL = true>
KD_INLINE RemoteMsg remote_msg(const RemoteIn& r, uint32_t e, uint32_t t, bool remote) {
    RemoteMsg q;
    const uint32_t j = r.add_idx[e];
    const uint4 res = r.add_res[e];
    const uint32_t peer_pod = r.N.key(KDTN_K_PEER_POD, j);
    uint32_t id[6];
    if (remote) {                                   // UpdateRemote: the peer daemon's side
        id[0] = r.pods[res.x].w & 0x7FFFFFFFu;      // peerPod.NetNs
        id[1] = r.N.key(KDTN_K_PEER_INTF, j);
        id[2] = r.N.key(KDTN_K_PEER_IP, j);
        id[3] = r.t_src[t];                         // localPod.SrcIp
    } else {                                        // physical: the local pod's side
        id[0] = r.t_netns[t];
        id[1] = r.N.key(KDTN_K_LOCAL_INTF, j);
        id[2] = r.N.key(KDTN_K_LOCAL_IP, j);
        id[3] = peer_pod;                           // TrimPrefix(PeerPod, "physical/") below
    }
    id[4] = r.t_ns[t];                              // localPod.KubeNs
    id[5] = peer_pod;
    uint32_t bad = 0;
#pragma unroll
    for (int k = 0; k < 6; ++k) {
        q.s[k] = sref<FULL>(r.kd_tab, id[k]);
        bad |= q.s[k].y;
    }
#pragma unroll
    for (int k = 0; k < KDTN_NPROP; ++k) {
        q.p[k] = sref<FULL>(r.pd_tab, r.N.prop(k, j));
        bad |= q.p[k].y;
    }
    if (!remote) {                                  // TrimPrefix(PeerPod, "physical/")
        q.s[3].x += 9u;
        q.s[3].y -= 9u;
    }
    q.gap = r.N.gap(j);
    q.vni = (int32_t)res.y;
    q.ok = (bad & STR_BAD) == 0;
    return q;
}

KD_INLINE uint32_t remote_body_size(const RemoteMsg& q, uint32_t* psz) {
    uint32_t n = 0, p = 0;
#pragma unroll
    for (int k = 0; k < 6; ++k) n += str_field(slen(q.s[k]));
    if (q.vni) n += 1u + vlen((uint64_t)(int64_t)q.vni);
#pragma unroll
    for (int k = 0; k < KDTN_NPROP; ++k) p += str_field(slen(q.p[k]));
    if (q.gap) p += 1u + vlen(q.gap);
    *psz = p;
    return n + 1u + vlen(p) + p;
}

// One thread per add entry (add-list order: the entry's columns are read coalesced): the
// size of its message, if it has one (0 when a string is not valid UTF-8).
__global__ void __launch_bounds__(BLOCK) k_remote_entry_sizes(RemoteIn r, uint32_t* msz_e) {
    const uint32_t e = blockIdx.x * BLOCK + threadIdx.x;
    const uint32_t kind = e < r.n_add ? remote_kind(r, e) : 0u;
    if (__ballot(kind != 0) == 0) return;           // wave-uniform
    const uint32_t t = entry_topo_wave(r.add_off, r.T, e, kind != 0);
    if (!kind) return;
    const RemoteMsg q = remote_msg<false>(r, e, t, kind == 1);
    uint32_t psz;
    const uint32_t body = remote_body_size(q, &psz);
    msz_e[e] = q.ok ? vlen(body) + body : 0u;
}

// message m's size from its add entry's (one gather per message, fan-out order)
__global__ void __launch_bounds__(BLOCK) k_remote_msg_sizes(RemoteIn r, const uint32_t* msz_e, const uint32_t* tsz_e,
                                                            uint32_t* msz, uint32_t* tsz) {
    const uint32_t m = blockIdx.x * BLOCK + threadIdx.x;
    if (m >= r.n_msgs) return;
    const bool remote = m < r.n_remote;
    const uint32_t e = remote ? r.rem_idx[m] : r.phys_idx[m - r.n_remote];
    msz[m] = msz_e[e];
    tsz[m] = remote ? tsz_e[e] : 0u;
}

KD_INLINE void write_remote(WSink& o, const RemoteIn& r, const RemoteMsg& q) {
    uint32_t psz;
    o.varint(remote_body_size(q, &psz));
#pragma unroll
    for (int k = 0; k < 5; ++k) str_field_out(o, (uint32_t)k + 1, r.kd_bytes, q.s[k]);
    if (q.vni) {
        o.byte(6u << 3);
        o.varint((uint64_t)(int64_t)q.vni);
    }
    o.byte(7u << 3 | 2u);
    o.varint(psz);
#pragma unroll
    for (int k = 0; k < KDTN_NPROP; ++k) {
        if (k == KDTN_P_DUPLICATE && q.gap) {
            o.byte(7u << 3);
            o.varint(q.gap);
        }
        str_field_out(o, (uint32_t)(k < KDTN_P_DUPLICATE ? k + 1 : k + 2), r.pd_bytes, q.p[k]);
    }
    str_field_out(o, 8, r.kd_bytes, q.s[5]);
}

// One thread per add entry with a message, in add-list order (its columns read coalesced),
// writing the message at its fan-out position. A wave's messages for one daemon are one
// contiguous run of the arena (fan-out order keeps add-list order within a daemon), so the
// wave stores them through its LDS image dword by dword (wave_segments_write).
__global__ void __launch_bounds__(BLOCK) k_remote_write(RemoteIn r, const uint64_t* off, uint8_t* arena) {
    __shared__ uint32_t img[BLOCK / 64][REMOTE_IMG / 4];
    const uint32_t e = blockIdx.x * BLOCK + threadIdx.x;
    const uint32_t kind = e < r.n_add ? remote_kind(r, e) : 0u;
    if (__ballot(kind != 0) == 0) return;           // wave-uniform
    const uint32_t t = entry_topo_wave(r.add_off, r.T, e, kind != 0);
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

}  // namespace kdtn
