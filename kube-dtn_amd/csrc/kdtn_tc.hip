// kdtn_tc.hip — `tc` argv synthesis for the TBF qdiscs.
//
// SetVethQdiscs (common/qdisc.go:201-290) adds netem over netlink and the TBF with
//   exec("tc", "qdisc", "add", "dev", <veth LinkName>, "parent", "1:1", "handle", "10:0",
//        "tbf", "rate", fmt.Sprint(Rate), "burst", fmt.Sprint(Buffer), "latency", "50ms",
//        "minburst", fmt.Sprint(Minburst))                                   (:252-266)
// ("parent 1:1 handle 10:0" because MakeQdiscs always puts the netem first). For every
// AddLinks / UpdateLinks entry whose MakeQdiscs produced a TBF and no error, this stage
// writes that argv (NUL-terminated arguments) for the entry's local interface
// (link.LocalIntf: the veth of UpdateLinks (handler.go:649-658), the local end of a
// same-node veth pair or VXLAN interface) and, for a same-node veth pair, for the peer end
// (link.PeerIntf, common/veth.go:53-60). Only entries the daemon reaches (k_reach: no
// earlier failing link in the topology's Del/Add/Update RPC sequence) run tc. Layout: two
// command slots per add entry, then one per update entry; slot g's argv =
// bytes[off[g], off[g+1]) (empty when it runs no tc command).
#include "kdtn_encode.h"

namespace kdtn {

KD_INLINE uint32_t ndigits(uint64_t v) {
    uint32_t n = 1;
    while (v >= 10u) { v /= 10u; ++n; }
    return n;
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

// command slot g: add entry g/2 (even: LocalIntf, odd: PeerIntf of a same-node veth pair),
// then update entry g - 2*n_add (LocalIntf)
KD_INLINE TcEntry tc_entry(const TcIn& w, uint32_t g) {
    TcEntry t{0, 0, 0, 0, false};
    const bool upd = g >= 2u * w.n_add;
    const uint32_t e = upd ? g - 2u * w.n_add : g >> 1;
    const bool peer_end = !upd && (g & 1u);
    if (((upd ? w.reach_upd : w.reach_add)[e] & REACH_ON) == 0) return t;   // batch aborted earlier
    const uint2* q = (upd ? w.upd_qdisc : w.add_qdisc) + (size_t)e * 9;
    const uint4 r = (upd ? w.upd_res : w.add_res)[e];
    const uint32_t flags = q[8].y;                         // has_netem | has_tbf<<8 | err<<16
    if (((flags >> 8) & 0xFFu) == 0 || ((flags >> 16) & 0xFFu) != 0 || ((r.w >> 8) & 0xFFu) != 0) return t;
    if (!upd) {                        // addLink sets qdiscs only on veth / VXLAN interfaces
        const uint32_t kind = r.w & 0xFFu;
        if (kind != KDTN_KIND_SAME_NODE && kind != KDTN_KIND_CROSS_NODE && kind != KDTN_KIND_PHYSICAL) return t;
        if (peer_end && kind != KDTN_KIND_SAME_NODE) return t;   // CreateVeth: both ends (veth.go:53-60)
    }
    const uint32_t j = (upd ? w.upd_idx : w.add_idx)[e];
    t.intf = w.N.key(peer_end ? KDTN_K_PEER_INTF : KDTN_K_LOCAL_INTF, j);
    t.buffer = q[6].y;                                     // kdtn_qdisc word 13
    t.rate = ((uint64_t)q[7].y << 32) | q[7].x;            // words 14, 15
    t.minburst = q[8].x;                                   // word 16
    t.on = true;
    return t;
}

__global__ void __launch_bounds__(BLOCK) k_tc_sizes(TcIn w, uint32_t* size) {
    const uint32_t g = blockIdx.x * BLOCK + threadIdx.x;
    if (g >= 2u * w.n_add + w.n_upd) return;
    const TcEntry t = tc_entry(w, g);
    size[g] = t.on ? TC_FIXED + (w.kd_offs[t.intf + 1] - w.kd_offs[t.intf]) + ndigits(t.rate) +
                         ndigits(t.buffer) + ndigits(t.minburst)
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
    const uint32_t l0 = (uint32_t)(v % 10000u);
    v /= 10000u;
    const uint32_t l1 = (uint32_t)(v % 10000u);
    v /= 10000u;
    const uint32_t l2 = (uint32_t)(v % 10000u);
    v /= 10000u;
    const uint32_t l3 = (uint32_t)(v % 10000u);
    const uint32_t l4 = (uint32_t)(v / 10000u);          // < 1845 (2^64 < 10^20)
    const int k = l4 ? 4 : l3 ? 3 : l2 ? 2 : l1 ? 1 : 0;
    const uint32_t top = k == 4 ? l4 : k == 3 ? l3 : k == 2 ? l2 : k == 1 ? l1 : l0;
    const uint32_t nd = ndigits(top);
    o.put(dig4(top) >> (8u * (4u - nd)), nd);
    if (k >= 4) o.put(dig4(l3), 4u);
    if (k >= 3) o.put(dig4(l2), 4u);
    if (k >= 2) o.put(dig4(l1), 4u);
    if (k >= 1) o.put(dig4(l0), 4u);
    o.byte(0u);
}

KD_INLINE void write_tbf_argv(WSink& o, const uint8_t* kd_bytes, const uint32_t* kd_offs, const TcEntry& t) {
    lit(o, "qdisc");
    lit(o, "add");
    lit(o, "dev");
    const uint32_t b = kd_offs[t.intf], len = kd_offs[t.intf + 1] - b;
    o.str(kd_bytes, b, len);
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

// slot g's argv at [off[g], off[g+1]): a wave's slots are one contiguous range (wave_image_write)
__global__ void __launch_bounds__(BLOCK) k_tc_write(TcIn w, const uint64_t* off, uint8_t* arena) {
    __shared__ uint32_t img[BLOCK / 64][WIRE_IMG / 4];
    const uint32_t g = blockIdx.x * BLOCK + threadIdx.x;
    TcEntry t{0, 0, 0, 0, false};
    uint64_t s0 = 0, s1 = 0;
    if (g < 2u * w.n_add + w.n_upd) {
        t = tc_entry(w, g);
        s0 = off[g];
        s1 = off[g + 1];
    }
    wave_image_write(img[threadIdx.x >> 6], t.on, s0, s1, arena,
                     [&](WSink& o) __attribute__((always_inline)) { write_tbf_argv(o, w.kd_bytes, w.kd_offs, t); });
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

// one thread per add entry (add-list order); the sizes are gathered into message order by
// k_remote_msg_sizes
__global__ void __launch_bounds__(BLOCK) k_tc_remote_entry_sizes(RemoteIn r, uint32_t* tsz_e) {
    const uint32_t e = blockIdx.x * BLOCK + threadIdx.x;
    if (e >= r.n_add || !(r.send[e] & REACH_SEND)) return;
    const TcEntry t = tc_remote_entry(r, e);
    tsz_e[e] = t.on ? TC_FIXED + (r.kd_offs[t.intf + 1] - r.kd_offs[t.intf]) + ndigits(t.rate) + ndigits(t.buffer) +
                          ndigits(t.minburst)
                    : 0u;
}

// one thread per add entry, writing its command at its message's position (add-list order;
// per-daemon runs stored through the wave's LDS image, wave_segments_write)
__global__ void __launch_bounds__(BLOCK) k_tc_remote_write(RemoteIn r, const uint64_t* off, uint8_t* arena) {
    __shared__ uint32_t img[BLOCK / 64][WIRE_IMG / 4];
    const uint32_t e = blockIdx.x * BLOCK + threadIdx.x;
    TcEntry t{0, 0, 0, 0, false};
    uint64_t s0 = 0, s1 = 0;
    if (e < r.n_add) {
        t = tc_remote_entry(r, e);
        if (t.on) {
            const uint32_t m = r.rem_inv[e];
            s0 = off[m];
            s1 = off[m + 1];
        }
    }
    if (__ballot(s1 > s0) == 0) return;             // wave-uniform
    wave_segments_write(img[threadIdx.x >> 6], s1 > s0, s0, s1, arena,
                        [&](WSink& o) __attribute__((always_inline)) { write_tbf_argv(o, r.kd_bytes, r.kd_offs, t); });
}

}  // namespace kdtn
