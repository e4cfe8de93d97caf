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
#include "kdtn_kernels.h"

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

struct Out {
    uint8_t* p;
    KD_INLINE void lit(const char* s) {
        while (*s) *p++ = (uint8_t)*s++;
        *p++ = 0;
    }
    KD_INLINE void num(uint64_t v) {
        const uint32_t n = ndigits(v);
        for (uint32_t k = n; k-- > 0;) {
            p[k] = (uint8_t)('0' + v % 10u);
            v /= 10u;
        }
        p += n;
        *p++ = 0;
    }
};

KD_INLINE void write_tbf_argv(Out& o, const uint8_t* kd_bytes, const uint32_t* kd_offs, const TcEntry& t) {
    o.lit("qdisc");
    o.lit("add");
    o.lit("dev");
    const uint32_t b = kd_offs[t.intf], len = kd_offs[t.intf + 1] - b;
    for (uint32_t k = 0; k < len; ++k) *o.p++ = kd_bytes[b + k];
    *o.p++ = 0;
    o.lit("parent");
    o.lit("1:1");
    o.lit("handle");
    o.lit("10:0");
    o.lit("tbf");
    o.lit("rate");
    o.num(t.rate);
    o.lit("burst");
    o.num(t.buffer);
    o.lit("latency");
    o.lit("50ms");
    o.lit("minburst");
    o.num(t.minburst);
}

__global__ void __launch_bounds__(BLOCK) k_tc_write(TcIn w, const uint64_t* off, uint8_t* arena) {
    const uint32_t g = blockIdx.x * BLOCK + threadIdx.x;
    if (g >= 2u * w.n_add + w.n_upd) return;
    const TcEntry t = tc_entry(w, g);
    if (!t.on) return;
    Out o{arena + off[g]};
    write_tbf_argv(o, w.kd_bytes, w.kd_offs, t);
}

// The receiving daemon's TBF command for RemotePod message m (m < n_remote): the peer
// daemon's Update runs SetupVxLan on link.PeerIntf → MakeQdiscs (the same properties, which
// built on the sending side) → SetVethQdiscs (daemon/vxlan/vxlan.go:31-51), unless its
// CreateOrUpdate rejects IntfIp (kdtn_resolved.remote_err). Physical messages have none here
// (their tc runs on LocalIntf: kdtn_epoch_tc slot 2e).
KD_INLINE TcEntry tc_remote_entry(const RemoteIn& r, uint32_t m) {
    TcEntry t{0, 0, 0, 0, false};
    if (m >= r.n_remote) return t;
    const uint32_t e = r.rem_idx[m];
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

__global__ void __launch_bounds__(BLOCK) k_tc_remote_sizes(RemoteIn r, uint32_t* size) {
    const uint32_t m = blockIdx.x * BLOCK + threadIdx.x;
    if (m >= r.n_msgs) return;
    const TcEntry t = tc_remote_entry(r, m);
    size[m] = t.on ? TC_FIXED + (r.kd_offs[t.intf + 1] - r.kd_offs[t.intf]) + ndigits(t.rate) + ndigits(t.buffer) +
                         ndigits(t.minburst)
                   : 0u;
}

__global__ void __launch_bounds__(BLOCK) k_tc_remote_write(RemoteIn r, const uint64_t* off, uint8_t* arena) {
    const uint32_t m = blockIdx.x * BLOCK + threadIdx.x;
    if (m >= r.n_msgs) return;
    const TcEntry t = tc_remote_entry(r, m);
    if (!t.on) return;
    Out o{arena + off[m]};
    write_tbf_argv(o, r.kd_bytes, r.kd_offs, t);
}

}  // namespace kdtn
