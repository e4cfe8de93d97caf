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
    size[g] = tc_size(w.kd, t);
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
                     [&](WSink& o) __attribute__((always_inline)) { write_tbf_argv(o, w.kd, t); });
}

}  // namespace kdtn
