// kdtn_vni.hip — VxlanManager state after the epoch (include/kdtn.h kdtn_epoch_vni_apply).
//
// The daemons' maps change as the reached entries run: delLink deletes VNI 5000+uid on the
// local node when the map holds the local pod's netns there (handler.go:484-487); a
// cross-node addLink stores (vni, local netns) on the local node after SetupVxLan
// (:440) and the peer daemon's Update stores (vni, peer netns) on the peer's node
// (:192, reached unless remote_err); a physical peer's local Update stores (vni, local netns)
// (:355-371 → :192). Map ops are sync.Map Store / Delete (daemon/vxlan/manager.go:57-63).
// Deterministic order (the reference's is goroutine order): every delete first, then every
// add; per key the first add in (topology, add-list, local-before-remote) order wins.
//
// Order dependence (kdtn_vni_contested): a key's result depends on the goroutine order when
// two entries Store different netns values under it, or when an entry Stores exactly the netns
// a reached delLink of the same key compares Get(vni) against (delete-then-store keeps it,
// store-then-delete removes it). k_vni_dtab_insert puts every reached delete {node, vni,
// netns} in a table, k_vni_contest flags the winning add of each such key, and the flags are
// compacted in the winners' order.
//
// Kernels: k_vni_cuts / k_vni_ops (entry-parallel: where each topology's RPC sequence stops,
// then one op slot per del entry and two per add entry), k_vni_shadow / k_vni_del (snapshot entries that are not,
// or no longer, in the map: shadowed duplicates, deleted keys), then the
// new map as a first-wins table over [add ops, surviving snapshot entries] (k_vni_insert)
// and its visible entries compacted in that order (k_vni_vis_count / k_scan_top /
// k_vni_vis_write).
#include "kdtn_encode.h"

namespace kdtn {

// Where each topology's RPC sequence stops (reach rule of k_reach, entry-parallel so a hub
// topology's thousands of entries are not walked by one thread): cut[2t] = the first DelLinks
// entry with a MakeVeth error, cut[2t + 1] = the first AddLinks entry not reached (a failing
// entry, or the one after a rejected RemotePod). 0xFFFFFFFF = none (memset).
__global__ void __launch_bounds__(BLOCK) k_vni_cuts(VniOpsIn f, uint32_t* cut) {
    const uint32_t x = blockIdx.x * BLOCK + threadIdx.x;
    if (x < f.n_del) {
        if ((f.r.del_res[x].w >> 8) & 0xFFu) atomicMin(&cut[2 * entry_topo(f.r.del_off, f.r.T, x)], x);
    } else if (x < f.n_del + f.n_add) {
        const uint32_t e = x - f.n_del;
        const uint4 r = f.r.add_res[e];
        uint32_t c = 0xFFFFFFFFu;
        if (add_fails(r, qdisc_err(f.r.add_qdisc, e))) c = e;
        else if ((r.w & 0xFFu) == KDTN_KIND_CROSS_NODE && (r.w >> 24)) c = e + 1;   // remote Update failed
        if (c != 0xFFFFFFFFu) atomicMin(&cut[2 * entry_topo(f.r.add_off, f.r.T, e) + 1], c);
    }
}

// One thread per entry: a del entry before its topology's del cut deletes on a vni_hit; an
// add entry of a topology whose dels all succeeded, before the add cut, stores (vni, local
// netns) on the local node (cross-node, physical) and, cross-node without remote_err,
// (vni, peer netns) on the peer's node.
__global__ void __launch_bounds__(BLOCK) k_vni_ops(VniOpsIn f, const uint32_t* cut, uint4* ops) {
    const uint32_t x = blockIdx.x * BLOCK + threadIdx.x;
    const uint4 none = make_uint4(0u, 0u, 0u, VOP_NONE);
    const uint32_t td = entry_topo_wave(f.r.del_off, f.r.T, x, x < f.n_del);
    const uint32_t ta = entry_topo_wave(f.r.add_off, f.r.T, x - f.n_del, x >= f.n_del && x < f.n_del + f.n_add);
    if (x < f.n_del) {
        const uint32_t t = td;
        const uint4 r = f.r.del_res[x];
        uint4 op = none;
        if (x < cut[2 * t])                                                  // reached; vni_hit :484-487
            op = make_uint4(f.t_src[t], r.y, f.t_netns[t], ((r.w >> 16) & 0xFFu) ? VOP_DEL : VOP_DEL_MISS);
        ops[x] = op;
    } else if (x < f.n_del + f.n_add) {
        const uint32_t e = x - f.n_del;
        const uint32_t t = ta;
        uint4 lo = none, rm = none;
        if (cut[2 * t] == 0xFFFFFFFFu && e < cut[2 * t + 1]) {
            const uint4 r = f.r.add_res[e];
            const uint32_t kind = r.w & 0xFFu;
            if (kind == KDTN_KIND_CROSS_NODE || kind == KDTN_KIND_PHYSICAL)
                lo = make_uint4(f.t_src[t], r.y, f.t_netns[t], VOP_ADD);       // :440 / :192
            if (kind == KDTN_KIND_CROSS_NODE && (r.w >> 24) == 0)
                rm = make_uint4(r.z, r.y, f.pods[r.x].w & 0x7FFFFFFFu, VOP_ADD);   // peer node :192
        }
        uint4* aops = ops + f.n_del;
        aops[2 * (size_t)e] = lo;
        aops[2 * (size_t)e + 1] = rm;
    }
}

// slot of key (node, vni) in the snapshot table (entries ents[slots[h]]), or 0xFFFFFFFF
KD_INLINE uint32_t vni_find(const uint4* ents, const uint32_t* slots, uint32_t mask, uint32_t node, uint32_t vni) {
    for (uint32_t h = vni_home(node, vni, mask);; h = (h + 1) & mask) {
        const uint32_t s = slots[h];
        if (s == 0xFFFFFFFFu) return s;
        const uint4 e = ents[s];
        if (e.x == node && e.y == vni) return s;
    }
}

__global__ void __launch_bounds__(BLOCK) k_vni_del(const uint4* ops, uint32_t n_del, const uint4* ents,
                                                   const uint32_t* slots, uint32_t mask, uint8_t* dead) {
    const uint32_t j = blockIdx.x * BLOCK + threadIdx.x;
    if (j >= n_del) return;
    const uint4 op = ops[j];
    if (op.w != VOP_DEL || mask == 0) return;
    const uint32_t i = vni_find(ents, slots, mask, op.x, op.y);
    if (i != 0xFFFFFFFFu) dead[i] = 1;
}

// snapshot entries shadowed by an earlier entry of the same key (first wins) are not in the map
__global__ void __launch_bounds__(BLOCK) k_vni_shadow(const uint4* ents, uint32_t n_ents, const uint32_t* slots,
                                                      uint32_t mask, uint8_t* dead) {
    const uint32_t i = blockIdx.x * BLOCK + threadIdx.x;
    if (i >= n_ents) return;
    const uint4 e = ents[i];
    dead[i] = vni_find(ents, slots, mask, e.x, e.y) != i;
}

// Extended entry x: add op x (x < n_ops) or snapshot entry x - n_ops; present = an add op,
// or a snapshot entry that is the visible one of its key (the snapshot's own first wins)
// and was not deleted.
KD_INLINE bool ext_entry(const uint4* add_ops, uint32_t n_ops, const uint4* ents, const uint8_t* dead, uint32_t x,
                         uint4* e) {
    if (x < n_ops) {
        *e = add_ops[x];
        return e->w == VOP_ADD;
    }
    const uint32_t i = x - n_ops;
    *e = ents[i];
    return !dead[i];
}

__global__ void __launch_bounds__(BLOCK) k_vni_insert(const uint4* add_ops, uint32_t n_ops, const uint4* ents,
                                                      const uint8_t* dead, uint32_t n_ents, uint32_t* slots,
                                                      uint32_t mask) {
    const uint32_t x = blockIdx.x * BLOCK + threadIdx.x;
    if (x >= n_ops + n_ents) return;
    uint4 e;
    if (!ext_entry(add_ops, n_ops, ents, dead, x, &e)) return;
    for (uint32_t h = vni_home(e.x, e.y, mask);; h = (h + 1) & mask) {
        const uint32_t prev = atomicCAS(&slots[h], 0xFFFFFFFFu, x);
        if (prev == 0xFFFFFFFFu) return;
        uint4 o;
        ext_entry(add_ops, n_ops, ents, dead, prev, &o);
        if (o.x == e.x && o.y == e.y) {
            atomicMin(&slots[h], x);                  // first in extended order wins
            return;
        }
    }
}

KD_INLINE bool ext_visible(const uint4* add_ops, uint32_t n_ops, const uint4* ents, const uint8_t* dead, uint32_t n_ents,
                           const uint32_t* slots, uint32_t mask, uint32_t x, uint4* e) {
    if (x >= n_ops + n_ents || !ext_entry(add_ops, n_ops, ents, dead, x, e)) return false;
    for (uint32_t h = vni_home(e->x, e->y, mask);; h = (h + 1) & mask) {
        const uint32_t s = slots[h];
        if (s == 0xFFFFFFFFu) return false;
        uint4 o;
        ext_entry(add_ops, n_ops, ents, dead, s, &o);
        if (o.x == e->x && o.y == e->y) return s == x;
    }
}

// Visible entries per scan chunk; each entry's visibility is kept as a byte (vis) for the
// write pass, so the table is probed once per entry.
__global__ void __launch_bounds__(BLOCK) k_vni_vis_count(const uint4* add_ops, uint32_t n_ops, const uint4* ents,
                                                         const uint8_t* dead, uint32_t n_ents, const uint32_t* slots,
                                                         uint32_t mask, uint8_t* vis, uint64_t* part) {
    __shared__ uint64_t sh[BLOCK / 64];
    const uint32_t b0 = blockIdx.x * SCAN_CHUNK + threadIdx.x * 4;
    uint64_t v = 0;
    uint4 e;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        const bool m = ext_visible(add_ops, n_ops, ents, dead, n_ents, slots, mask, b0 + k, &e);
        if (b0 + k < n_ops + n_ents) vis[b0 + k] = m;
        v += m ? 1u : 0u;
    }
    uint64_t tot;
    block_exclusive(v, sh, &tot);
    if (threadIdx.x == 0) part[blockIdx.x] = tot;
}

__global__ void __launch_bounds__(BLOCK) k_vni_vis_write(const uint4* add_ops, uint32_t n_ops, const uint4* ents,
                                                         const uint8_t* dead, uint32_t n_ents, const uint8_t* vis,
                                                         const uint64_t* part, uint32_t* node, int32_t* vni,
                                                         uint32_t* net_ns, uint32_t* n_out) {
    __shared__ uint64_t sh[BLOCK / 64];
    const uint32_t b0 = blockIdx.x * SCAN_CHUNK + threadIdx.x * 4;
    bool m[4];
    uint4 e[4];
    uint64_t v = 0;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        m[k] = b0 + k < n_ops + n_ents && vis[b0 + k];
        if (m[k]) ext_entry(add_ops, n_ops, ents, dead, b0 + k, &e[k]);
        v += m[k] ? 1u : 0u;
    }
    uint64_t tot;
    uint64_t x = part[blockIdx.x] + block_exclusive(v, sh, &tot);
#pragma unroll
    for (int k = 0; k < 4; ++k)
        if (m[k]) {
            node[x] = e[k].x;
            vni[x] = (int32_t)e[k].y;
            net_ns[x] = e[k].z;
            ++x;
        }
    if (blockIdx.x == gridDim.x - 1 && threadIdx.x == 0) *n_out = (uint32_t)(part[blockIdx.x] + tot);
}

// every reached delete (hit or miss) as a key {node, vni, netns} (duplicates allowed)
__global__ void __launch_bounds__(BLOCK) k_vni_dtab_insert(const uint4* dels, uint32_t n_del, uint4* dkeys,
                                                           uint32_t* dused, uint32_t dmask) {
    const uint32_t j = blockIdx.x * BLOCK + threadIdx.x;
    if (j >= n_del) return;
    const uint4 d = dels[j];
    if (d.w != VOP_DEL && d.w != VOP_DEL_MISS) return;
    for (uint32_t h = (uint32_t)hash64(((uint64_t)d.x << 32) ^ ((uint64_t)d.y << 16) ^ d.z) & dmask;;
         h = (h + 1) & dmask) {
        if (atomicCAS(&dused[h], 0u, 1u) == 0u) {
            dkeys[h] = make_uint4(d.x, d.y, d.z, 0u);
            return;
        }
    }
}

KD_INLINE bool dtab_has(const uint4* dkeys, const uint32_t* dused, uint32_t dmask, uint32_t node, uint32_t vni,
                        uint32_t netns) {
    if (dmask == 0) return false;
    for (uint32_t h = (uint32_t)hash64(((uint64_t)node << 32) ^ ((uint64_t)vni << 16) ^ netns) & dmask;;
         h = (h + 1) & dmask) {
        if (!dused[h]) return false;
        const uint4 k = dkeys[h];
        if (k.x == node && k.y == vni && k.z == netns) return true;
    }
}

// One thread per add op: flag the winning add of its key when this op stores another netns
// than the winner, or stores the netns a reached delete of the key compares against.
__global__ void __launch_bounds__(BLOCK) k_vni_contest(const uint4* add_ops, uint32_t n_ops, const uint4* ents,
                                                       const uint8_t* dead, const uint32_t* slots, uint32_t mask,
                                                       const uint4* dkeys, const uint32_t* dused, uint32_t dmask,
                                                       uint32_t* flag) {
    const uint32_t x = blockIdx.x * BLOCK + threadIdx.x;
    if (x >= n_ops) return;
    const uint4 op = add_ops[x];
    if (op.w != VOP_ADD) return;
    uint32_t w = 0xFFFFFFFFu;                          // the key's winner (an add op: adds come first)
    for (uint32_t h = vni_home(op.x, op.y, mask);; h = (h + 1) & mask) {
        const uint32_t sl = slots[h];
        if (sl == 0xFFFFFFFFu) break;
        uint4 o;
        ext_entry(add_ops, n_ops, ents, dead, sl, &o);
        if (o.x == op.x && o.y == op.y) {
            w = sl;
            break;
        }
    }
    if (w >= n_ops) return;                            // (cannot happen: x itself was inserted)
    const bool other = w != x && add_ops[w].z != op.z;
    if (other || dtab_has(dkeys, dused, dmask, op.x, op.y, op.z)) flag[w] = 1u;
}

__global__ void __launch_bounds__(BLOCK) k_vni_contest_write(const uint4* add_ops, const uint32_t* flag,
                                                             const uint64_t* pos, uint32_t n_ops, uint32_t* node,
                                                             int32_t* vni) {
    const uint32_t x = blockIdx.x * BLOCK + threadIdx.x;
    if (x >= n_ops || !flag[x]) return;
    const uint4 op = add_ops[x];
    node[pos[x]] = op.x;
    vni[pos[x]] = (int32_t)op.y;
}

}  // namespace kdtn
