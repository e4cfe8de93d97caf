// kdtn_fanout.hip — RemotePod fan-out grouping.
//
// For every AddLinks entry that makes the daemon call UpdateRemote — classified
// CROSS_NODE (handler.go:419-453), its qdisc built (SetupVxLan → MakeQdiscs,
// daemon/vxlan/vxlan.go:40, fails before the RPC) and REACHED: no earlier link of its batch,
// and no DelLinks entry of its topology, failed (handler.go:601-607,
// topology_controller.go:93-106) — the RemotePod RPC goes to the peer's daemon at
// peer status.src_ip (common/utils.go:39-67). The reference sends one RPC per link; this
// stage groups them per destination daemon, so a caller can send one batch per node:
// nodes in ascending kdict-id order of their src_ip, entries of a node in add-list order.
//
// Kernels: k_reach_cuts / k_reach (entry-parallel RPC-order first-error rule, marks senders
// and their nodes in flag bytes per key-string id), k_fan_nodes_* (compaction of marked node ids → dense
// node index), k_fan_count / k_fan_scatter (single-wave workgroups over chunks of 4,096
// entries: LDS histogram, node-major scan of the (node, chunk) counts, stable scatter).
#include "kdtn_encode.h"

namespace kdtn {

// Which entries the daemons reach (include/kdtn.h): Reconcile sends each topology's
// DelLinks, AddLinks, UpdateLinks in that order (topology_controller.go:93-116) and each
// handler stops at its first failing link (handler.go:601-607, 622-628, 644-662). Entry-
// parallel in two launches, so a hub topology's thousands of entries are not walked by one
// thread: k_reach_cuts records per topology the first failing del, the first add that stops
// the batch (a failing link, or a cross-node link whose RemotePod the peer rejects — both
// reached themselves) and the first failing update (one atomicMin per such entry into
// cut[3t + list], 0xFFFFFFFF = none); k_reach then writes per add entry REACH_ON |
// REACH_SEND, per update entry REACH_ON, and (mark != nullptr) marks the destination
// daemon of every RemotePod sent.
__global__ void __launch_bounds__(BLOCK) k_reach_cuts(ReachIn f, uint32_t nd, uint32_t na, uint32_t nu, uint32_t* cut,
                                                      uint8_t* st_add) {
    const uint32_t x = blockIdx.x * BLOCK + threadIdx.x;
    if (x < nd) {
        if ((f.del_res[x].w >> 8) & 0xFFu) atomicMin(&cut[3 * entry_topo(f.del_off, f.T, x)], x);   // delLink error
    } else if (x < nd + na) {
        const uint32_t e = x - nd;
        const uint4 r = f.add_res[e];
        const uint32_t qe = f.add_qerr ? f.add_qerr[e] : qdisc_err(f.add_qdisc, e);
        const bool fails = add_fails(r, qe);
        if (fails || (r.w >> 24))                                            // or remote Update failed
            atomicMin(&cut[3 * entry_topo(f.add_off, f.T, e) + 1], e);
        st_add[e] = (!fails && sends_remote(r, qe)) ? REACH_SEND : 0;        // k_reach reads this byte
        if (f.add_node) f.add_node[e] = r.z;
    } else if (x < nd + na + nu) {
        const uint32_t e = x - nd - na;
        if ((f.upd_res[e].w >> 8) & 0xFFu) atomicMin(&cut[3 * entry_topo(f.upd_off, f.T, e) + 2], e);   // MakeVeth / MakeQdiscs
    }
}

__global__ void __launch_bounds__(BLOCK) k_reach(ReachIn f, uint32_t na, uint32_t nu, const uint32_t* cut,
                                                 const uint8_t* st_add, uint32_t* mark, uint8_t* reach_add,
                                                 uint8_t* reach_upd) {
    const uint32_t x = blockIdx.x * BLOCK + threadIdx.x;
    const uint32_t ta = entry_topo_wave_c(f.add_off, f.add_coarse, f.T, x, x < na);
    const uint32_t tu = entry_topo_wave_c(f.upd_off, f.upd_coarse, f.T, x - na, x >= na && x < na + nu);
    if (x < na) {
        const uint32_t t = ta;
        uint8_t a = 0;
        if (cut[3 * t] == 0xFFFFFFFFu && x <= cut[3 * t + 1]) {
            a = REACH_ON;
            if (st_add[x] & REACH_SEND) {               // no failure, RemotePod sent (k_reach_cuts)
                a |= REACH_SEND;
                // a flag byte per key-string id: a few dozen daemons take millions of marks, so
                // a flag is stored only while it reads clear (a stale read stores again,
                // harmlessly; plain stores: an atomic OR into shared bitmap words serialised)
                if (mark) {
                    const uint32_t node = f.add_node ? f.add_node[x] : f.add_res[x].z;
                    uint8_t* m = reinterpret_cast<uint8_t*>(mark);
                    if (!m[node]) m[node] = 1;
                }
            }
        }
        reach_add[x] = a;
    } else if (x < na + nu) {
        const uint32_t e = x - na;
        const uint32_t t = tu;
        reach_upd[e] = (cut[3 * t] == 0xFFFFFFFFu && cut[3 * t + 1] == 0xFFFFFFFFu && e <= cut[3 * t + 2]) ? REACH_ON : 0;
    }
}

__global__ void __launch_bounds__(BLOCK) k_list_coarse(const uint32_t* offs, uint32_t T, uint32_t* coarse) {
    const uint32_t t = blockIdx.x * BLOCK + threadIdx.x;
    if (t >= T) return;
    const uint32_t a = offs[t], b = offs[t + 1];
    for (uint32_t w = (a + 63u) >> 6; (w << 6) < b; ++w) coarse[w] = t;   // groups starting in t
}

// nonzero flag bytes of a marked node id's word: bit 8k of the result = byte k is set
KD_INLINE uint32_t flag_bytes(uint32_t w) { return ((w | (w >> 1) | (w >> 2) | (w >> 3) | (w >> 4) | (w >> 5) | (w >> 6) | (w >> 7)) & 0x01010101u); }

// marked node ids (flag bytes, read as words of four) → dense node indices in id order (chunks of
// SCAN_CHUNK words)
__global__ void __launch_bounds__(BLOCK) k_fan_nodes_count(const uint32_t* mark, uint32_t nw, uint64_t* part) {
    __shared__ uint64_t sh[BLOCK / 64];
    const uint32_t b0 = blockIdx.x * SCAN_CHUNK + threadIdx.x * 4;
    uint64_t v = 0;
#pragma unroll
    for (int k = 0; k < 4; ++k) v += b0 + k < nw ? __popc(flag_bytes(mark[b0 + k])) : 0u;
    uint64_t tot;
    block_exclusive(v, sh, &tot);
    if (threadIdx.x == 0) part[blockIdx.x] = tot;
}

__global__ void __launch_bounds__(BLOCK) k_fan_nodes_write(const uint32_t* mark, uint32_t nw, const uint64_t* part,
                                                           uint32_t* node_idx, uint32_t* nodes, uint32_t* n_nodes) {
    __shared__ uint64_t sh[BLOCK / 64];
    const uint32_t b0 = blockIdx.x * SCAN_CHUNK + threadIdx.x * 4;
    uint32_t m[4];
    uint64_t v = 0;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        m[k] = b0 + k < nw ? flag_bytes(mark[b0 + k]) : 0u;
        v += __popc(m[k]);
    }
    uint64_t tot;
    uint64_t x = part[blockIdx.x] + block_exclusive(v, sh, &tot);
#pragma unroll
    for (int k = 0; k < 4; ++k)
        for (uint32_t w = m[k]; w; w &= w - 1u) {
            const uint32_t id = (b0 + k) * 4u + ((uint32_t)__builtin_ctz(w) >> 3);
            node_idx[id] = (uint32_t)x;
            nodes[x] = id;
            ++x;
        }
    if (blockIdx.x == gridDim.x - 1 && threadIdx.x == 0) *n_nodes = (uint32_t)(part[blockIdx.x] + tot);
}

// (node, chunk) counts: one wave per chunk of FAN_CHUNK entries, LDS histogram
__global__ void __launch_bounds__(64) k_fan_count(FanIn f, const uint8_t* send, const uint32_t* node_idx,
                                                  const uint32_t* n_nodes, uint32_t* counts, uint32_t nchunks) {
    extern __shared__ uint32_t h[];                          // [n_nodes] (dynamic: occupancy)
    const uint32_t nn = *n_nodes;
    if (nn > FAN_NODE_CAP) return;                          // reported by the host
    for (uint32_t k = threadIdx.x; k < nn; k += 64) h[k] = 0;
    __syncthreads();
    const uint32_t c = blockIdx.x, e0 = c * FAN_CHUNK, e1 = min(e0 + FAN_CHUNK, f.n_add);
    // every round's loads first (two dependent levels for the chunk instead of per round)
    constexpr int RND = FAN_CHUNK / 64;
    uint32_t z[RND];
#pragma unroll
    for (int r = 0; r < RND; ++r) {
        const uint32_t e = e0 + r * 64 + threadIdx.x;
        z[r] = (e < e1 && (send[e] & REACH_SEND)) ? (f.add_node ? f.add_node[e] : f.add_res[e].z) : 0xFFFFFFFFu;
    }
#pragma unroll
    for (int r = 0; r < RND; ++r)
        if (z[r] != 0xFFFFFFFFu) z[r] = node_idx[z[r]];
#pragma unroll
    for (int r = 0; r < RND; ++r)
        if (z[r] != 0xFFFFFFFFu) atomicAdd(&h[z[r]], 1u);
    __syncthreads();
    for (uint32_t k = threadIdx.x; k < nn; k += 64) counts[(size_t)k * nchunks + c] = h[k];
}

// stable scatter: rounds of 64 entries in order. Within a round, the lanes that share a
// node find each other with one ballot per bit of the dense node index (mask = lanes whose
// index agrees on every bit), so a lane's rank among them is a popcount of the lower lanes;
// a running per-node counter in LDS carries the order across rounds.
__global__ void __launch_bounds__(64) k_fan_scatter(FanIn f, const uint8_t* send, const uint32_t* node_idx,
                                                    const uint32_t* n_nodes, const uint64_t* base, uint32_t nchunks,
                                                    uint32_t* out_idx, uint32_t* out_inv) {
    extern __shared__ uint32_t run[];                        // [n_nodes]
    const uint32_t nn = *n_nodes;
    if (nn > FAN_NODE_CAP) return;
    const uint32_t c = blockIdx.x, e0 = c * FAN_CHUNK, e1 = min(e0 + FAN_CHUNK, f.n_add);
    for (uint32_t k = threadIdx.x; k < nn; k += 64) run[k] = (uint32_t)base[(size_t)k * nchunks + c];
    __syncthreads();
    const int lane = threadIdx.x;
    const uint64_t lt = lane == 0 ? 0ull : (~0ull >> (64 - lane));
    const int nbits = nn > 1 ? 32 - __clz((int)(nn - 1)) : 0;
    constexpr int RND = FAN_CHUNK / 64;
    uint32_t z[RND];                                         // every round's node first
#pragma unroll
    for (int q = 0; q < RND; ++q) {
        const uint32_t e = e0 + q * 64 + lane;
        z[q] = (e < e1 && (send[e] & REACH_SEND)) ? (f.add_node ? f.add_node[e] : f.add_res[e].z) : 0xFFFFFFFFu;
    }
#pragma unroll
    for (int q = 0; q < RND; ++q)
        if (z[q] != 0xFFFFFFFFu) z[q] = node_idx[z[q]];
#pragma unroll
    for (int q = 0; q < RND; ++q) {
        const uint32_t e = e0 + q * 64 + lane;
        const bool on = z[q] != 0xFFFFFFFFu;
        const uint32_t node = on ? z[q] : 0u;
        const uint64_t act = __ballot(on);
        if (!act) continue;                                  // wave-uniform
        uint64_t same = act;
        for (int b = 0; b < nbits; ++b) {
            const bool bit = (node >> b) & 1u;
            const uint64_t m = __ballot(on && bit);
            same &= bit ? m : ~m;
        }
        const uint32_t b0 = on ? run[node] : 0u;
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
        const uint32_t rank = (uint32_t)__popcll(same & lt);
        if (on && rank == 0) run[node] = b0 + (uint32_t)__popcll(same);
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
        if (on) {
            out_idx[b0 + rank] = e;
            out_inv[e] = b0 + rank;                          // the entry's message index
        }
    }
}

}  // namespace kdtn
