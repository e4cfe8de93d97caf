// kdtn_state.hip — device-resident epoch state across reconciles (SURVEY §8(a2) commit,
// §8(b) ownership): the Topology status commit and the delta upload.
//
// Reconcile ends, for a Topology whose batches all succeeded (or that it saw for the first
// time), with Status.Links = Spec.Links (controllers/topology_controller.go:125-138); one that
// failed returns before the status write and keeps its old status. kdtn_epoch_commit applies
// that to the resident link stores: the realised store is rebuilt from the desired segments
// of the committed Topologies and the realised segments of the others, on the GPU, so the
// next epoch needs no realised upload at all. kdtn_epoch_upload_delta then replaces the
// desired segments of the Topologies whose spec changed: each new record is either a
// reference to a record of the previous desired store or an inline record of the delta, so
// the host link carries only what changed.
//
// Both are one "assemble" pass: every output record of Topology t comes from a per-topology
// source — a contiguous segment of store A, of store B, or a list of record references
// (A record, or B record with ASM_B) — with new offsets from a scan of the lengths.
#include "kdtn_encode.h"

namespace kdtn {

// commit plan: committed Topologies take their desired segment (B), the others keep their
// realised one (A). cut: k_reach_cuts' first failing entry per (topology, list), NONE = none;
// mask (optional): the caller's commit decision per topology.
__global__ void __launch_bounds__(BLOCK) k_commit_plan(DevTopos T, const uint8_t* action, const uint32_t* cut,
                                                       const uint8_t* mask, uint32_t* len, uint32_t* base,
                                                       uint8_t* mode, uint8_t* flags_out, uint32_t* n_commit) {
    const uint32_t t = blockIdx.x * BLOCK + threadIdx.x;
    bool commit = false;
    if (t < T.n) {
        const uint8_t a = action[t];
        if (mask) commit = mask[t] != 0;
        else if (a == KDTN_ACT_CREATED) commit = true;                         // :81-85, then :136
        else if (a == KDTN_ACT_DIFF)                                           // every RPC succeeded
            commit = cut[3 * t] == 0xFFFFFFFFu && cut[3 * t + 1] == 0xFFFFFFFFu && cut[3 * t + 2] == 0xFFFFFFFFu;
        const uint8_t fl = T.flags[t];
        if (commit) {
            len[t] = T.des_off[t + 1] - T.des_off[t];
            base[t] = T.des_off[t];
            mode[t] = ASM_SEG_B;
            // Status.Links = Spec.Links: a nil spec makes the status nil
            flags_out[t] = (uint8_t)((fl & ~KDTN_TOPO_STATUS_NIL) | ((fl & KDTN_TOPO_SPEC_NIL) ? KDTN_TOPO_STATUS_NIL : 0));
        } else {
            len[t] = T.real_off[t + 1] - T.real_off[t];
            base[t] = T.real_off[t];
            mode[t] = ASM_SEG_A;
            flags_out[t] = fl;
        }
    }
    // the count: one atomic per block into one of 32 counters (one atomic per wave on a single
    // word serialised the launch: 181 µs for 1M topologies)
    __shared__ uint32_t wsum[BLOCK / 64];
    const uint64_t m = __ballot(commit);
    if ((threadIdx.x & 63) == 0) wsum[threadIdx.x >> 6] = (uint32_t)__popcll(m);
    __syncthreads();
    if (threadIdx.x == 0) {
        uint32_t n = 0;
#pragma unroll
        for (int w = 0; w < BLOCK / 64; ++w) n += wsum[w];
        if (n) atomicAdd(n_commit + (blockIdx.x & 31u), n);
    }
}

// Every Topology committed (kdtn_epoch_commit with an all-ones mask): Status.Links = Spec.Links
// for all of them, so the realised store becomes the desired store as it stands and only the
// status-nil flags change (a nil spec makes the status nil).
__global__ void __launch_bounds__(BLOCK) k_commit_all_flags(uint8_t* flags, uint32_t T) {
    const uint32_t t = blockIdx.x * BLOCK + threadIdx.x;
    if (t >= T) return;
    const uint8_t fl = flags[t];
    flags[t] = (uint8_t)((fl & ~KDTN_TOPO_STATUS_NIL) | ((fl & KDTN_TOPO_SPEC_NIL) ? KDTN_TOPO_STATUS_NIL : 0));
}

// delta plan: changed Topologies (chg[t] = index into the delta, NONE = unchanged) take their
// reference list; the others keep their previous desired segment. Changed rows also take
// their new status.src_ip / status.net_ns / spec-nil bit.
__global__ void __launch_bounds__(BLOCK) k_delta_plan(DevTopos T, const uint32_t* chg, const uint32_t* d_off,
                                                      const uint32_t* d_src, const uint32_t* d_netns,
                                                      const uint8_t* d_nil, uint32_t* len, uint32_t* base,
                                                      uint8_t* mode, uint32_t* src_ip, uint32_t* net_ns,
                                                      uint8_t* flags, uint32_t* row_list, uint32_t* row_n) {
    const uint32_t t = blockIdx.x * BLOCK + threadIdx.x;
    if (t >= T.n) return;
    const uint32_t c = chg[t];
    if (c == 0xFFFFFFFFu) {
        len[t] = T.des_off[t + 1] - T.des_off[t];
        base[t] = T.des_off[t];
        mode[t] = ASM_SEG_A;
        return;
    }
    len[t] = d_off[c + 1] - d_off[c];
    base[t] = d_off[c];
    mode[t] = ASM_REF;
    const uint8_t fl = flags[t];
    const uint8_t nfl = (uint8_t)((fl & ~KDTN_TOPO_SPEC_NIL) | (d_nil[c] ? KDTN_TOPO_SPEC_NIL : 0));
    if (src_ip[t] != d_src[c] || net_ns[t] != d_netns[c] || fl != nfl)
        row_list[atomicAdd(row_n, 1u)] = t;            // a changed pod-status row (any order)
    src_ip[t] = d_src[c];
    net_ns[t] = d_netns[c];
    flags[t] = nfl;
}

__global__ void __launch_bounds__(BLOCK) k_delta_map(const uint32_t* topo, uint32_t n, uint32_t* chg) {
    const uint32_t c = blockIdx.x * BLOCK + threadIdx.x;
    if (c < n) chg[topo[c]] = c;
}

// u64 exclusive offsets (k_scan_final) → the u32 offsets of a topology table
__global__ void __launch_bounds__(BLOCK) k_off_narrow(const uint64_t* in, uint32_t n, uint32_t* out) {
    const uint32_t i = blockIdx.x * BLOCK + threadIdx.x;
    if (i <= n) out[i] = (uint32_t)in[i];
}

KD_INLINE void copy_record(const uint32_t* sbase, uint32_t j, uint32_t* dbase, uint32_t d) {
    const uint32_t* src = sbase + (size_t)(j >> 6) * TILE_WORDS + (j & 63u);
    uint32_t* dst = dbase + (size_t)(d >> 6) * TILE_WORDS + (d & 63u);
    uint32_t v[LINK_COLS32];
#pragma unroll
    for (int c = 0; c < LINK_COLS32; ++c) v[c] = src[c * TILE_RECS];
    const int64_t u = reinterpret_cast<const int64_t*>(sbase + (size_t)(j >> 6) * TILE_WORDS + LINK_COLS32 * TILE_RECS)[j & 63u];
#pragma unroll
    for (int c = 0; c < LINK_COLS32; ++c) dst[c * TILE_RECS] = v[c];
    reinterpret_cast<int64_t*>(dbase + (size_t)(d >> 6) * TILE_WORDS + LINK_COLS32 * TILE_RECS)[d & 63u] = u;
}

// one thread per output record d: its topology by binary search over the new offsets, then
// one record copied from the plan's source (coalesced within a segment: consecutive outputs
// read consecutive source records)
__global__ void __launch_bounds__(BLOCK) k_store_assemble(const uint32_t* off, uint32_t nt, const uint32_t* base,
                                                          const uint8_t* mode, const uint32_t* ref, DevLinks A,
                                                          DevLinks B, uint32_t n, uint32_t* out) {
    const uint32_t d = blockIdx.x * BLOCK + threadIdx.x;
    const uint32_t t = entry_topo_wave(off, nt, d, d < n);   // (all lanes: wave-cooperative)
    if (d >= n) return;
    const uint32_t k = base[t] + (d - off[t]);
    const uint8_t m = mode[t];
    if (m == ASM_SEG_A) copy_record(A.base, k, out, d);
    else if (m == ASM_SEG_B) copy_record(B.base, k, out, d);
    else {
        const uint32_t r = ref[k];
        if (r & KDTN_DELTA_NEW) copy_record(B.base, r & ~KDTN_DELTA_NEW, out, d);
        else copy_record(A.base, r, out, d);
    }
}

// Link-store upload from SoA columns: the host columns arrive by linear copies into a staging
// buffer (stage + c*n: the 7 key, 12 property and gap columns; the uid column after them), and
// this pass writes the 64-record tiles (coalesced on both sides) and takes the maximum of every
// id column (colmax[0..18]) for the range check the host makes before the upload is accepted.
__global__ void __launch_bounds__(BLOCK) k_soa_to_tiles(const uint32_t* stage, const int64_t* uid, uint32_t n,
                                                        uint32_t* out, uint32_t* colmax) {
    __shared__ uint32_t red[BLOCK / 64][COL_GAP];
    uint32_t mx[COL_GAP];
#pragma unroll
    for (int c = 0; c < COL_GAP; ++c) mx[c] = 0;
    for (uint32_t i = blockIdx.x * BLOCK + threadIdx.x; i < n; i += gridDim.x * BLOCK) {
        uint32_t* dst = out + (size_t)(i >> 6) * TILE_WORDS + (i & 63u);
#pragma unroll
        for (int c = 0; c < LINK_COLS32; ++c) {
            const uint32_t v = __builtin_nontemporal_load(stage + (size_t)c * n + i);
            if (c < COL_GAP) mx[c] = v > mx[c] ? v : mx[c];
            dst[c * TILE_RECS] = v;
        }
        reinterpret_cast<int64_t*>(out + (size_t)(i >> 6) * TILE_WORDS + LINK_COLS32 * TILE_RECS)[i & 63u] =
            __builtin_nontemporal_load(uid + i);
    }
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
#pragma unroll
    for (int c = 0; c < COL_GAP; ++c) {
        uint32_t v = mx[c];
#pragma unroll
        for (int d = 32; d >= 1; d >>= 1) {
            const uint32_t o = __shfl_xor(v, d, 64);
            v = o > v ? o : v;
        }
        if (lane == 0) red[wave][c] = v;
    }
    __syncthreads();
    if (threadIdx.x < COL_GAP) {
        uint32_t v = 0;
#pragma unroll
        for (int w = 0; w < BLOCK / 64; ++w) v = red[w][threadIdx.x] > v ? red[w][threadIdx.x] : v;
        atomicMax(colmax + threadIdx.x, v);
    }
}

// Pod-status rows of the Topologies a delta changed (status.src_ip / net_ns / spec nil), as
// {pod index, 0, 0, 0}, row entries; entries past n are padding (pod index ~0). Exchanged
// between ranks instead of the whole table when the tables of the previous rows are resident.
__global__ void __launch_bounds__(BLOCK) k_pods_pack(DevTopos T, const uint32_t* topo, uint32_t n, uint32_t cap,
                                                     uint32_t rank_base, uint4* out) {
    const uint32_t k = blockIdx.x * BLOCK + threadIdx.x;
    if (k >= cap) return;
    if (k >= n) {
        out[2 * k] = make_uint4(0xFFFFFFFFu, 0u, 0u, 0u);
        return;
    }
    const uint32_t t = topo[k];
    out[2 * k] = make_uint4(rank_base + t, 0u, 0u, 0u);
    out[2 * k + 1] = make_uint4(T.ns[t], T.name[t], T.src_ip[t],
                                T.net_ns[t] | ((T.flags[t] & KDTN_TOPO_SPEC_NIL) ? 0x80000000u : 0u));
}

// Apply changed rows to the resident pod table and to their pods' direct lookup slots (the
// slot of the pod's name when this pod owns it in the current build; a name shared by several
// pods is answered from the overflow table, which reads the row itself). The name, its
// namespace and the PHYSICAL bit of the name string do not change.
__global__ void __launch_bounds__(BLOCK) k_pods_patch(const uint4* ent, uint32_t n, uint4* pods, uint4* slots,
                                                      uint32_t stamp, uint32_t nd) {
    const uint32_t k = blockIdx.x * BLOCK + threadIdx.x;
    if (k >= n) return;
    const uint32_t g = ent[2 * k].x;
    if (g == 0xFFFFFFFFu) return;
    const uint4 row = ent[2 * k + 1];
    pods[g] = row;
    if (row.y >= nd) return;
    const uint4 w = slots[row.y];
    if ((w.w >> 1) != stamp || (w.w & 1u) || (w.y >> 2) != g) return;
    slots[row.y] = make_uint4(w.x, (g << 2) | (w.y & 2u) | (row.w >> 31),
                              row.z | ((row.w & 0x7FFFFFFFu) == 0 ? 0x80000000u : 0u), w.w);
}

}  // namespace kdtn
