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

// wave-OR of an error word, one atomic per wave
KD_INLINE void delta_err(uint32_t e, uint32_t* err) {
#pragma unroll
    for (int d = 32; d >= 1; d >>= 1) e |= __shfl_xor(e, d, 64);
    if ((threadIdx.x & 63) == 0 && e) atomicOr(err, e);
}

// delta plan, one thread per topology t of the NEW table: changed Topologies (chg[t] = index
// into the delta, NONE = unchanged) take their reference list, the others their previous
// desired segment. With a topology map (prev) every row comes from its previous row or, for a
// created Topology, from the delta (ns / name; status.links nil, no realised records), and the
// realised plan (rlen / rbase) carries each kept Topology's status segment to its new position;
// a previous index named twice or out of range, or a created Topology absent from the changed
// list, is an error. Without a map (identity) a changed row whose pod-status fields move is
// listed for the resident pod-table patch. New columns go to `out` (the state is untouched
// until the host accepts the delta).
__global__ void __launch_bounds__(BLOCK) k_delta_plan(DeltaPlanIn in, DeltaPlanOut o) {
    if (*o.err) return;                             // k_delta_check refused the delta's arrays
    const uint32_t t = blockIdx.x * BLOCK + threadIdx.x;
    uint32_t e = 0;
    if (t < in.n_topos) {
        const DevTopos& T = in.T0;
        const uint32_t c = in.chg[t];
        uint32_t p = t;
        if (in.prev) {
            p = in.prev[t];
            if (p != KDTN_DELTA_NEW) {
                if (p >= T.n) {
                    e |= DERR_PREV;
                    p = KDTN_DELTA_NEW;
                } else if (atomicOr(o.seen + (p >> 5), 1u << (p & 31u)) & (1u << (p & 31u))) {
                    e |= DERR_PREV;                                  // named twice
                }
            } else if (c == 0xFFFFFFFFu) {
                e |= DERR_NEW;                                       // created without a spec
            }
        }
        uint32_t ns = 0, name = 0, src = 0, netns = 0, dlen = 0, dbase = 0, rlen = 0, rbase = 0;
        uint8_t fl = KDTN_TOPO_STATUS_NIL, mode = ASM_SEG_A;
        if (p != KDTN_DELTA_NEW) {
            ns = T.ns[p];
            name = T.name[p];
            src = T.src_ip[p];
            netns = T.net_ns[p];
            fl = T.flags[p];
            dbase = T.des_off[p];
            dlen = T.des_off[p + 1] - dbase;
            rbase = T.real_off[p];
            rlen = T.real_off[p + 1] - rbase;
        } else if (c != 0xFFFFFFFFu) {
            ns = in.d_ns[c];
            name = in.d_name[c];
            if (ns >= in.D || name >= in.D) e |= DERR_IDS;
        }
        if (c != 0xFFFFFFFFu) {
            dbase = in.d_off[c];
            dlen = in.d_off[c + 1] - dbase;
            mode = ASM_REF;
            const uint8_t nfl = (uint8_t)((fl & ~KDTN_TOPO_SPEC_NIL) | (in.d_nil[c] ? KDTN_TOPO_SPEC_NIL : 0));
            if (!in.prev && (src != in.d_src[c] || netns != in.d_netns[c] || fl != nfl))
                o.row_list[atomicAdd(o.row_n, 1u)] = t;              // a changed pod-status row (any order)
            src = in.d_src[c];
            netns = in.d_netns[c];
            fl = nfl;
        }
        o.dlen[t] = dlen;
        o.dbase[t] = dbase;
        o.dmode[t] = mode;
        o.src_ip[t] = src;
        o.net_ns[t] = netns;
        o.flags[t] = fl;
        if (in.prev) {
            o.ns[t] = ns;
            o.name[t] = name;
            o.rlen[t] = rlen;
            o.rbase[t] = rbase;
        }
    }
    delta_err(e, o.err);
}

__global__ void __launch_bounds__(BLOCK) k_delta_map(const uint32_t* topo, uint32_t n, uint32_t T, uint32_t* chg) {
    const uint32_t c = blockIdx.x * BLOCK + threadIdx.x;
    if (c < n && topo[c] < T) chg[topo[c]] = c;
}

// The delta's arrays checked on the GPU instead of host loops: thread i checks changed entry i
// (topology index in range and strictly ascending, offsets monotone, a nil spec without
// records, status ids in the dictionary) and references i, i + grid, ... (previous record in
// range, inline record in range); thread 0 also compares the kept dictionaries' arena offsets
// with the ones the resident state was parsed from (before this call's upload overwrites them).
__global__ void __launch_bounds__(BLOCK) k_delta_check(DeltaCheckIn in, uint32_t* err) {
    const uint32_t i = blockIdx.x * BLOCK + threadIdx.x;
    uint32_t e = 0;
    if (i < in.n) {
        const uint32_t t = in.topo[i];
        if (t >= in.n_topos || (i && t <= in.topo[i - 1])) e |= DERR_TOPO;
        if (in.off[i + 1] < in.off[i]) e |= DERR_OFF;
        if (in.nil[i] && in.off[i + 1] != in.off[i]) e |= DERR_NIL;
        if (in.src[i] >= in.D || in.netns[i] >= in.D) e |= DERR_IDS;
    }
    for (uint32_t k = i; k < in.nref; k += gridDim.x * BLOCK) {
        const uint32_t r = in.ref[k];
        if ((r & KDTN_DELTA_NEW) ? (r & ~KDTN_DELTA_NEW) >= in.n_new : r >= in.n_old) e |= DERR_REF;
    }
    if (i == 0) {
        if (in.kd_keep && in.kd_offs[in.kd_keep] != in.kd_expect) e |= DERR_KEEP;
        if (in.pd_keep && in.pd_offs[in.pd_keep] != in.pd_expect) e |= DERR_KEEP;
    }
    delta_err(e, err);
}

// the totals the host reads back with the delta's one synchronisation
__global__ void k_delta_totals(const uint64_t* doff, uint32_t Tn, const uint64_t* roff, uint32_t* misc) {
    if (threadIdx.x != 0) return;
    const uint64_t n = doff[Tn], m = roff ? roff[Tn] : 0ull;
    misc[MISC_DELTA_N] = (uint32_t)n;
    misc[MISC_DELTA_N + 1] = (uint32_t)(n >> 32);
    misc[MISC_DELTA_M] = (uint32_t)m;
    misc[MISC_DELTA_M + 1] = (uint32_t)(m >> 32);
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
// read consecutive source records). Delta uploads (g != NULL): n bounds the grid and the exact
// count is the one the offsets' scan left on the device (no host readback first); nothing is
// copied when the delta was refused (its references are not trusted); with skip_new the
// inline records (still in flight over the host link) are left to k_delta_inline.
__global__ void __launch_bounds__(BLOCK) k_store_assemble(const uint32_t* off, uint32_t nt, const uint32_t* base,
                                                          const uint8_t* mode, const uint32_t* ref, DevLinks A,
                                                          DevLinks B, uint32_t n, AsmGuard g, uint32_t* out) {
    if (g.err) {
        if (*g.err) return;
        const uint64_t m = *g.n_dev;
        n = m < n ? (uint32_t)m : n;
    }
    const uint32_t d = blockIdx.x * BLOCK + threadIdx.x;
    const uint32_t t = entry_topo_wave(off, nt, d, d < n);   // (all lanes: wave-cooperative)
    if (d >= n) return;
    const uint32_t k = base[t] + (d - off[t]);
    const uint8_t m = mode[t];
    if (m == ASM_SEG_A) copy_record(A.base, k, out, d);
    else if (m == ASM_SEG_B) copy_record(B.base, k, out, d);
    else if (!g.skip_ref) {
        const uint32_t r = ref[k];
        if (r & KDTN_DELTA_NEW) {
            if (!g.skip_new) copy_record(B.base, r & ~KDTN_DELTA_NEW, out, d);
        } else {
            copy_record(A.base, r, out, d);
        }
    }
}

// The reference lists of a delta once they have arrived (k_store_assemble placed the kept
// segments meanwhile): one thread per reference k, its changed Topology c (wave-cooperative
// search over the delta's offsets), output position off[topo[c]] + (k - d_off[c]); a previous
// record is copied there, an inline record's position goes to dest (k_delta_place writes the
// record when its columns have arrived; a record referenced twice raises `multi`).
__global__ void __launch_bounds__(BLOCK) k_delta_refs(const uint32_t* d_off, const uint32_t* topo, uint32_t n,
                                                      const uint32_t* ref, uint32_t nref, const uint32_t* off,
                                                      DevLinks A, const uint32_t* err, uint32_t* dest,
                                                      uint32_t* multi, uint32_t* out) {
    if (*err) return;                                  // (wave-uniform: the search below is cooperative)
    const uint32_t k = blockIdx.x * BLOCK + threadIdx.x;
    const uint32_t c = entry_topo_wave(d_off, n, k, k < nref);
    if (k >= nref) return;
    const uint32_t r = ref[k];
    const uint32_t d = off[topo[c]] + (k - d_off[c]);
    if (r & KDTN_DELTA_NEW) {
        if (atomicExch(dest + (r & ~KDTN_DELTA_NEW), d) != 0xFFFFFFFFu) atomicOr(multi, 1u);
    } else {
        copy_record(A.base, r, out, d);
    }
}

// Inline records of a delta from the staging columns (k_soa_to_tiles' input) straight to their
// positions in the new desired store, plus the id-range column maxima; unreferenced records
// (dest ~0) are skipped. Nothing is written when the delta was refused. One launch per staged
// copy: columns [c0, c1) (and the uid column when with_uid), so each group of columns is placed
// as soon as its copy has arrived while the next group still crosses the host link.
__global__ void __launch_bounds__(BLOCK) k_delta_place(const uint32_t* stage, const int64_t* uid, uint32_t n,
                                                       const uint32_t* dest, const uint32_t* err, uint32_t* out,
                                                       uint32_t* colmax, uint32_t c0, uint32_t c1, uint32_t with_uid) {
    __shared__ uint32_t red[BLOCK / 64][COL_GAP];
    uint32_t mx[COL_GAP];
#pragma unroll
    for (int c = 0; c < COL_GAP; ++c) mx[c] = 0;
    const bool ok = *err == 0;
    for (uint32_t i = blockIdx.x * BLOCK + threadIdx.x; i < n; i += gridDim.x * BLOCK) {
        const uint32_t d = ok ? dest[i] : 0xFFFFFFFFu;
        uint32_t* dst = out + (size_t)(d >> 6) * TILE_WORDS + (d & 63u);
#pragma unroll
        for (int c = 0; c < LINK_COLS32; ++c) {
            if ((uint32_t)c < c0 || (uint32_t)c >= c1) continue;
            const uint32_t v = __builtin_nontemporal_load(stage + (size_t)c * n + i);
            if (c < COL_GAP) mx[c] = v > mx[c] ? v : mx[c];
            if (d != 0xFFFFFFFFu) dst[c * TILE_RECS] = v;
        }
        if (with_uid && d != 0xFFFFFFFFu)
            reinterpret_cast<int64_t*>(out + (size_t)(d >> 6) * TILE_WORDS + LINK_COLS32 * TILE_RECS)[d & 63u] =
                __builtin_nontemporal_load(uid + i);
    }
    if (c0 >= (uint32_t)COL_GAP) return;                 // no id column in this launch
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
#pragma unroll
    for (int c = 0; c < COL_GAP; ++c) {
        uint32_t v = mx[c];
#pragma unroll
        for (int dd = 32; dd >= 1; dd >>= 1) {
            const uint32_t o = __shfl_xor(v, dd, 64);
            v = o > v ? o : v;
        }
        if (lane == 0) red[wave][c] = v;
    }
    __syncthreads();
    if (threadIdx.x >= c0 && threadIdx.x < c1 && threadIdx.x < (uint32_t)COL_GAP) {
        uint32_t v = 0;
#pragma unroll
        for (int w = 0; w < BLOCK / 64; ++w) v = red[w][threadIdx.x] > v ? red[w][threadIdx.x] : v;
        atomicMax(colmax + threadIdx.x, v);
    }
}

// The general placement when an inline record is referenced more than once (k_delta_refs'
// multi flag): one thread per reference k, records from the tiles of the staged delta.
__global__ void __launch_bounds__(BLOCK) k_delta_inline(const uint32_t* d_off, const uint32_t* topo, uint32_t n,
                                                        const uint32_t* ref, uint32_t nref, const uint32_t* off,
                                                        DevLinks B, const uint32_t* err, uint32_t* out) {
    if (*err) return;
    const uint32_t k = blockIdx.x * BLOCK + threadIdx.x;
    if (k >= nref) return;
    const uint32_t r = ref[k];
    if (!(r & KDTN_DELTA_NEW)) return;
    const uint32_t c = entry_topo(d_off, n, k);
    copy_record(B.base, r & ~KDTN_DELTA_NEW, out, off[topo[c]] + (k - d_off[c]));
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
