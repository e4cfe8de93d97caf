// kdtn_kernels.hip — device code of the reconcile epoch. See kdtn_kernels.h for the
// data layout and launch order; DESIGN.md for the roofline accounting.
#include "kdtn_kernels.h"

namespace kdtn {

// ======================================================================================
// small helpers
// ======================================================================================
KD_INLINE uint32_t mix32(uint32_t h, uint32_t w) {
    h ^= w;
    h *= 0x85EBCA6Bu;
    h ^= h >> 13;
    return h;
}
KD_INLINE uint32_t fin32(uint32_t h) {
    h ^= h >> 16;
    h *= 0xC2B2AE35u;
    h ^= h >> 16;
    return h;
}
KD_INLINE uint64_t hash64(uint64_t x) {
    x ^= x >> 33;
    x *= 0xFF51AFD7ED558CCDull;
    x ^= x >> 33;
    x *= 0xC4CEB9FE1A85EC53ull;
    x ^= x >> 33;
    return x;
}

// 32-bit hash of the EqualWithoutProperties key (7 string ids + uid).
KD_INLINE uint32_t key_hash(const DevLinks& L, uint32_t i) {
    uint32_t h = 0x9E3779B9u;
#pragma unroll
    for (int k = 0; k < KDTN_NKEY; ++k) h = mix32(h, L.key[k][i]);
    uint64_t u = (uint64_t)L.uid[i];
    h = mix32(h, (uint32_t)u);
    h = mix32(h, (uint32_t)(u >> 32));
    return fin32(h);
}

// EqualWithoutProperties (controllers/topology_controller.go:342-351). Interned ids:
// equal ids ⇔ equal strings.
KD_INLINE bool key_eq(const DevLinks& A, uint32_t i, const DevLinks& B, uint32_t j) {
    bool eq = A.uid[i] == B.uid[j];
#pragma unroll
    for (int k = 0; k < KDTN_NKEY; ++k) eq = eq && (A.key[k][i] == B.key[k][j]);
    return eq;
}

// reflect.DeepEqual(old.Properties, new.Properties) (:294): 12 strings + Gap.
KD_INLINE bool props_eq(const DevLinks& A, uint32_t i, const DevLinks& B, uint32_t j) {
    bool eq = A.gap[i] == B.gap[j];
#pragma unroll
    for (int k = 0; k < KDTN_NPROP; ++k) eq = eq && (A.prop[k][i] == B.prop[k][j]);
    return eq;
}

// largest tt in [lo, hi) with off[tt] <= idx  (the segment containing idx)
KD_INLINE int find_seg(const uint32_t* off, int lo, int hi, uint32_t idx) {
    while (hi - lo > 1) {
        int mid = (lo + hi) >> 1;
        if (off[mid] <= idx) lo = mid;
        else hi = mid;
    }
    return lo;
}

KD_INLINE uint64_t lanemask_lt() {
    const int lane = threadIdx.x & 63;
    return lane == 0 ? 0ull : (~0ull >> (64 - lane));
}

// ======================================================================================
// dictionary parsing
// ======================================================================================
__global__ void __launch_bounds__(BLOCK) k_kdict_flags(const uint8_t* bytes, const uint32_t* offs,
                                                       uint32_t n, uint8_t* flags,
                                                       uint32_t* default_id) {
    uint32_t i = blockIdx.x * BLOCK + threadIdx.x;
    if (i >= n) return;
    const uint32_t b = offs[i], len = offs[i + 1] - b;
    const uint8_t* s = bytes + b;
    uint8_t f = 0;
    if (len) {
        if (!cidr_ok(s, len)) f |= KF_CIDR_BAD;   // common/veth.go:22
        if (!mac_ok(s, len)) f |= KF_MAC_BAD;     // common/veth.go:33
    }
    if (len == 9 && s[0] == 'l' && s[1] == 'o' && s[2] == 'c' && s[3] == 'a' && s[4] == 'l' &&
        s[5] == 'h' && s[6] == 'o' && s[7] == 's' && s[8] == 't')
        f |= KF_LOCALHOST;                        // common.Localhost (handler.go:333)
    if (len >= 9 && s[0] == 'p' && s[1] == 'h' && s[2] == 'y' && s[3] == 's' && s[4] == 'i' &&
        s[5] == 'c' && s[6] == 'a' && s[7] == 'l' && s[8] == '/')
        f |= KF_PHYSICAL;                         // handler.go:348
    if (len == 7 && s[0] == 'd' && s[1] == 'e' && s[2] == 'f' && s[3] == 'a' && s[4] == 'u' &&
        s[5] == 'l' && s[6] == 't')
        atomicMin(default_id, i);                 // getPod: ns "" → "default" (handler.go:29-31)
    flags[i] = f;
}

__global__ void __launch_bounds__(BLOCK) k_pdict_parse(const uint8_t* bytes, const uint32_t* offs,
                                                       uint32_t n, double tick, uint4* parsed,
                                                       uint64_t* rate) {
    uint32_t i = blockIdx.x * BLOCK + threadIdx.x;
    if (i >= n) return;
    const uint32_t b = offs[i], len = offs[i + 1] - b;
    const uint8_t* s = bytes + b;
    uint32_t fl = 0, dur = 0, ticks = 0, pu = 0;
    uint64_t r = 0;
    if (!parse_duration_us(s, len, &dur)) { fl |= PF_DUR_ERR; dur = 0; }
    else ticks = time2tick(dur, tick);
    float pct;
    if (!parse_pct(s, len, &pct)) fl |= PF_PCT_ERR;
    else pu = p2u(pct);
    if (!parse_rate(s, len, &r)) { fl |= PF_RATE_ERR; r = 0; }
    parsed[i] = make_uint4(pu, dur, ticks, fl);
    rate[i] = r;
}

// ======================================================================================
// pod-status table + hash tables
// ======================================================================================
__global__ void __launch_bounds__(BLOCK) k_pods_fill(DevTopos T, uint32_t slice, uint32_t rank_base,
                                                     uint4* pods) {
    uint32_t t = blockIdx.x * BLOCK + threadIdx.x;
    if (t >= slice) return;
    uint4 e;
    if (t < T.n) {
        e.x = T.ns[t];
        e.y = T.name[t];
        e.z = T.src_ip[t];
        e.w = T.net_ns[t] | ((T.flags[t] & KDTN_TOPO_SPEC_NIL) ? 0x80000000u : 0u);
    } else {
        e = make_uint4(0xFFFFFFFFu, 0xFFFFFFFFu, 0u, 0u);   // padding: never inserted
    }
    pods[rank_base + t] = e;
}

__global__ void __launch_bounds__(BLOCK) k_pod_ht_build(const uint4* pods, uint32_t total,
                                                        uint64_t* keys, uint32_t* vals,
                                                        uint32_t mask) {
    uint32_t g = blockIdx.x * BLOCK + threadIdx.x;
    if (g >= total) return;
    const uint4 e = pods[g];
    if (e.x == 0xFFFFFFFFu) return;
    const uint64_t key = ((uint64_t)e.x << 32) | e.y;
    uint32_t h = (uint32_t)hash64(key) & mask;
    for (;;) {
        unsigned long long prev = atomicCAS((unsigned long long*)&keys[h], ~0ull, (unsigned long long)key);
        if (prev == ~0ull || prev == key) {
            atomicMin(&vals[h], g);                 // informer store: first topology wins
            return;
        }
        h = (h + 1) & mask;
    }
}

__global__ void __launch_bounds__(BLOCK) k_vni_ht_build(const uint32_t* node, const int32_t* vni,
                                                        uint32_t n, uint64_t* keys, uint32_t* vals,
                                                        uint32_t mask) {
    uint32_t v = blockIdx.x * BLOCK + threadIdx.x;
    if (v >= n) return;
    const uint64_t key = ((uint64_t)node[v] << 32) | (uint32_t)vni[v];
    uint32_t h = (uint32_t)hash64(key) & mask;
    for (;;) {
        unsigned long long prev = atomicCAS((unsigned long long*)&keys[h], ~0ull, (unsigned long long)key);
        if (prev == ~0ull || prev == key) {
            atomicMin(&vals[h], v);
            return;
        }
        h = (h + 1) & mask;
    }
}

KD_INLINE uint32_t pod_lookup(const DevTables& tb, uint32_t ns, uint32_t name) {
    if (ns == 0xFFFFFFFFu) return 0xFFFFFFFFu;
    const uint64_t key = ((uint64_t)ns << 32) | name;
    uint32_t h = (uint32_t)hash64(key) & tb.pod_mask;
    for (;;) {
        const uint64_t k = tb.pod_keys[h];
        if (k == key) return tb.pod_vals[h];
        if (k == ~0ull) return 0xFFFFFFFFu;
        h = (h + 1) & tb.pod_mask;
    }
}

// VxlanManager.Get(vni) on node `node`: net_ns id, or 0xFFFFFFFF when absent.
KD_INLINE uint32_t vni_lookup(const DevTables& tb, uint32_t node, int32_t vni) {
    if (tb.vni_mask == 0) return 0xFFFFFFFFu;
    const uint64_t key = ((uint64_t)node << 32) | (uint32_t)vni;
    uint32_t h = (uint32_t)hash64(key) & tb.vni_mask;
    for (;;) {
        const uint64_t k = tb.vni_keys[h];
        if (k == key) return tb.vni_netns[tb.vni_vals[h]];
        if (k == ~0ull) return 0xFFFFFFFFu;
        h = (h + 1) & tb.vni_mask;
    }
}

// ======================================================================================
// k_diff: Reconcile gate + CalcDiff, one workgroup per TPW consecutive topologies.
// ======================================================================================
struct DiffShared {
    uint32_t ooff[TPW + 1];
    uint32_t noff[TPW + 1];
    uint8_t tflag[TPW];
    uint8_t dirty[TPW];
    uint8_t act[TPW];
    uint32_t cnt[3];
    uint32_t hash[CAP];
    uint8_t flag[CAP];
    uint8_t lt[CAP];
};

// need element comparisons: both lists non-nil and non-empty
KD_INLINE bool need_cmp(const DiffShared& sh, int tt) {
    return (sh.tflag[tt] & (KDTN_TOPO_STATUS_NIL | KDTN_TOPO_SPEC_NIL)) == 0 &&
           sh.ooff[tt + 1] > sh.ooff[tt] && sh.noff[tt + 1] > sh.noff[tt];
}

// Process the topologies [tb, te) of this workgroup as one window. hsh/flg hold the
// window's records (old part first, then new part); lt == nullptr ⇒ single topology.
__device__ void diff_window(DiffShared& sh, int tb, int te, const DevLinks& O, const DevLinks& N,
                            uint32_t* hsh, uint8_t* flg, uint8_t* lt, const DiffOut& out,
                            uint32_t t0) {
    const uint32_t wo0 = sh.ooff[tb], wo1 = sh.ooff[te];
    const uint32_t wn0 = sh.noff[tb], wn1 = sh.noff[te];
    const uint32_t no = wo1 - wo0, nn = wn1 - wn0, tot = no + nn;
    const int tid = threadIdx.x;

    // A. segment of every record; key hashes where comparisons are needed
    for (uint32_t r = tid; r < tot; r += BLOCK) {
        const bool old = r < no;
        const uint32_t idx = old ? wo0 + r : wn0 + (r - no);
        int tt = tb;
        if (lt) {
            tt = find_seg(old ? sh.ooff : sh.noff, tb, te, idx);
            lt[r] = (uint8_t)tt;
        }
        if (need_cmp(sh, tt)) hsh[r] = old ? key_hash(O, idx) : key_hash(N, idx);
    }
    __syncthreads();

    // B. old side: first key-equal new record (CalcDiff :289-303) + positional DeepEqual (:77)
    for (uint32_t r = tid; r < no; r += BLOCK) {
        const int tt = lt ? lt[r] : tb;
        if (!need_cmp(sh, tt)) continue;
        const uint32_t i = wo0 + r;
        const uint32_t h = hsh[r];
        const uint32_t ns_ = sh.noff[tt], ne_ = sh.noff[tt + 1];
        uint32_t first = 0xFFFFFFFFu;
        for (uint32_t j = ns_; j < ne_; ++j) {
            if (hsh[no + (j - wn0)] == h && key_eq(O, i, N, j)) { first = j; break; }
        }
        uint8_t f = 0;
        if (first == 0xFFFFFFFFu) f = RF_DEL;
        else if (!props_eq(O, i, N, first)) {
            f = RF_UPD;
            out.otarget[i] = first;
        }
        const uint32_t ko = sh.ooff[tt + 1] - sh.ooff[tt], kn = ne_ - ns_;
        if (ko == kn) {
            const uint32_t jp = ns_ + (i - sh.ooff[tt]);
            bool eq;
            if (first == jp) eq = (f == 0);
            else eq = hsh[no + (jp - wn0)] == h && key_eq(O, i, N, jp) && props_eq(O, i, N, jp);
            if (!eq) sh.dirty[tt] = 1;
        }
        flg[r] = f;
    }
    // C. new side: any key-equal old record (CalcDiff :305-316)
    for (uint32_t r = tid; r < nn; r += BLOCK) {
        const int tt = lt ? lt[no + r] : tb;
        if (!need_cmp(sh, tt)) continue;
        const uint32_t j = wn0 + r;
        const uint32_t h = hsh[no + r];
        bool found = false;
        for (uint32_t i = sh.ooff[tt]; i < sh.ooff[tt + 1]; ++i) {
            if (hsh[i - wo0] == h && key_eq(O, i, N, j)) { found = true; break; }
        }
        flg[no + r] = found ? 0 : RF_ADD;
    }
    __syncthreads();

    // D. action per topology (topology_controller.go:77-88)
    for (int tt = tb + tid; tt < te; tt += BLOCK) {
        const uint8_t tf = sh.tflag[tt];
        const bool st_nil = tf & KDTN_TOPO_STATUS_NIL, sp_nil = tf & KDTN_TOPO_SPEC_NIL;
        const uint32_t ko = sh.ooff[tt + 1] - sh.ooff[tt], kn = sh.noff[tt + 1] - sh.noff[tt];
        uint8_t a;
        if (st_nil || sp_nil) a = (st_nil && sp_nil) ? KDTN_ACT_SKIP : (st_nil ? KDTN_ACT_CREATED : KDTN_ACT_DIFF);
        else a = (ko == kn && !sh.dirty[tt]) ? KDTN_ACT_SKIP : KDTN_ACT_DIFF;
        sh.act[tt] = a;
        out.action[t0 + tt] = a;
    }
    __syncthreads();

    // E. masked flags out + per-workgroup counts
    uint32_t cd = 0, cu = 0, ca = 0;
    for (uint32_t base = 0; base < tot; base += BLOCK) {
        const uint32_t r = base + tid;
        uint8_t f = 0;
        bool old = false;
        if (r < tot) {
            old = r < no;
            const int tt = lt ? lt[r] : tb;
            if (sh.act[tt] == KDTN_ACT_DIFF) {
                if (need_cmp(sh, tt)) f = flg[r];
                else f = old ? RF_DEL : RF_ADD;   // the other list is empty
            }
            if (old) out.oflag[wo0 + r] = f;
            else out.nflag[wn0 + (r - no)] = f;
        }
        cd += __popcll(__ballot(old && (f & RF_DEL)));
        cu += __popcll(__ballot(old && (f & RF_UPD)));
        ca += __popcll(__ballot(!old && r < tot && (f & RF_ADD)));
    }
    if ((tid & 63) == 0) {
        atomicAdd(&sh.cnt[0], cd);
        atomicAdd(&sh.cnt[1], cu);
        atomicAdd(&sh.cnt[2], ca);
    }
    __syncthreads();
}

__global__ void __launch_bounds__(BLOCK) k_diff(DevTopos T, DevLinks O, DevLinks N, DiffOut out) {
    __shared__ DiffShared sh;
    const uint32_t wg = blockIdx.x;
    const uint32_t t0 = wg * TPW;
    const int nt = (int)min((uint32_t)TPW, T.n - t0);
    const int tid = threadIdx.x;
    if (tid <= nt) {
        sh.ooff[tid] = T.real_off[t0 + tid];
        sh.noff[tid] = T.des_off[t0 + tid];
    }
    if (tid < nt) {
        sh.tflag[tid] = T.flags[t0 + tid];
        sh.dirty[tid] = 0;
    }
    if (tid < 3) sh.cnt[tid] = 0;
    __syncthreads();
    const uint32_t total = (sh.ooff[nt] - sh.ooff[0]) + (sh.noff[nt] - sh.noff[0]);
    if (total <= (uint32_t)CAP) {
        diff_window(sh, 0, nt, O, N, sh.hash, sh.flag, sh.lt, out, t0);
    } else {
        for (int tt = 0; tt < nt; ++tt) {
            const uint32_t k = (sh.ooff[tt + 1] - sh.ooff[tt]) + (sh.noff[tt + 1] - sh.noff[tt]);
            if (k <= (uint32_t)CAP) {
                diff_window(sh, tt, tt + 1, O, N, sh.hash, sh.flag, nullptr, out, t0);
            } else {
                const uint32_t gofs = sh.ooff[tt] + sh.noff[tt];
                diff_window(sh, tt, tt + 1, O, N, out.hscratch + gofs, out.fscratch + gofs, nullptr,
                            out, t0);
            }
        }
    }
    if (tid < 3) out.wg_cnt[wg * 3 + tid] = sh.cnt[tid];
}

// ======================================================================================
// k_scan: exclusive scan of per-workgroup counts (3 lists), single workgroup of 1024.
// ======================================================================================
__global__ void __launch_bounds__(1024) k_scan(const uint32_t* wg_cnt, uint32_t nwg, uint32_t* wg_base,
                                               uint32_t* totals, uint32_t T, uint32_t* del_off,
                                               uint32_t* add_off, uint32_t* upd_off) {
    __shared__ uint32_t s_w[16][3];
    __shared__ uint32_t s_carry[3];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    if (tid < 3) s_carry[tid] = 0;
    __syncthreads();
    const uint32_t per = 16;                       // items per thread per tile
    const uint32_t tile = 1024 * per;
    for (uint32_t t0 = 0; t0 < nwg; t0 += tile) {
        uint32_t loc[3] = {0, 0, 0};
        const uint32_t b = t0 + tid * per;
        for (uint32_t q = 0; q < per; ++q) {
            const uint32_t w = b + q;
            if (w < nwg) {
                loc[0] += wg_cnt[w * 3 + 0];
                loc[1] += wg_cnt[w * 3 + 1];
                loc[2] += wg_cnt[w * 3 + 2];
            }
        }
        uint32_t incl[3];
        for (int c = 0; c < 3; ++c) {
            uint32_t v = loc[c];
            for (int d = 1; d < 64; d <<= 1) {
                uint32_t o = __shfl_up(v, d, 64);
                if (lane >= d) v += o;
            }
            incl[c] = v;
            if (lane == 63) s_w[wave][c] = v;
        }
        __syncthreads();
        uint32_t run[3];
        for (int c = 0; c < 3; ++c) {
            uint32_t pre = s_carry[c];
            for (int w = 0; w < wave; ++w) pre += s_w[w][c];
            run[c] = pre + incl[c] - loc[c];
        }
        for (uint32_t q = 0; q < per; ++q) {
            const uint32_t w = b + q;
            if (w < nwg) {
                for (int c = 0; c < 3; ++c) {
                    wg_base[w * 3 + c] = run[c];
                    run[c] += wg_cnt[w * 3 + c];
                }
            }
        }
        __syncthreads();
        if (tid < 3) {
            uint32_t s = 0;
            for (int w = 0; w < 16; ++w) s += s_w[w][tid];
            s_carry[tid] += s;
        }
        __syncthreads();
    }
    if (tid == 0) {
        totals[0] = s_carry[0];   // del
        totals[1] = s_carry[1];   // upd
        totals[2] = s_carry[2];   // add
        del_off[T] = s_carry[0];
        upd_off[T] = s_carry[1];
        add_off[T] = s_carry[2];
    }
}

// ======================================================================================
// k_emit: batch lists + delLink/addLink/UpdateLinks pure prefix + MakeQdiscs
// ======================================================================================
struct EmitShared {
    uint32_t ooff[TPW + 1];
    uint32_t noff[TPW + 1];
    uint8_t act[TPW];
    uint32_t ns[TPW], src[TPW], netns[TPW];
    uint32_t cnt[3][TPW];     // del, upd, add per topology
    uint32_t wsum[BLOCK / 64][2];
};

// MakeQdiscs over parsed dictionary entries (common/qdisc.go:20-126 + netlink NewNetem)
KD_INLINE void make_qdisc(const DevLinks& L, uint32_t j, const uint4* pp, const uint64_t* prate,
                          uint32_t* q /* 18 words */) {
#pragma unroll
    for (int w = 0; w < 18; ++w) q[w] = 0;
    uint32_t id[KDTN_NPROP];
    const uint32_t gap = L.gap[j];
    bool empty = gap == 0;
#pragma unroll
    for (int k = 0; k < KDTN_NPROP; ++k) {
        id[k] = L.prop[k][j];
        empty = empty && id[k] == 0;             // id 0 == "" (proto.Size == 0, :24)
    }
    if (empty) return;
    const uint4 lat = pp[id[KDTN_P_LATENCY]];
    const uint4 lco = pp[id[KDTN_P_LATENCY_CORR]];
    const uint4 jit = pp[id[KDTN_P_JITTER]];
    const uint4 los = pp[id[KDTN_P_LOSS]];
    const uint4 lsc = pp[id[KDTN_P_LOSS_CORR]];
    const uint4 dup = pp[id[KDTN_P_DUPLICATE]];
    const uint4 dpc = pp[id[KDTN_P_DUPLICATE_CORR]];
    const uint4 rop = pp[id[KDTN_P_REORDER_PROB]];
    const uint4 roc = pp[id[KDTN_P_REORDER_CORR]];
    const uint4 cop = pp[id[KDTN_P_CORRUPT_PROB]];
    const uint4 coc = pp[id[KDTN_P_CORRUPT_CORR]];
    const uint4 rt = pp[id[KDTN_P_RATE]];
    uint32_t err = 0;                            // first failing parse, reference order
    if (lat.w & PF_DUR_ERR) err = KDTN_E_LATENCY;
    else if (lco.w & PF_PCT_ERR) err = KDTN_E_LATENCY_CORR;
    else if (jit.w & PF_DUR_ERR) err = KDTN_E_JITTER;
    else if (los.w & PF_PCT_ERR) err = KDTN_E_LOSS;
    else if (lsc.w & PF_PCT_ERR) err = KDTN_E_LOSS_CORR;
    else if (dup.w & PF_PCT_ERR) err = KDTN_E_DUPLICATE;
    else if (dpc.w & PF_PCT_ERR) err = KDTN_E_DUPLICATE_CORR;
    else if (rop.w & PF_PCT_ERR) err = KDTN_E_REORDER_PROB;
    else if (roc.w & PF_PCT_ERR) err = KDTN_E_REORDER_CORR;
    else if (cop.w & PF_PCT_ERR) err = KDTN_E_CORRUPT_PROB;
    else if (coc.w & PF_PCT_ERR) err = KDTN_E_CORRUPT_CORR;
    else if (rt.w & PF_RATE_ERR) err = KDTN_E_RATE;
    if (err) {
        q[17] = err << 16;                       // byte 70 = err
        return;
    }
    // NewNetem
    const uint32_t lat_us = lat.y, jit_us = jit.y;
    const uint32_t loss = los.x, dupl = dup.x;
    const uint32_t lat_t = lat.z;                // time2Tick(latency)
    q[0] = lat_t;                                                   // latency
    q[1] = (lat_us > 0 && jit_us > 0) ? lco.x : 0u;                // delay_corr
    q[2] = 1000u;                                                   // limit
    q[3] = loss;                                                    // loss
    q[4] = loss > 0 ? lsc.x : 0u;                                   // loss_corr
    uint32_t g = gap;
    if (rop.x > 0 && g == 0) g = 1;
    q[5] = g;                                                       // gap
    q[6] = dupl;                                                    // duplicate
    q[7] = dupl > 0 ? dpc.x : 0u;                                   // duplicate_corr
    q[8] = lat_t > 0 ? jit.z : jit_us;                              // jitter
    q[9] = rop.x;
    q[10] = roc.x;
    q[11] = cop.x;
    q[12] = coc.x;
    const uint64_t rate = prate[id[KDTN_P_RATE]];
    uint32_t has_tbf = 0;
    if (rate != 0) {
        uint32_t burst = (uint32_t)(rate / 250ull);              // getTbfBurst
        if (burst < 5000u) burst = 5000u;
        q[13] = burst;
        q[14] = (uint32_t)rate;
        q[15] = (uint32_t)(rate >> 32);
        q[16] = 1500u;
        has_tbf = 1;
    }
    q[17] = 1u | (has_tbf << 8);                 // has_netem, has_tbf, err=0
}

KD_INLINE void store_qdisc(uint2* dst, const uint32_t* q) {
#pragma unroll
    for (int w = 0; w < 9; ++w) dst[w] = make_uint2(q[2 * w], q[2 * w + 1]);
}

KD_INLINE uint4 pack_res(uint32_t peer, int32_t vni, uint32_t vtep, uint32_t kind, uint32_t err,
                         uint32_t hit) {
    return make_uint4(peer, (uint32_t)vni, vtep, kind | (err << 8) | (hit << 16));
}

// MakeVeth(netns, intf, ip, mac) validity from key-string flags (common/veth.go:21-36)
KD_INLINE uint32_t veth_err(const uint8_t* kf, uint32_t ip, uint32_t mac, uint32_t ecidr,
                            uint32_t emac) {
    if (kf[ip] & KF_CIDR_BAD) return ecidr;
    if (kf[mac] & KF_MAC_BAD) return emac;
    return 0;
}

KD_INLINE int32_t vni_of(int32_t base, int64_t uid) {   // common/utils.go:29-31
    return (int32_t)(uint32_t)((uint64_t)(int64_t)base + (uint64_t)uid);
}

// block-wide exclusive scan of two 0/1 flags; returns chunk totals
KD_INLINE void block_scan2(EmitShared& sh, uint32_t a, uint32_t b, uint32_t* ea, uint32_t* eb,
                           uint32_t* ta, uint32_t* tb) {
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const uint64_t ba = __ballot(a), bb = __ballot(b);
    const uint64_t lt = lanemask_lt();
    if (lane == 0) {
        sh.wsum[wave][0] = __popcll(ba);
        sh.wsum[wave][1] = __popcll(bb);
    }
    __syncthreads();
    uint32_t pa = 0, pb = 0, sa = 0, sb = 0;
#pragma unroll
    for (int w = 0; w < BLOCK / 64; ++w) {
        const uint32_t xa = sh.wsum[w][0], xb = sh.wsum[w][1];
        if (w < wave) { pa += xa; pb += xb; }
        sa += xa;
        sb += xb;
    }
    *ea = pa + __popcll(ba & lt);
    *eb = pb + __popcll(bb & lt);
    *ta = sa;
    *tb = sb;
    __syncthreads();
}

__global__ void __launch_bounds__(BLOCK) k_emit(DevTopos T, DevLinks O, DevLinks N,
                                                const uint8_t* oflag, const uint32_t* otarget,
                                                const uint8_t* nflag, const uint8_t* action,
                                                DevTables tb, EmitOut out) {
    __shared__ EmitShared sh;
    const uint32_t wg = blockIdx.x;
    const uint32_t t0 = wg * TPW;
    const int nt = (int)min((uint32_t)TPW, T.n - t0);
    const int tid = threadIdx.x;
    if (tid <= nt) {
        sh.ooff[tid] = T.real_off[t0 + tid];
        sh.noff[tid] = T.des_off[t0 + tid];
    }
    if (tid < nt) {
        sh.act[tid] = action[t0 + tid];
        sh.ns[tid] = T.ns[t0 + tid];
        sh.src[tid] = T.src_ip[t0 + tid];
        sh.netns[tid] = T.net_ns[t0 + tid];
    }
    if (tid < TPW) {
        sh.cnt[0][tid] = 0;
        sh.cnt[1][tid] = 0;
        sh.cnt[2][tid] = 0;
    }
    __syncthreads();
    const uint32_t base_del = out.wg_base[wg * 3 + 0];
    const uint32_t base_upd = out.wg_base[wg * 3 + 1];
    const uint32_t base_add = out.wg_base[wg * 3 + 2];
    const bool do_res = out.stages & KDTN_STAGE_RESOLVE;
    const bool do_q = out.stages & KDTN_STAGE_QDISC;
    const uint32_t dflt = *tb.default_id;

    // ---- old side: DelLinks / UpdateLinks entries, status order ------------------------
    const uint32_t o0 = sh.ooff[0], o1 = sh.ooff[nt];
    uint32_t carry_d = 0, carry_u = 0;
    for (uint32_t c = o0; c < o1; c += BLOCK) {
        const uint32_t i = c + tid;
        const uint8_t f = i < o1 ? oflag[i] : 0;
        const uint32_t isd = f & RF_DEL, isu = (f & RF_UPD) ? 1u : 0u;
        uint32_t ed, eu, td, tu;
        block_scan2(sh, isd, isu, &ed, &eu, &td, &tu);
        if (isd | isu) {
            const int tt = find_seg(sh.ooff, 0, nt, i);
            if (isd) {
                const uint32_t e = base_del + carry_d + ed;
                out.del_idx[e] = i;
                atomicAdd(&sh.cnt[0][tt], 1u);
                if (do_res) {
                    // delLink (handler.go:461-492)
                    const int32_t vni = vni_of(tb.vxlan_base, O.uid[i]);
                    const uint32_t err = veth_err(tb.kflags, O.key[KDTN_K_LOCAL_IP][i],
                                                  O.key[KDTN_K_LOCAL_MAC][i], KDTN_E_VETH_CIDR,
                                                  KDTN_E_VETH_MAC);
                    uint32_t hit = 0;
                    if (!err) hit = vni_lookup(tb, sh.src[tt], vni) == sh.netns[tt];
                    out.del_res[e] = pack_res(0xFFFFFFFFu, vni, 0, 0, err, hit);
                }
            }
            if (isu) {
                const uint32_t e = base_upd + carry_u + eu;
                const uint32_t j = otarget[i];
                out.upd_idx[e] = j;
                atomicAdd(&sh.cnt[1][tt], 1u);
                uint32_t q[18];
                if (do_q || do_res) make_qdisc(N, j, tb.pparsed, tb.prate, q);
                if (do_q) store_qdisc(out.upd_qdisc + (size_t)e * 9, q);
                if (do_res) {
                    // UpdateLinks (handler.go:644-663): MakeVeth(local), then MakeQdiscs
                    const int32_t vni = vni_of(tb.vxlan_base, N.uid[j]);
                    uint32_t err = veth_err(tb.kflags, N.key[KDTN_K_LOCAL_IP][j],
                                            N.key[KDTN_K_LOCAL_MAC][j], KDTN_E_VETH_CIDR,
                                            KDTN_E_VETH_MAC);
                    if (!err) err = (q[17] >> 16) & 0xFF;
                    out.upd_res[e] = pack_res(0xFFFFFFFFu, vni, 0, 0, err, 0);
                }
            }
        }
        carry_d += td;
        carry_u += tu;
    }

    // ---- new side: AddLinks entries, spec order -----------------------------------------
    const uint32_t n0 = sh.noff[0], n1 = sh.noff[nt];
    uint32_t carry_a = 0;
    for (uint32_t c = n0; c < n1; c += BLOCK) {
        const uint32_t j = c + tid;
        const uint32_t isa = (j < n1) ? (nflag[j] & RF_ADD) : 0u;
        uint32_t ea, e2, ta, t2;
        block_scan2(sh, isa, 0u, &ea, &e2, &ta, &t2);
        if (isa) {
            const int tt = find_seg(sh.noff, 0, nt, j);
            const uint32_t e = base_add + carry_a + ea;
            out.add_idx[e] = j;
            atomicAdd(&sh.cnt[2][tt], 1u);
            uint32_t q[18];
            if (do_q) {
                make_qdisc(N, j, tb.pparsed, tb.prate, q);
                store_qdisc(out.add_qdisc + (size_t)e * 9, q);
            }
            if (do_res) {
                // addLink pure prefix (handler.go:316-459)
                const int32_t vni = vni_of(tb.vxlan_base, N.uid[j]);
                uint32_t err = veth_err(tb.kflags, N.key[KDTN_K_LOCAL_IP][j],
                                        N.key[KDTN_K_LOCAL_MAC][j], KDTN_E_VETH_CIDR,
                                        KDTN_E_VETH_MAC);                       // :327
                uint32_t kind = 0, peer = 0xFFFFFFFFu, vtep = 0, hit = 0;
                if (!err) {
                    const uint32_t pp = N.key[KDTN_K_PEER_POD][j];
                    const uint8_t pf = tb.kflags[pp];
                    if (pf & KF_LOCALHOST) {
                        kind = KDTN_KIND_MACVLAN;                                  // :333
                    } else if (pf & KF_PHYSICAL) {
                        kind = KDTN_KIND_PHYSICAL;                                 // :348
                        vtep = pp;
                        const uint32_t nsx = vni_lookup(tb, sh.src[tt], vni);    // :177-179
                        hit = (nsx != 0xFFFFFFFFu && nsx != sh.netns[tt]);
                    } else {
                        const uint32_t lns = sh.ns[tt] == 0 ? dflt : sh.ns[tt];  // :29-31
                        const uint32_t g = pod_lookup(tb, lns, pp);               // :375
                        if (g == 0xFFFFFFFFu) {
                            err = KDTN_E_PEER_LOOKUP;
                        } else {
                            peer = g;
                            const uint4 pe = tb.pods[g];
                            const uint32_t p_src = pe.z, p_ns = pe.w & 0x7FFFFFFFu;
                            if (pe.w & 0x80000000u) {
                                err = KDTN_E_PEER_NO_LINKS;                        // :380-384
                            } else if (p_src == 0 || p_ns == 0) {
                                kind = KDTN_KIND_PEER_DEAD;                        // :386-395
                            } else if (p_src == sh.src[tt]) {
                                kind = KDTN_KIND_SAME_NODE;                        // :399-418
                                err = veth_err(tb.kflags, N.key[KDTN_K_PEER_IP][j],
                                               N.key[KDTN_K_PEER_MAC][j], KDTN_E_PEER_VETH_CIDR,
                                               KDTN_E_PEER_VETH_MAC);
                            } else {
                                kind = KDTN_KIND_CROSS_NODE;                       // :419-453
                                vtep = p_src;
                                const uint32_t nsx = vni_lookup(tb, p_src, vni);
                                hit = (nsx != 0xFFFFFFFFu && nsx != p_ns);
                            }
                        }
                    }
                }
                out.add_res[e] = pack_res(peer, vni, vtep, kind, err, hit);
            }
        }
        carry_a += ta;
    }
    __syncthreads();

    // ---- per-topology batch offsets: wave 0, lane = topology --------------------------
    if (tid < 64) {
        const int tt = tid;
        const uint32_t bases[3] = {base_del, base_upd, base_add};
        uint32_t* offs[3] = {out.del_off, out.upd_off, out.add_off};
        for (int c = 0; c < 3; ++c) {
            const uint32_t x = (tt < nt) ? sh.cnt[c][tt] : 0u;
            uint32_t v = x;
            for (int d = 1; d < 64; d <<= 1) {
                const uint32_t o = __shfl_up(v, d, 64);
                if (tt >= d) v += o;
            }
            if (tt < nt) offs[c][t0 + tt] = bases[c] + v - x;
        }
    }
}

// Standalone MakeQdiscs over a batch of property sets (kdtn_make_qdiscs).
__global__ void __launch_bounds__(BLOCK) k_qdisc_batch(DevLinks props, const uint4* pparsed,
                                                       const uint64_t* prate, uint2* out) {
    const uint32_t j = blockIdx.x * BLOCK + threadIdx.x;
    if (j >= props.n) return;
    uint32_t q[18];
    make_qdisc(props, j, pparsed, prate, q);
    store_qdisc(out + (size_t)j * 9, q);
}

}  // namespace kdtn
