// kdtn_engine.hip — host side of libkdtn.so: the C-ABI of include/kdtn.h over the
// HIP kernels of kdtn_kernels.hip. One kdtn_ctx per process/GPU; device buffers are
// owned by the context and reused across epochs (high-water-mark growth).
#include <hip/hip_runtime.h>
#include <hsa/hsa.h>
#include <hsa/hsa_ext_amd.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <string>
#include <vector>

#include "../../include/kdtn.h"
#include "kdtn_kernels.h"

using namespace kdtn;

namespace {

constexpr int kMaxTimers = 32;
constexpr int kSyncSpinUs = 2000;     // kdtn_epoch_sync: event polling before the blocking wait

struct DevBuf {
    void* p = nullptr;
    size_t cap = 0;
};

#define HIP_TRY(expr)                                                                    \
    do {                                                                                 \
        hipError_t _e = (expr);                                                          \
        if (_e != hipSuccess) {                                                          \
            std::snprintf(g_last_error, sizeof(g_last_error), "%s: %s (%s:%d)", #expr,   \
                          hipGetErrorString(_e), __FILE__, __LINE__);                    \
            return KDTN_EIO;                                                             \
        }                                                                                \
    } while (0)

thread_local char g_last_error[512] = "";

size_t align_up(size_t x, size_t a) { return (x + a - 1) / a * a; }

uint32_t next_pow2(uint64_t x) {
    uint64_t p = 64;
    while (p < x) p <<= 1;
    return (uint32_t)p;
}

}  // namespace

// Link table storage: one allocation in 64-record tiles (AoSoA, kdtn_kernels.h), so kernels
// receive one base pointer per table.
struct DevLinkStore {
    DevBuf buf;
    uint32_t n = 0;
    DevLinks view{};
};

struct kdtn_ctx {
    int device = 0;
    uint32_t n_cus = 256;
    kdtn_config cfg{};
    hipStream_t own_stream = nullptr;
    hipStream_t stream = nullptr;
    hipStream_t comm_stream = nullptr;          // RCCL pod-status exchange (nranks > 1)
    hipStream_t copy_stream = nullptr;          // delta uploads: host-to-device copies beside the kernels
    hipStream_t side_stream = nullptr;          // the pod lookup build beside the dictionary parses
    hipStream_t side_hi = nullptr;              // (profiling A/B: the same at the highest priority)
    hipEvent_t ev_front = nullptr, ev_side = nullptr;
    hipEvent_t ev_cp[4] = {};
    hipEvent_t ev_col[LINK_COLS32 + 1] = {};   // a delta's staged column copies (+ uid), each placed on arrival
    hipStream_t d2h_stream = nullptr;           // kdtn_epoch_download_async: the outputs' copies
    hipEvent_t ev_dl_ready = nullptr, ev_dl_done = nullptr;
    bool dl_pending = false;                    // an async download's copies may still be reading outputs
    // Downloads on one SDMA engine (hsa_amd_memory_async_copy_on_engine): the copy engine alone
    // reaches the host link's rate (56 GB/s D2H, profiles/r05d_sdma_probe.jsonl) and takes no
    // CUs, where the runtime's device-to-host copies in this process run as blit kernels. Used
    // when every destination is page-locked host memory, else the HIP copies.
    bool sdma_tried = false, sdma_ok = false, dl_sdma = false;
    bool sdma_inited = false;   // hsa_init held and dl_sig created (outlives sdma_ok after a failed issue)
    hsa_agent_t sdma_gpu{}, sdma_cpu{};
    uint32_t sdma_engine[2] = {0, 0};   // the download's engines (bit masks; [1] = 0: one engine)
    hsa_signal_t dl_sig{};
    hipEvent_t ev_fill = nullptr, ev_ag = nullptr;
    // dictionaries; parsed tables persist across uploads for an append-only interner
    // (kdtn_epoch_in.kdict_keep / pdict_keep): *_valid strings have valid parsed tables, a run
    // parses [*_from, n) — the strings its upload added
    DevBuf kd_bytes, kd_offs, kd_bits, pd_bytes, pd_offs, pd_pct, pd_dur, pd_rate, pd_rerr, kd_special;
    uint32_t D = 0, P = 0;
    uint32_t kd_from = 0, pd_from = 0, kd_valid = 0, pd_valid = 0, kb_cap = 0;
    uint32_t si_k = 0, si_p = 0;           // leading strings whose inline encoder entries are built

    // topologies
    DevBuf t_ns, t_name, t_src, t_netns, t_flags, t_roff, t_noff;
    // sharded ingest: selection, scans, the shard's tables before they are swapped in
    DevBuf sh_keep, sh_kreal, sh_kdes, sh_tidx, sh_roff64, sh_noff64, sh_doc;
    DevBuf sh_ns, sh_name, sh_src, sh_netns, sh_flags, sh_roff, sh_noff;
    uint32_t T = 0;
    // links
    DevLinkStore real, des;
    DevLinkStore sh_real, sh_des;              // sharded ingest: the shard's link stores (swapped in)
    uint32_t sh_T = 0;                         // sharded ingest: topologies of the shard (doc index table)
    // vni table
    DevBuf v_node, v_vni, v_netns, v_ents, v_slots, v_table;
    uint32_t V = 0, vni_mask = 0;
    // kdtn_epoch_vni_apply: ops, snapshot marks, the new map's table, arrays and scan partials
    DevBuf vx_ops, vx_dead, vx_slots, vx_node, vx_vni, vx_netns, vx_part, vx_cut, vx_vis;
    // v_node/v_vni/v_netns: the snapshot of the current upload (what vni_hit is decided
    // against, re-runs included); r_*: the map kdtn_epoch_vni_apply produced, which becomes
    // the next KDTN_VNI_RESIDENT upload's snapshot. The resident map is r_* when vres_in_r.
    DevBuf r_node, r_vni, r_netns;
    bool vres_ok = false;          // a map usable as KDTN_VNI_RESIDENT exists
    bool vres_in_r = false;
    // sharded apply: every rank's ops gathered in rank order ([dels][adds]), by RCCL or imported
    DevBuf vx_cnt, vx_send, vx_recv, vx_gops;
    DevBuf vx_flag, vx_dkeys, vx_dused, vx_cpos, vx_cpart, vx_cnode, vx_cvni;   // order-dependent keys
    uint32_t vx_ncont = 0;
    bool vx_contest_ok = false;      // a vni_apply ran since the last run
    uint64_t vx_gd = 0, vx_ga = 0;
    bool vx_imported = false;
    uint32_t vres_n = 0, vres_D = 0;   // its entries; the dictionary size its ids were made for
    // pods
    DevBuf pods, pod_ovf, pod_direct;
    uint32_t slice = 0, pod_total = 0, ovf_mask = 0, kb_words = 0, pod_stamp = 0;
    // late pods (kdtn_epoch_late_pods): rows [pod_total, pod_total + n_late) of `pods`, after
    // the gathered table; cleared by the next upload, delta, ingest or commit (prepare_work)
    uint32_t n_late = 0;
    // pods_ready: pods / pod_direct / pod_ovf hold the complete tables of the current rows (a
    // full build ran and every later row change was patched). pods_delta: this upload's rows were
    // patched in kdtn_epoch_upload_delta, so its runs do no pod-table work.
    bool pods_ready = false, pods_delta = false;
    DevBuf pd_send, pd_recv, pd_cnt;
    bool traced = false;
    // work
    DevBuf otarget, sync, misc, hscratch, fscratch, trace, stage;
    uint32_t nwg = 0;
    // outputs
    DevBuf action, del_off, add_off, upd_off, del_idx, add_idx, upd_idx;
    DevBuf del_res, add_res, upd_res, add_qdisc, upd_qdisc, add_qerr;
    // wire encoding
    DevBuf kd_si, kd_len1, pd_si, pd_len1, w_rel, w_topo, w_size, w_err, w_off, w_part, w_arena, w_pinfo;
    uint64_t w_bytes = 0;
    bool encoded = false;
    // RemotePod fan-out
    DevBuf f_mark, f_send, f_node_idx, f_nodes, f_counts, f_base, f_part, f_idx, f_inv, f_reach_upd, f_cut, f_st, f_node;
    bool fan_valid = false;                    // the fan-out of the last run is in f_* (fanout_compute)
    bool lc_valid = false;                     // lc: coarse entry -> topology indexes of the last run's lists
    bool si_run = false;                       // the string tables were built since the last run
    DevBuf lc[3];
    uint32_t fan_nn = 0, fan_nsend = 0;
    // RemotePod messages (kdtn_epoch_remote_encode)
    DevBuf rp_flag, rp_pos, rp_phys, rp_msz, rp_moff, rp_tsz, rp_toff, rp_part, rp_arena, rp_tc, rp_msz_e, rp_tsz_e;
    uint32_t rp_n = 0, rp_nr = 0;
    uint64_t rp_bytes = 0, rp_tc_bytes = 0;
    bool rp_done = false;
    // resident state: commit / delta plans, the delta's arrays and inline records
    DevBuf st_cnt, st_len, st_base, st_mode, st_flags, st_off64, st_part, st_off32, st_mask, st_chg;
    DevBuf dl_topo, dl_src, dl_netns, dl_nil, dl_off, dl_ref, dl_rows;
    // delta with a topology-set change: the map, created rows' names, the realised plan
    DevBuf dl_prev, dl_ns, dl_name, dl_dest, dl_pack, st_rlen, st_rbase, st_roff64, st_rpart, st_roff32, st_seen;
    // incremental CR ingest (kdtn_json_ingest_delta): the document's scratch tables and local
    // dictionaries, the id maps into the resident dictionaries, the topology-key match
    DevBuf ji_ns, ji_name, ji_src, ji_netns, ji_flags, ji_roff, ji_noff, ji_kb, ji_ko, ji_pb, ji_po;
    DevLinkStore ji_des, ji_real;
    DevBuf ji_kmap, ji_pmap, ji_miss, ji_mlen, ji_rank, ji_boff, ji_nil, ji_keep, ji_kpos, ji_claim, ji_res,
        ji_created, ji_cpos, ji_keys, ji_vals, ji_dkeys, ji_del, ji_ref;
    // resident string indexes (string → id) of the dictionaries' first n strings
    struct StrIndex {
        DevBuf slots;
        uint32_t n = 0, mask = 0;
    } ix_k, ix_p;
    uint64_t kd_arena = 0, pd_arena = 0;       // dictionary arena bytes (host-known: tables_info)
    DevLinkStore dl_rec;
    bool tables_cur = false;                   // j_info describes the current tables (kdtn_epoch_tables_info)
    // tc argv
    DevBuf tc_size, tc_off, tc_part, tc_arena;
    uint64_t tc_bytes = 0;
    uint32_t tc_n = 0;
    bool tc_done = false;
    // CR ingest (kdtn_ingest.hip): document, block masks, token stream, decode scratch
    DevBuf j_doc, j_q, j_bs, j_hb, j_esc, j_qcnt, j_qoff, j_tok, j_open, j_close, j_gcnt, j_goff;
    DevBuf j_olist, j_vlist, j_slist;
    uint32_t j_kcap = 0, j_pcap = 0;   // intern table sizes that fit the last document
    DevBuf j_toks, j_par, j_role, j_ecls, j_odep, j_ord, j_tagg, j_gagg, j_cnt3, j_coff3, j_small, j_part;
    DevBuf j_tflags, j_owner, j_vown, j_kslots, j_krep, j_pslots, j_prep, j_heap;
    DevBuf j_kkeys, j_pkeys;     // dense key words of the intern tables
    DevBuf j_rows;               // row-major staging of the decoded link records (JS_ROW words each)
    DevBuf j_bits, j_bcnt, j_wrank, j_kslot_id, j_pslot_id, j_len, j_off64, j_sofid;
    uint64_t j_n = 0;
    uint32_t j_nb = 0;
    bool j_loaded = false, j_done = false;
    kdtn_ingest_info j_info{};
    // host-visible counters
    hipEvent_t ev_done = nullptr;  // the epoch's last command (kdtn_epoch_sync polls it)
    uint32_t* h_misc = nullptr;   // pinned: [1]=del, [2]=upd, [3]=add, [4]=look-back error (sync header words)
    // coherent page-locked words the epoch's last kernel writes itself ([0..2] list totals, [3]
    // look-back error): no readback copy per epoch (a 16-B blit kernel, 5.6 µs + a dispatch);
    // kdtn_epoch_sync moves them to h_misc[1..4]
    uint32_t* h_tot = nullptr;
    bool uploaded = false;
    bool ran = false;
    bool synced = false;   // h_misc[1..4] hold the last run's list totals (kdtn_epoch_sync or counts_fresh)
    uint32_t last_stages = 0;
    // multi-GPU
    ncclComm_t comm = nullptr;
    int nranks = 1, rank = 0;
    bool pods_imported = false;   // host transport: this epoch's global pod table is in place
    bool pods_rank_major = true;  // pod table rank-major (uploads) vs document order (sharded ingest)
    // kdtn_json_ingest_shard leaves the context as rank `shard` of `nshards` for its epoch; the
    // next upload or ingest restores the rank setup the caller had before (sh_saved_*)
    bool sh_active = false;
    int sh_saved_nranks = 1, sh_saved_rank = 0;
    // timers: 0 none, 1 k_reconcile (+ placement) only, 2 every stage (kdtn_set_timing)
    int timing = 2;
    hipEvent_t ev[kMaxTimers + 1] = {};
    const char* ev_name[kMaxTimers] = {};
    int n_ev = 0;
    // per-stage HIP-event times summed over the epochs synced since the last reset
    // (kdtn_timer_totals): a timed loop reads them once instead of once per epoch
    const char* acc_name[kMaxTimers] = {};
    double acc_ms[kMaxTimers] = {};
    uint32_t acc_n[kMaxTimers] = {};
    int n_acc = 0;
};

namespace {

// Replaced device buffers are retired, not freed at once: hipFree synchronises the whole
// device (measured: 1.3-1.5 ms inside a delta upload whose copies and kernels were in flight
// on two streams, every overlap lost), so they are freed together once more than
// kRetireBytes are waiting (one synchronisation for many regrowths) or when a context is
// destroyed. Retired buffers belong to no context: nothing enqueues work on them any more, and
// hipFree completes the work already in flight first. The bound is 32 GB of the 288 GB: a
// resident config-3 chain retires ≈ 8.5 GB while its rotating buffers reach their sizes, and
// at 8 GB that flush (≈ 10 frees, 5.6 ms) landed inside an epoch of the steady state
// (profiles/r04p_resident_alloc_log.txt).
constexpr size_t kRetireBytes = (size_t)32 << 30;
struct Retired {
    std::mutex m;
    std::vector<void*> p;
    size_t bytes = 0;
};
Retired& retired() {
    static Retired r;
    return r;
}
// (profiling build, KDTN_ALLOC_LOG set) allocations of 16 MB and more and the flushes, on stderr
void alloc_log(const char* what, size_t bytes) {
#if KDTN_PROFILING
    static const bool on = std::getenv("KDTN_ALLOC_LOG") != nullptr;
    if (on && bytes >= (16u << 20)) std::fprintf(stderr, "[kdtn alloc] %s %zu MB\n", what, bytes >> 20);
#else
    (void)what;
    (void)bytes;
#endif
}
// SDMA downloads in flight (any context): a retired buffer may be one they read
struct SdmaInflight {
    std::mutex m;
    std::vector<uint64_t> sig;
};
SdmaInflight& sdma_inflight() {
    static SdmaInflight f;
    return f;
}
void sdma_wait(hsa_signal_t sg) {
    while (hsa_signal_wait_scacquire(sg, HSA_SIGNAL_CONDITION_EQ, 0, UINT64_MAX, HSA_WAIT_STATE_ACTIVE) != 0) {
    }
}
void retired_flush() {
    {
        SdmaInflight& f = sdma_inflight();
        std::lock_guard<std::mutex> lk(f.m);
        for (uint64_t h : f.sig) sdma_wait(hsa_signal_t{h});
    }
    Retired& r = retired();
    std::lock_guard<std::mutex> lk(r.m);
    alloc_log("flush", r.bytes);
    for (void* p : r.p) (void)hipFree(p);
    r.p.clear();
    r.bytes = 0;
}
void retire(void* p, size_t bytes) {
    if (!p) return;
    Retired& r = retired();
    bool flush;
    {
        std::lock_guard<std::mutex> lk(r.m);
        r.p.push_back(p);
        r.bytes += bytes;
        flush = r.bytes > kRetireBytes;
    }
    if (flush) retired_flush();
}

// hipMalloc that first gives back the retired buffers when the device is out of memory (up to
// kRetireBytes may only be waiting to be freed; hipFree waits for the work that uses them)
hipError_t dev_malloc(void** p, size_t bytes) {
    hipError_t e = hipMalloc(p, bytes);
    if (e == hipErrorOutOfMemory || e == hipErrorMemoryAllocation) {
        (void)hipGetLastError();
        retired_flush();
        e = hipMalloc(p, bytes);
    }
    return e;
}

int ensure(DevBuf& b, size_t bytes) {
    bytes = std::max<size_t>(bytes, 256);
    if (b.cap >= bytes) return KDTN_OK;
    // grown buffers get 1/8 headroom (from 1 MB on): epoch sizes drift from epoch to epoch
    // (a churn chain's record counts); the old buffer is retired (no device synchronisation)
    if (bytes >= (1u << 20)) bytes = (bytes + bytes / 8 + 0xFFFFF) & ~(size_t)0xFFFFF;
    retire(b.p, b.cap);
    b.p = nullptr;
    b.cap = 0;
    alloc_log("ensure", bytes);
    hipError_t e = dev_malloc(&b.p, bytes);
    if (e != hipSuccess) {
        std::snprintf(g_last_error, sizeof(g_last_error), "hipMalloc(%zu): %s", bytes,
                      hipGetErrorString(e));
        b.p = nullptr;
        return KDTN_ENOMEM;
    }
    b.cap = bytes;
    return KDTN_OK;
}
// Grow b to at least `bytes`, keeping its first `keep` bytes (stream-ordered copy).
int ensure_keep(DevBuf& b, size_t bytes, size_t keep, hipStream_t s) {
    bytes = std::max<size_t>(bytes, 256);
    if (b.cap >= bytes) return KDTN_OK;
    if (!keep || !b.p) return ensure(b, bytes);
    const size_t cap = std::max(bytes, b.cap + b.cap / 2);
    alloc_log("ensure_keep", cap);
    void* np = nullptr;
    hipError_t e = dev_malloc(&np, cap);
    if (e != hipSuccess) {
        std::snprintf(g_last_error, sizeof(g_last_error), "hipMalloc(%zu): %s", cap, hipGetErrorString(e));
        return KDTN_ENOMEM;
    }
    HIP_TRY(hipMemcpyAsync(np, b.p, std::min(keep, b.cap), hipMemcpyDeviceToDevice, s));
    retire(b.p, b.cap);                  // (stream-ordered after the copy: no synchronisation)
    b.p = np;
    b.cap = cap;
    return KDTN_OK;
}

void release(DevBuf& b) {
    retire(b.p, b.cap);
    b.p = nullptr;
    b.cap = 0;
}

#define TRY(expr)                   \
    do {                            \
        int _r = (expr);            \
        if (_r != KDTN_OK) return _r; \
    } while (0)

// Scope guard of a call that enqueued copies from caller memory: an early (error) return waits
// for the streams; the normal path disarms it once it has synchronised itself.
struct StreamsDrain {
    hipStream_t a, b;
    bool armed = true;
    ~StreamsDrain() {
        if (!armed) return;
        (void)hipStreamSynchronize(a);
        if (b != a) (void)hipStreamSynchronize(b);
    }
};

int upload(kdtn_ctx* c, DevBuf& b, const void* src, size_t bytes) {
    TRY(ensure(b, bytes));
    if (bytes) HIP_TRY(hipMemcpyAsync(b.p, src, bytes, hipMemcpyHostToDevice, c->stream));
    return KDTN_OK;
}

template <typename T>
T* dp(DevBuf& b) { return static_cast<T*>(b.p); }

// arenas get 64 B of slack: dictionary slices are staged with 16-B loads
int upload_arena(kdtn_ctx* c, DevBuf& b, const void* src, size_t bytes) {
    TRY(ensure(b, bytes + 64));
    if (bytes) HIP_TRY(hipMemcpyAsync(b.p, src, bytes, hipMemcpyHostToDevice, c->stream));
    return KDTN_OK;
}

// Dictionary arena + offsets, uploading only what follows the first `keep` strings (offs[keep],
// the kept prefix's end, stays the device's own: the keep checks compare it with the host's).
// The copies go on `hs` (the context stream unless a delta overlaps them with its kernels).
int upload_dict(kdtn_ctx* c, DevBuf& bytes, DevBuf& offs, const kdtn_strtab& t, uint32_t keep, hipStream_t hs) {
    const size_t b0 = t.offs[keep], b1 = t.offs[t.n];
    TRY(ensure_keep(bytes, b1 + 64, keep ? b0 : 0, c->stream));
    TRY(ensure_keep(offs, ((size_t)t.n + 1) * 4, keep ? ((size_t)keep + 1) * 4 : 0, c->stream));
    if (b1 > b0) HIP_TRY(hipMemcpyAsync(static_cast<uint8_t*>(bytes.p) + b0, t.bytes + b0, b1 - b0,
                                        hipMemcpyHostToDevice, hs));
    const uint32_t o0 = keep ? keep + 1 : 0;
    if (t.n + 1 > o0)
        HIP_TRY(hipMemcpyAsync(static_cast<uint32_t*>(offs.p) + o0, t.offs + o0, ((size_t)t.n + 1 - o0) * 4,
                               hipMemcpyHostToDevice, hs));
    return KDTN_OK;
}

// k_reconcile sync block: 16 B (ticket, error word) + 3 look-back granules per workgroup,
// padded to 16 B (memset size % 16 == 0, cdna_hip_programming.md G16)
// ticket + error word, look-back granules [nwg*3] u64, then VAR_DIFF counts and bases [nwg*3] u32 each
// (16-B aligned: k_place_scan reads and writes them as uint4)
size_t sync_counts_at(uint32_t nwg) { return align_up(SYNC_HEADER_BYTES + (size_t)nwg * 24, 16); }
size_t sync_bytes(uint32_t nwg) { return sync_counts_at(nwg) + 2 * align_up((size_t)nwg * 12, 16); }

// from: the kept prefix of an append-only upload (its offsets were checked when uploaded and
// check_keep compares offs[keep] with the device copy), so only [from, n] is walked
int check_strtab(const kdtn_strtab& t, const char* what, uint32_t from = 0) {
    if (t.n == 0 || !t.offs || (!t.bytes && t.offs[t.n] != 0)) {
        std::snprintf(g_last_error, sizeof(g_last_error), "%s: empty dictionary (id 0 must be \"\")", what);
        return KDTN_EINVAL;
    }
    if (t.n >= 0x7FFFFFFFu) {
        std::snprintf(g_last_error, sizeof(g_last_error), "%s: too many strings", what);
        return KDTN_EINVAL;
    }
    if (t.offs[0] != 0 || t.offs[1] != 0) {
        std::snprintf(g_last_error, sizeof(g_last_error), "%s: id 0 must be the empty string", what);
        return KDTN_EINVAL;
    }
    for (uint32_t i = from < t.n ? from : t.n; i < t.n; ++i)
        if (t.offs[i + 1] < t.offs[i]) {
            std::snprintf(g_last_error, sizeof(g_last_error), "%s: offsets not monotone at %u", what, i);
            return KDTN_EINVAL;
        }
    return KDTN_OK;
}

int check_ids(const uint32_t* col, uint32_t n, uint32_t lim, const char* what) {
    if (n && !col) {
        std::snprintf(g_last_error, sizeof(g_last_error), "%s: missing column", what);
        return KDTN_EINVAL;
    }
    uint32_t mx = 0;
    for (uint32_t i = 0; i < n; ++i) mx = std::max(mx, col[i]);
    if (n && mx >= lim) {
        std::snprintf(g_last_error, sizeof(g_last_error), "%s: id %u out of range (%u strings)", what, mx, lim);
        return KDTN_EINVAL;
    }
    return KDTN_OK;
}

int check_offsets(const uint32_t* off, uint32_t T, uint32_t n, const char* what) {
    if (!off) {
        std::snprintf(g_last_error, sizeof(g_last_error), "%s: missing offsets", what);
        return KDTN_EINVAL;
    }
    if (off[0] != 0 || off[T] != n) {
        std::snprintf(g_last_error, sizeof(g_last_error), "%s: offsets must span [0,%u]", what, n);
        return KDTN_EINVAL;
    }
    for (uint32_t t = 0; t < T; ++t)
        if (off[t + 1] < off[t]) {
            std::snprintf(g_last_error, sizeof(g_last_error), "%s: offsets not monotone at %u", what, t);
            return KDTN_EINVAL;
        }
    return KDTN_OK;
}

constexpr uint32_t STAGED_UPLOAD_MIN = 1u << 16;   // records: below it, 2-D copies straight into tiles

// A link table's columns as host runs: consecutive columns whose host arrays are adjacent (a
// caller holding key[7][n] / prop[12][n] blocks) become one copy into the staging buffer.
// segs (optional): the column ranges of the copies, in copy order, each followed by an event
// on hs (c->ev_col[k]); returns their count in *nseg
int stage_columns(kdtn_ctx* c, uint8_t* st, const kdtn_link_table& L, size_t col, hipStream_t hs,
                  uint32_t (*segs)[2] = nullptr, int* nseg = nullptr) {
    const uint32_t* src[LINK_COLS32];
    for (int k = 0; k < KDTN_NKEY; ++k) src[COL_KEY0 + k] = L.key[k];
    for (int k = 0; k < KDTN_NPROP; ++k) src[COL_PROP0 + k] = L.prop[k];
    src[COL_GAP] = L.gap;
    int ns = 0;
    for (int a = 0; a < LINK_COLS32;) {
        int b = a + 1;
        while (b < LINK_COLS32 && reinterpret_cast<const uint8_t*>(src[b]) ==
                                      reinterpret_cast<const uint8_t*>(src[b - 1]) + col)
            ++b;
        HIP_TRY(hipMemcpyAsync(st + (size_t)a * col, src[a], (size_t)(b - a) * col, hipMemcpyHostToDevice, hs));
        if (segs) {
            segs[ns][0] = (uint32_t)a;
            segs[ns][1] = (uint32_t)b;
            HIP_TRY(hipEventRecord(c->ev_col[ns], hs));
        }
        ++ns;
        a = b;
    }
    if (nseg) *nseg = ns;
    return KDTN_OK;
}

// defer: the id-range check's column maxima stay in misc[MISC_COLMAX..] for the caller to read
// back with its own synchronisation (the staged path is then taken for any size)
int upload_links(kdtn_ctx* c, DevLinkStore& s, const kdtn_link_table& L, uint32_t D, uint32_t P,
                 const char* what, bool defer = false) {
    const uint32_t n = L.n;
    for (int k = 0; k < KDTN_NKEY; ++k)
        if (n && !L.key[k]) return check_ids(L.key[k], n, D, what);          // missing column
    for (int k = 0; k < KDTN_NPROP; ++k)
        if (n && !L.prop[k]) return check_ids(L.prop[k], n, P, what);
    if (n && (!L.uid || !L.gap)) {
        std::snprintf(g_last_error, sizeof(g_last_error), "%s: missing uid/gap", what);
        return KDTN_EINVAL;
    }
    const size_t tiles = ((size_t)std::max<uint32_t>(n, 1) + TILE_RECS - 1) / TILE_RECS;
    const size_t tile_bytes = (size_t)TILE_WORDS * 4;
    TRY(ensure(s.buf, tiles * tile_bytes));
    uint8_t* base = static_cast<uint8_t*>(s.buf.p);
    s.view.base = reinterpret_cast<const uint32_t*>(base);
    s.view.n = n;
    s.n = n;
    if (n >= STAGED_UPLOAD_MIN || defer) {
        // large tables: one linear copy per column (full host-link rate) into a staging buffer,
        // then the tiles and the id-range check in one GPU pass (no host pass over the columns)
        const size_t col = (size_t)n * 4, uid_at = align_up(col * LINK_COLS32, 8);
        TRY(ensure(c->stage, uid_at + (size_t)n * 8 + 128));
        uint8_t* st = static_cast<uint8_t*>(c->stage.p);
        TRY(ensure(c->misc, 256));
        uint32_t* colmax = reinterpret_cast<uint32_t*>(static_cast<uint8_t*>(c->misc.p) + MISC_COLMAX * 4);
        HIP_TRY(hipMemsetAsync(colmax, 0, COL_GAP * 4, c->stream));
        if (!n) return KDTN_OK;
        TRY(stage_columns(c, st, L, col, c->stream));
        HIP_TRY(hipMemcpyAsync(st + uid_at, L.uid, (size_t)n * 8, hipMemcpyHostToDevice, c->stream));
        k_soa_to_tiles<<<std::min<uint32_t>((n + BLOCK - 1) / BLOCK, 4 * c->n_cus), BLOCK, 0, c->stream>>>(
            reinterpret_cast<const uint32_t*>(st), reinterpret_cast<const int64_t*>(st + uid_at), n,
            reinterpret_cast<uint32_t*>(base), colmax);
        HIP_TRY(hipGetLastError());
        if (defer) return KDTN_OK;
        uint32_t mx[COL_GAP];
        HIP_TRY(hipMemcpyAsync(mx, colmax, sizeof(mx), hipMemcpyDeviceToHost, c->stream));
        HIP_TRY(hipStreamSynchronize(c->stream));
        for (int k = 0; k < COL_GAP; ++k) {
            const uint32_t lim = k < KDTN_NKEY ? D : P;
            if (mx[k] >= lim) {
                std::snprintf(g_last_error, sizeof(g_last_error), "%s: id %u out of range (%u strings)", what, mx[k], lim);
                return KDTN_EINVAL;
            }
        }
        return KDTN_OK;
    }
    for (int k = 0; k < KDTN_NKEY; ++k) TRY(check_ids(L.key[k], n, D, what));
    for (int k = 0; k < KDTN_NPROP; ++k) TRY(check_ids(L.prop[k], n, P, what));
    // tiles of 64 records (kdtn_kernels.h DevLinks): each column is a 2-D copy with a
    // 256-B (uid: 512-B) run per tile
    auto put = [&](int col, const void* src, size_t esz) -> int {
        const size_t full = n / TILE_RECS, tail = n % TILE_RECS;
        const size_t run = TILE_RECS * esz;
        uint8_t* dst = base + (size_t)col * TILE_RECS * 4;
        if (full)
            HIP_TRY(hipMemcpy2DAsync(dst, tile_bytes, src, run, run, full, hipMemcpyHostToDevice, c->stream));
        if (tail)
            HIP_TRY(hipMemcpyAsync(dst + full * tile_bytes, static_cast<const uint8_t*>(src) + full * run,
                                   tail * esz, hipMemcpyHostToDevice, c->stream));
        return KDTN_OK;
    };
    if (n) {
        for (int k = 0; k < KDTN_NKEY; ++k) TRY(put(COL_KEY0 + k, L.key[k], 4));
        for (int k = 0; k < KDTN_NPROP; ++k) TRY(put(COL_PROP0 + k, L.prop[k], 4));
        TRY(put(COL_GAP, L.gap, 4));
        TRY(put(COL_UID, L.uid, 8));
    }
    return KDTN_OK;
}

uint32_t nblocks(uint64_t n, int block = BLOCK) { return (uint32_t)((n + block - 1) / block); }

// Each timing event costs ≈5 µs of stream time on MI355X (measured: two consecutive marks
// with nothing between them read 5.4 µs), so epoch stages are marked at a level.
void timer_mark(kdtn_ctx* c, const char* name, int level = 0) {
    if (c->n_ev >= kMaxTimers || c->timing < level) return;
    c->ev_name[c->n_ev] = name;
    (void)hipEventRecord(c->ev[c->n_ev + 1], c->stream);
    c->n_ev++;
}

DevTopos topo_view(kdtn_ctx* c) {
    DevTopos t;
    t.ns = dp<uint32_t>(c->t_ns);
    t.name = dp<uint32_t>(c->t_name);
    t.src_ip = dp<uint32_t>(c->t_src);
    t.net_ns = dp<uint32_t>(c->t_netns);
    t.flags = dp<uint8_t>(c->t_flags);
    t.real_off = dp<uint32_t>(c->t_roff);
    t.des_off = dp<uint32_t>(c->t_noff);
    t.n = c->T;
    return t;
}

// Parse the property strings [p0, n): one thread per (string, interpretation) when split
// (three launches' worth of waves in one grid), else one thread per string.
void launch_pdict(kdtn_ctx* c, uint32_t p0, uint32_t n) {
    bool split = KDTN_PD_SPLIT_DEFAULT;
#if KDTN_PROFILING
    if (const char* ev = std::getenv("KDTN_PD_SPLIT")) split = std::atoi(ev) != 0;
    if (const char* ev = std::getenv("KDTN_PD_ONLY")) {           // one interpretation alone (A/B)
        const int w = std::atoi(ev);
        auto one = [&](auto kern) {
            kern<<<nblocks(n - p0), BLOCK, 0, c->stream>>>(dp<uint8_t>(c->pd_bytes), dp<uint32_t>(c->pd_offs), p0, n,
                                                          c->cfg.tick_in_usec, dp<uint32_t>(c->pd_pct),
                                                          dp<uint2>(c->pd_dur), dp<uint2>(c->pd_rate),
                                                          dp<uint32_t>(c->pd_rerr));
        };
        if (w == PD_DUR) { one(k_pdict_only<PD_DUR>); return; }
        if (w == PD_PCT) { one(k_pdict_only<PD_PCT>); return; }
        if (w == PD_RATE) { one(k_pdict_only<PD_RATE>); return; }
        if (w == (PD_RATE | PD_RATE_GENERIC)) { one(k_pdict_only<PD_RATE | PD_RATE_GENERIC>); return; }
    }
#endif
    const dim3 grid(nblocks(n - p0), split ? 3 : 1);
    auto go = [&](auto kern) {
        kern<<<grid, BLOCK, 0, c->stream>>>(dp<uint8_t>(c->pd_bytes), dp<uint32_t>(c->pd_offs), p0, n,
                                            c->cfg.tick_in_usec, dp<uint32_t>(c->pd_pct), dp<uint2>(c->pd_dur),
                                            dp<uint2>(c->pd_rate), dp<uint32_t>(c->pd_rerr));
    };
    if (split) go(k_pdict_parse<true>);
    else go(k_pdict_parse<false>);
}

// Special key-string ids (SPECIAL_DEFAULT / SPECIAL_LOCALHOST) at or past the parse start
// are forgotten when an upload sets it; every run's k_kdict_flags re-finds them there.
void clip_specials(kdtn_ctx* c) {
    if (c->kd_special.p) k_special_clip<<<1, 64, 0, c->stream>>>(dp<uint32_t>(c->kd_special), c->kd_from & ~63u);
}

// per-string parse tables of both dictionaries (c->D, c->P set), keeping the parsed
// tables of the first c->kd_valid / c->pd_valid strings. kbits holds KB_NSETS bitsets at a
// stride of kb_cap words; growing the stride moves each set.
int prepare_dicts(kdtn_ctx* c) {
    const uint32_t D = c->D, P = c->P;
    hipStream_t s = c->stream;
    const uint32_t need = (uint32_t)(((uint64_t)D + 63) / 64 * 2);
    if (need > c->kb_cap || !c->kd_bits.p) {
        // stride a multiple of 2 words (kdtn_kernels.h kb_words): growth by 1.5x rounded up
        const uint32_t cap = (std::max<uint32_t>(need, c->kd_valid ? c->kb_cap + c->kb_cap / 2 : 0) + 1u) & ~1u;
        DevBuf nb;
        TRY(ensure(nb, (size_t)KB_NSETS * cap * 4 + 4));
        const uint32_t keepw = (uint32_t)(((uint64_t)c->kd_valid + 63) / 64 * 2);
        if (keepw && c->kd_bits.p)
            HIP_TRY(hipMemcpy2DAsync(nb.p, (size_t)cap * 4, c->kd_bits.p, (size_t)c->kb_cap * 4, (size_t)keepw * 4,
                                     KB_NSETS, hipMemcpyDeviceToDevice, s));
        release(c->kd_bits);                 // retired: stream-ordered after the copy
        c->kd_bits = nb;
        c->kb_cap = cap;
    }
    c->kb_words = c->kb_cap;
    const size_t pv = c->pd_valid;
    TRY(ensure_keep(c->pd_pct, (size_t)P * 4, pv * 4, s));
    TRY(ensure_keep(c->pd_dur, (size_t)P * 8, pv * 8, s));
    TRY(ensure_keep(c->pd_rate, (size_t)P * 8, pv * 8, s));
    TRY(ensure_keep(c->pd_rerr, (size_t)nblocks(P) * BLOCK / 8, (pv + 63) / 64 * 8, s));
    TRY(ensure(c->kd_special, 64));
    clip_specials(c);
    return KDTN_OK;
}

// VxlanManager snapshot ids valid for a dictionary of D strings. KDTN_VNI_RESIDENT needs a
// resident map whose ids still name the same strings: the upload keeps (kdict_keep) at least
// the vres_D strings the map was made for — every upload since kept that prefix, since an
// upload that kept less either replaced the map or was refused here. A dictionary the engine
// builds itself (JSON ingest) cannot keep a prefix (keep = 0).
int check_vnis(kdtn_ctx* c, const kdtn_vni_table& vn, uint32_t D, uint32_t keep) {
    if (vn.n == KDTN_VNI_RESIDENT) {
        if (!c->vres_ok || keep < c->vres_D || D < c->vres_D) {
            std::snprintf(g_last_error, sizeof(g_last_error),
                          "KDTN_VNI_RESIDENT: the resident VXLAN map's ids (%u strings) are not a kept prefix "
                          "of this dictionary (kdict_keep %u)", c->vres_D, keep);
            return KDTN_EINVAL;
        }
        return KDTN_OK;
    }
    TRY(check_ids(vn.node, vn.n, D, "vnis.node"));
    return check_ids(vn.net_ns, vn.n, D, "vnis.net_ns");
}

// Append-only dictionaries: the first *_keep strings equal the previous upload's (the arena
// offset of the kept prefix is checked against the device copy).
int check_keep(kdtn_ctx* c, const kdtn_strtab& kd, const kdtn_strtab& pd, uint32_t kk, uint32_t pk) {
    const uint32_t D = kd.n, P = pd.n;
    uint32_t dev_off[2] = {0, 0};
    if (kk <= c->kd_valid && kk && kk <= D)
        HIP_TRY(hipMemcpyAsync(dev_off, dp<uint32_t>(c->kd_offs) + kk, 4, hipMemcpyDeviceToHost, c->stream));
    if (pk <= c->pd_valid && pk && pk <= P)
        HIP_TRY(hipMemcpyAsync(dev_off + 1, dp<uint32_t>(c->pd_offs) + pk, 4, hipMemcpyDeviceToHost, c->stream));
    if (kk || pk) HIP_TRY(hipStreamSynchronize(c->stream));
    if (kk > D || pk > P || kk > c->kd_valid || pk > c->pd_valid || (kk && kd.offs[kk] != dev_off[0]) ||
        (pk && pd.offs[pk] != dev_off[1])) {
        std::snprintf(g_last_error, sizeof(g_last_error),
                      "kdict_keep %u / pdict_keep %u: not a prefix of the previous upload's parsed dictionaries "
                      "(%u / %u strings)", kk, pk, c->kd_valid, c->pd_valid);
        return KDTN_EINVAL;
    }
    return KDTN_OK;
}

// upload the dictionaries past the kept prefixes and size their parsed tables
int upload_dicts(kdtn_ctx* c, const kdtn_strtab& kd, const kdtn_strtab& pd, uint32_t kk, uint32_t pk,
                 hipStream_t hs = nullptr) {
    if (!hs) hs = c->stream;
    c->D = kd.n;
    c->P = pd.n;
    // strings past the kept prefix may differ: an index that covers them is rebuilt (mask 0)
    if (kk < c->ix_k.n) c->ix_k.n = c->ix_k.mask = 0;
    if (pk < c->ix_p.n) c->ix_p.n = c->ix_p.mask = 0;
    c->kd_arena = kd.offs[kd.n];
    c->pd_arena = pd.offs[pd.n];
    c->kd_valid = kk;
    c->pd_valid = pk;
    c->kd_from = kk;
    c->pd_from = pk;
    c->si_k = std::min(c->si_k, kk);
    c->si_p = std::min(c->si_p, pk);
    TRY(upload_dict(c, c->kd_bytes, c->kd_offs, kd, kk, hs));
    TRY(upload_dict(c, c->pd_bytes, c->pd_offs, pd, pk, hs));
    return prepare_dicts(c);
}

// A sharded ingest's rank setup ends when the next upload or ingest starts.
void end_shard_ingest(kdtn_ctx* c) {
    if (!c->sh_active) return;
    c->nranks = c->sh_saved_nranks;
    c->rank = c->sh_saved_rank;
    c->pods_rank_major = true;
    c->pods_imported = false;
    c->pods_ready = false;                        // the pod table was in document order
    c->sh_T = 0;
    c->sh_active = false;
}

// everything an epoch needs besides its input tables: VNI snapshot, pod tables, work and
// output buffers (c->D, c->T set; shared by kdtn_epoch_upload and kdtn_json_ingest)
int prepare_vnis(kdtn_ctx* c, const kdtn_vni_table& vn) {
    const uint32_t D = c->D;
    const bool resident = vn.n == KDTN_VNI_RESIDENT;
    const uint32_t V = resident ? c->vres_n : vn.n;
    c->V = V;
    if (!resident) {
        TRY(upload(c, c->v_node, vn.node, (size_t)V * 4));
        TRY(upload(c, c->v_vni, vn.vni, (size_t)V * 4));
        TRY(upload(c, c->v_netns, vn.net_ns, (size_t)V * 4));
        c->vres_ok = true;                      // the uploaded map stays resident
        c->vres_in_r = false;
        c->vres_n = V;
        c->vres_D = D;
    } else if (c->vres_in_r) {                  // the applied map becomes this upload's snapshot
        std::swap(c->v_node, c->r_node);
        std::swap(c->v_vni, c->r_vni);
        std::swap(c->v_netns, c->r_netns);
        c->vres_in_r = false;
    }
    c->vni_mask = V ? next_pow2((uint64_t)V * 2) - 1 : 0;
    TRY(ensure(c->v_ents, (size_t)V * 16));
    TRY(ensure(c->v_slots, (size_t)(c->vni_mask + 1) * 4));
    TRY(ensure(c->v_table, (size_t)(c->vni_mask + 1) * 16));
    return KDTN_OK;
}

// pod tables, work and output buffers for T = c->T topologies, M realised and N desired records
int prepare_work(kdtn_ctx* c, uint32_t slice, uint32_t M, uint32_t N) {
    const uint32_t D = c->D;
    if (slice != c->slice) c->pods_ready = false;
    c->slice = slice;
    if ((uint64_t)slice * (uint64_t)c->nranks > POD_INDEX) {
        std::snprintf(g_last_error, sizeof(g_last_error), "pod table of %llu entries exceeds 2^30",
                      (unsigned long long)slice * (unsigned long long)c->nranks);
        return KDTN_EINVAL;
    }
    c->pod_total = slice * (uint32_t)c->nranks;
    if (c->n_late) c->pods_ready = false;
    c->n_late = 0;
    c->ovf_mask = next_pow2((uint64_t)c->pod_total * 2) - 1;
    TRY(ensure(c->pods, (size_t)c->pod_total * 16));
    if (c->pod_ovf.cap < (size_t)(c->ovf_mask + 1) * 8) {       // stamped slots start zeroed
        TRY(ensure(c->pod_ovf, (size_t)(c->ovf_mask + 1) * 8));
        HIP_TRY(hipMemsetAsync(c->pod_ovf.p, 0, c->pod_ovf.cap, c->stream));
    }
    if (c->pod_direct.cap < (size_t)D * 16) {                  // stamps start from a zeroed table
        // headroom for append-only dictionaries: slots of ids past the last build read as empty
        // (stamp 0), so a delta upload that adds strings keeps the built table
        TRY(ensure(c->pod_direct, (size_t)D * 16 + (size_t)D * 4 + 4096));
        HIP_TRY(hipMemsetAsync(c->pod_direct.p, 0, c->pod_direct.cap, c->stream));   // stamp 0 = empty
        c->pods_ready = false;
    }

    const uint32_t nwg = (c->T + TPW - 1) / TPW;
    c->nwg = nwg;
    TRY(ensure(c->otarget, (size_t)M * 4));
    TRY(ensure(c->sync, sync_bytes(nwg)));
    TRY(ensure(c->misc, 256));
    TRY(ensure(c->hscratch, ((size_t)M + N) * 4));
    TRY(ensure(c->fscratch, (size_t)M + N));
    TRY(ensure(c->action, c->T));
    TRY(ensure(c->del_off, (size_t)(c->T + 1) * 4));
    TRY(ensure(c->add_off, (size_t)(c->T + 1) * 4));
    TRY(ensure(c->upd_off, (size_t)(c->T + 1) * 4));
    // the comparison build (both lists non-empty) emits deferred chunks into upper halves
    const size_t h = (M && N) ? 2 : 1;
    TRY(ensure(c->del_idx, h * M * 4));
    TRY(ensure(c->upd_idx, h * M * 4));
    TRY(ensure(c->add_idx, h * N * 4));
    TRY(ensure(c->del_res, h * M * 16));
    TRY(ensure(c->upd_res, h * M * 16));
    TRY(ensure(c->add_res, h * N * 16));
    TRY(ensure(c->upd_qdisc, h * M * 72));
    TRY(ensure(c->add_qdisc, h * N * 72));
    TRY(ensure(c->add_qerr, h * N + 16));
    return KDTN_OK;
}

int prepare_epoch(kdtn_ctx* c, const kdtn_vni_table& vn, uint32_t slice, uint32_t M, uint32_t N) {
    TRY(prepare_vnis(c, vn));
    return prepare_work(c, slice, M, N);
}

// The last run's list totals in h_misc[1..3] (and the look-back error in [4]), from the coherent
// host words k_reconcile writes: read_totals once the run has completed (kdtn_epoch_sync);
// counts_fresh for an output stage called without kdtn_epoch_sync waits for the run first, so
// no stage sizes its passes from the counts of an earlier epoch.
int read_totals(kdtn_ctx* c) {              // (the run has completed)
    for (int i = 0; i < 4; ++i) c->h_misc[1 + i] = __atomic_load_n(c->h_tot + i, __ATOMIC_ACQUIRE);
    if (c->h_misc[4] != 0) {
        std::snprintf(g_last_error, sizeof(g_last_error), "k_reconcile look-back timed out (0x%x)", c->h_misc[4]);
        return KDTN_EIO;
    }
    c->synced = true;
    return KDTN_OK;
}
int counts_fresh(kdtn_ctx* c) {
    if (c->synced) return KDTN_OK;
    HIP_TRY(hipStreamSynchronize(c->stream));
    return read_totals(c);
}

// Which batch entries the daemons reach (k_reach; include/kdtn.h): c->f_send (add) and
// c->f_reach_upd (update) flags of the last run; stamps destination daemons into `mark`.
// coarse entry -> topology indexes of the last run's del / add / upd lists (k_list_coarse),
// built by the first output stage after a run
int list_coarse(kdtn_ctx* c) {
    if (c->lc_valid) return KDTN_OK;
    const uint32_t cnt[3] = {c->h_misc[1], c->h_misc[3], c->h_misc[2]};   // del, add, upd
    DevBuf* offs[3] = {&c->del_off, &c->add_off, &c->upd_off};
    for (int l = 0; l < 3; ++l) {
        TRY(ensure(c->lc[l], ((size_t)cnt[l] / 64 + 2) * 4));
        if (c->T && cnt[l])
            k_list_coarse<<<nblocks(c->T), BLOCK, 0, c->stream>>>(dp<uint32_t>(*offs[l]), c->T, dp<uint32_t>(c->lc[l]));
    }
    HIP_TRY(hipGetLastError());
    c->lc_valid = true;
    return KDTN_OK;
}

int run_reach(kdtn_ctx* c, uint32_t* mark, uint32_t stamp) {
    const uint32_t nu = c->h_misc[2], na = c->h_misc[3];
    TRY(ensure(c->f_send, (size_t)na + 16));
    TRY(ensure(c->f_reach_upd, (size_t)nu + 16));
    ReachIn r{dp<uint32_t>(c->del_off), dp<uint4>(c->del_res), dp<uint32_t>(c->add_off), dp<uint4>(c->add_res),
              dp<uint2>(c->add_qdisc), dp<uint32_t>(c->upd_off), dp<uint4>(c->upd_res), c->T, stamp,
              dp<uint8_t>(c->add_qerr), nullptr, nullptr, nullptr};
    TRY(list_coarse(c));
    r.add_coarse = dp<uint32_t>(c->lc[1]);
    r.upd_coarse = dp<uint32_t>(c->lc[2]);
    if (mark) {                                     // the fan-out: dense node ids for its passes
        TRY(ensure(c->f_node, (size_t)na * 4 + 16));
        r.add_node = dp<uint32_t>(c->f_node);
    }
    const uint32_t nd = c->h_misc[1];
    TRY(ensure(c->f_cut, (size_t)c->T * 12 + 12));
    TRY(ensure(c->f_st, (size_t)na + 16));
    uint32_t* cut = dp<uint32_t>(c->f_cut);
    if (c->T) {
        HIP_TRY(hipMemsetAsync(cut, 0xFF, (size_t)c->T * 12, c->stream));
        if ((uint64_t)nd + na + nu)
            k_reach_cuts<<<nblocks((uint64_t)nd + na + nu), BLOCK, 0, c->stream>>>(r, nd, na, nu, cut,
                                                                                    dp<uint8_t>(c->f_st));
        if ((uint64_t)na + nu)
            k_reach<<<nblocks((uint64_t)na + nu), BLOCK, 0, c->stream>>>(r, na, nu, cut, dp<uint8_t>(c->f_st), mark,
                                                                         dp<uint8_t>(c->f_send),
                                                                         dp<uint8_t>(c->f_reach_upd));
    }
    return KDTN_OK;
}

// The encoders' inline string tables (StrTab) of both dictionaries, on the context stream,
// built by the first output stage after a run (the later stages of the epoch share them). Like
// the dictionary parses, the work is a function of the upload: the strings from the upload's
// keep index (and any never built) on; the entries before it are kept.
int str_tables(kdtn_ctx* c) {
    if (c->si_run && c->si_k == c->D && c->si_p == c->P) return KDTN_OK;
    hipStream_t s = c->stream;
    const uint32_t k0 = std::min(c->si_k, c->kd_from), p0 = std::min(c->si_p, c->pd_from);
    TRY(ensure_keep(c->kd_si, (size_t)c->D * SI_KW * 4 + 16, (size_t)k0 * SI_KW * 4, s));
    TRY(ensure_keep(c->kd_len1, (size_t)c->D + 16, k0, s));
    TRY(ensure_keep(c->pd_si, (size_t)c->P * SI_PW * 4 + 16, (size_t)p0 * SI_PW * 4, s));
    TRY(ensure_keep(c->pd_len1, (size_t)c->P + 16, p0, s));
    if (c->D > k0)
        k_str_inline<SI_KW><<<nblocks(c->D - k0), BLOCK, 0, s>>>(dp<uint8_t>(c->kd_bytes), dp<uint32_t>(c->kd_offs) + k0,
                                                                c->D - k0, dp<uint32_t>(c->kd_si) + (size_t)k0 * SI_KW,
                                                                dp<uint8_t>(c->kd_len1) + k0);
    if (c->P > p0)
        k_str_inline<SI_PW><<<nblocks(c->P - p0), BLOCK, 0, s>>>(dp<uint8_t>(c->pd_bytes), dp<uint32_t>(c->pd_offs) + p0,
                                                                c->P - p0, dp<uint32_t>(c->pd_si) + (size_t)p0 * SI_PW,
                                                                dp<uint8_t>(c->pd_len1) + p0);
    HIP_TRY(hipGetLastError());
    c->si_k = c->D;
    c->si_p = c->P;
    c->si_run = true;
    return KDTN_OK;
}

StrTab str_tab_kd(kdtn_ctx* c) {
    return StrTab{dp<uint32_t>(c->kd_si), dp<uint8_t>(c->kd_len1), dp<uint8_t>(c->kd_bytes)};
}
StrTab str_tab_pd(kdtn_ctx* c) {
    return StrTab{dp<uint32_t>(c->pd_si), dp<uint8_t>(c->pd_len1), dp<uint8_t>(c->pd_bytes)};
}

// exclusive scan of n u32 values into n+1 u64 offsets (out[n] = total): partial sums, a
// one-block scan of the partials, the final pass. (A single-pass decoupled look-back over
// 1024-value blocks measured slower on the output stages: 132 vs 52 us for 10M values, the
// look-back round trips of ~10k small blocks in the critical path.)
int scan_u32(kdtn_ctx* c, const uint32_t* in, uint32_t n, uint64_t* out) {
    const uint32_t nb = nblocks((uint64_t)n + 1, SCAN_CHUNK);
    TRY(ensure(c->j_part, (size_t)nb * 8));
    hipStream_t s = c->stream;
    k_scan_partial<<<nb, BLOCK, 0, s>>>(in, n, dp<uint64_t>(c->j_part));
    k_scan_top<<<1, SCAN_TOP_BLOCK, 0, s>>>(dp<uint64_t>(c->j_part), nb);
    k_scan_final<<<nb, BLOCK, 0, s>>>(in, n, dp<uint64_t>(c->j_part), out);
    HIP_TRY(hipGetLastError());
    return KDTN_OK;
}


}  // namespace

// ======================================================================================
// C-ABI
// ======================================================================================
extern "C" {

const char* kdtn_version(void) { return "kdtn-mi355x 0.1 (abi 1, gfx950)"; }

const char* kdtn_strerror(int code) {
    switch (code) {
    case KDTN_OK: return "ok";
    case KDTN_EINVAL: return g_last_error[0] ? g_last_error : "invalid argument";
    case KDTN_ENOMEM: return g_last_error[0] ? g_last_error : "out of memory";
    case KDTN_EIO: return g_last_error[0] ? g_last_error : "HIP/RCCL runtime error";
    case KDTN_ENOSPC: return "output capacity too small";
    case KDTN_ENODEV: return g_last_error[0] ? g_last_error : "no usable gfx950 device";
    default: return "unknown error";
    }
}

const char* kdtn_err_name(int e) {
    static const char* names[] = {"none", "veth_cidr", "veth_mac", "latency", "latency_corr",
                                  "jitter", "loss", "loss_corr", "duplicate", "duplicate_corr",
                                  "reorder_prob", "reorder_corr", "corrupt_prob", "corrupt_corr",
                                  "rate", "peer_lookup", "peer_no_links", "peer_veth_cidr",
                                  "peer_veth_mac", "remote_cidr"};
    if (e < 0 || e >= (int)(sizeof(names) / sizeof(names[0]))) return "unknown";
    return names[e];
}

double kdtn_psched_tick_in_usec(void) {
    // netlink initClock(): /proc/net/psched "t2us us2t clock_res hz" in hex
    FILE* f = std::fopen("/proc/net/psched", "r");
    if (!f) return 0.0;
    unsigned long long v[4];
    int got = std::fscanf(f, "%llx %llx %llx %llx", &v[0], &v[1], &v[2], &v[3]);
    std::fclose(f);
    if (got != 4 || v[1] == 0) return 0.0;
    if (v[2] == 1000000000ull) v[0] = v[1];
    const double clock_factor = (double)v[2] / 1000000.0;
    return (double)v[0] / (double)v[1] * clock_factor;
}

int kdtn_init(kdtn_ctx** out, const kdtn_config* cfg) {
    if (!out || !cfg) return KDTN_EINVAL;
    *out = nullptr;
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0) {
        std::snprintf(g_last_error, sizeof(g_last_error), "no HIP device visible");
        return KDTN_ENODEV;
    }
    int dev = cfg->device;
    if (dev < 0) HIP_TRY(hipGetDevice(&dev));
    if (dev >= ndev) return KDTN_EINVAL;
    HIP_TRY(hipSetDevice(dev));
    hipDeviceProp_t prop;
    HIP_TRY(hipGetDeviceProperties(&prop, dev));
    if (std::strncmp(prop.gcnArchName, "gfx950", 6) != 0) {
        std::snprintf(g_last_error, sizeof(g_last_error), "device %d is %s, libkdtn is built for gfx950",
                      dev, prop.gcnArchName);
        return KDTN_ENODEV;
    }
    kdtn_ctx* c = new kdtn_ctx();
    c->device = dev;
    c->cfg = *cfg;
    c->n_cus = (uint32_t)std::max(1, prop.multiProcessorCount);
    if (hipStreamCreateWithFlags(&c->own_stream, hipStreamNonBlocking) != hipSuccess) {
        delete c;
        return KDTN_EIO;
    }
    c->stream = c->own_stream;
    // words [0, 16): epoch sync header copy; [64, 128): the misc words a delta reads back
    if (hipHostMalloc(reinterpret_cast<void**>(&c->h_misc), 512, hipHostMallocDefault) != hipSuccess ||
        hipHostMalloc(reinterpret_cast<void**>(&c->h_tot), 64, hipHostMallocCoherent) != hipSuccess) {
        if (c->h_misc) (void)hipHostFree(c->h_misc);
        (void)hipStreamDestroy(c->own_stream);
        delete c;
        return KDTN_ENOMEM;
    }
    std::memset(c->h_tot, 0, 64);
    // timing events only (read after a stream sync): no system-scope fence, whose L2 write-back
    // and invalidate at every mark cost the timed epoch stream time
    for (int i = 0; i <= kMaxTimers; ++i) (void)hipEventCreateWithFlags(&c->ev[i], hipEventDisableSystemFence);
    (void)hipEventCreateWithFlags(&c->ev_done, hipEventDisableTiming);
    for (hipEvent_t& e : c->ev_cp) (void)hipEventCreateWithFlags(&e, hipEventDisableTiming);
    for (hipEvent_t& e : c->ev_col) (void)hipEventCreateWithFlags(&e, hipEventDisableTiming);
    if (hipStreamCreateWithFlags(&c->copy_stream, hipStreamNonBlocking) != hipSuccess) c->copy_stream = nullptr;
    if (hipStreamCreateWithFlags(&c->side_stream, hipStreamNonBlocking) != hipSuccess) c->side_stream = nullptr;
    {
        int lo = 0, hi = 0;
        if (hipDeviceGetStreamPriorityRange(&lo, &hi) != hipSuccess ||
            hipStreamCreateWithPriority(&c->side_hi, hipStreamNonBlocking, hi) != hipSuccess)
            c->side_hi = nullptr;
    }
    if (hipEventCreateWithFlags(&c->ev_front, hipEventDisableTiming) != hipSuccess) c->ev_front = nullptr;
    if (hipEventCreateWithFlags(&c->ev_side, hipEventDisableTiming) != hipSuccess) c->ev_side = nullptr;
    if (hipStreamCreateWithFlags(&c->d2h_stream, hipStreamNonBlocking) != hipSuccess) c->d2h_stream = nullptr;
    (void)hipEventCreateWithFlags(&c->ev_dl_ready, hipEventDisableTiming);
    (void)hipEventCreateWithFlags(&c->ev_dl_done, hipEventDisableTiming);
    *out = c;
    return KDTN_OK;
}

void kdtn_destroy(kdtn_ctx* c) {
    if (!c) return;
    (void)hipSetDevice(c->device);
    (void)kdtn_epoch_download_wait(c);
    (void)hipStreamSynchronize(c->stream);
    if (c->comm_stream) (void)hipStreamSynchronize(c->comm_stream);
    DevBuf* bufs[] = {&c->kd_bytes, &c->kd_offs, &c->kd_bits, &c->pd_bytes, &c->pd_offs,
                      &c->pd_pct, &c->pd_dur, &c->pd_rate, &c->pd_rerr, &c->t_ns, &c->t_name, &c->t_src,
                      &c->t_netns, &c->t_flags, &c->t_roff, &c->t_noff, &c->real.buf, &c->des.buf,
                      &c->v_node, &c->v_vni, &c->v_netns, &c->v_ents, &c->v_slots, &c->v_table, &c->pods,
                      &c->pod_ovf, &c->pod_direct, &c->otarget, &c->sync, &c->misc, &c->hscratch,
                      &c->fscratch, &c->action, &c->del_off, &c->add_off, &c->upd_off, &c->del_idx,
                      &c->add_idx, &c->upd_idx, &c->del_res, &c->add_res, &c->upd_res,
                      &c->add_qdisc, &c->upd_qdisc, &c->add_qerr, &c->kd_si, &c->kd_len1, &c->pd_si, &c->pd_len1, &c->w_rel,
                      &c->w_topo, &c->w_size, &c->w_err, &c->w_off, &c->w_part, &c->w_arena, &c->w_pinfo,
                      &c->f_mark, &c->f_send, &c->f_node_idx, &c->f_nodes, &c->f_counts, &c->f_base,
                      &c->f_part, &c->f_idx, &c->f_inv, &c->f_st, &c->f_node, &c->lc[0], &c->lc[1], &c->lc[2], &c->f_reach_upd, &c->tc_size, &c->tc_off, &c->tc_part, &c->tc_arena,
                      &c->j_doc, &c->j_q, &c->j_bs, &c->j_hb, &c->j_esc, &c->j_qcnt, &c->j_qoff, &c->j_tok, &c->j_open,
                      &c->j_close, &c->j_gcnt, &c->j_goff, &c->j_toks, &c->j_par,
                      &c->j_role, &c->j_ecls, &c->j_odep, &c->j_ord, &c->j_tagg, &c->j_gagg, &c->j_cnt3, &c->j_coff3, &c->j_small,
                      &c->j_part, &c->j_tflags, &c->j_owner, &c->j_rows, &c->j_kkeys, &c->j_pkeys, &c->j_vown, &c->j_kslots, &c->j_krep,
                      &c->j_pslots, &c->j_prep, &c->j_heap, &c->j_bits, &c->j_bcnt, &c->j_wrank,
                      &c->j_kslot_id, &c->j_pslot_id, &c->j_len, &c->j_off64, &c->j_sofid,
                      &c->j_olist, &c->j_vlist, &c->j_slist, &c->sh_keep, &c->sh_kreal,
                      &c->sh_kdes, &c->sh_tidx, &c->sh_roff64, &c->sh_noff64, &c->sh_doc, &c->sh_ns,
                      &c->sh_name, &c->sh_src, &c->sh_netns, &c->sh_flags, &c->sh_roff, &c->sh_noff,
                      &c->sh_des.buf, &c->sh_real.buf, &c->vx_ops, &c->vx_dead, &c->vx_slots, &c->vx_node,
                      &c->vx_vni, &c->vx_netns, &c->vx_part, &c->vx_cut, &c->f_cut, &c->vx_vis,
                      &c->r_node, &c->r_vni, &c->r_netns, &c->rp_flag, &c->rp_pos, &c->rp_phys,
                      &c->rp_msz, &c->rp_moff, &c->rp_tsz, &c->rp_toff, &c->rp_part, &c->rp_arena, &c->rp_tc, &c->rp_msz_e, &c->rp_tsz_e,
                      &c->st_cnt, &c->st_len, &c->st_base, &c->st_mode, &c->st_flags, &c->st_off64, &c->st_part,
                      &c->st_off32, &c->st_mask, &c->st_chg, &c->dl_topo, &c->dl_src, &c->dl_netns, &c->dl_nil,
                      &c->dl_off, &c->dl_ref, &c->dl_rec.buf, &c->stage, &c->vx_cnt, &c->vx_send, &c->vx_recv,
                      &c->vx_gops, &c->pd_send, &c->pd_recv, &c->pd_cnt, &c->dl_rows, &c->vx_flag,
                      &c->vx_dkeys, &c->vx_dused, &c->vx_cpos, &c->vx_cpart, &c->vx_cnode, &c->vx_cvni,
                      &c->dl_prev, &c->dl_ns, &c->dl_name, &c->dl_dest, &c->dl_pack, &c->st_rlen, &c->st_rbase, &c->st_roff64,
                      &c->st_rpart, &c->st_roff32, &c->st_seen, &c->ji_ns, &c->ji_name, &c->ji_src, &c->ji_netns,
                      &c->ji_flags, &c->ji_roff, &c->ji_noff, &c->ji_kb, &c->ji_ko, &c->ji_pb, &c->ji_po,
                      &c->ji_des.buf, &c->ji_real.buf, &c->ji_kmap, &c->ji_pmap, &c->ji_miss, &c->ji_mlen,
                      &c->ji_rank, &c->ji_boff, &c->ji_nil, &c->ji_keep, &c->ji_kpos, &c->ji_claim, &c->ji_res,
                      &c->ji_created, &c->ji_cpos, &c->ji_keys, &c->ji_vals, &c->ji_dkeys, &c->ji_del, &c->ji_ref,
                      &c->ix_k.slots, &c->ix_p.slots};
    for (DevBuf* b : bufs) release(*b);
    retired_flush();
    for (int i = 0; i <= kMaxTimers; ++i)
        if (c->ev[i]) (void)hipEventDestroy(c->ev[i]);
    if (c->comm) (void)ncclCommDestroy(c->comm);
    if (c->comm_stream) (void)hipStreamDestroy(c->comm_stream);
    if (c->ev_fill) (void)hipEventDestroy(c->ev_fill);
    if (c->ev_ag) (void)hipEventDestroy(c->ev_ag);
    if (c->ev_done) (void)hipEventDestroy(c->ev_done);
    for (hipEvent_t e : c->ev_cp)
        if (e) (void)hipEventDestroy(e);
    for (hipEvent_t e : c->ev_col)
        if (e) (void)hipEventDestroy(e);
    if (c->copy_stream) {
        (void)hipStreamSynchronize(c->copy_stream);
        (void)hipStreamDestroy(c->copy_stream);
    }
    for (hipStream_t st : {c->side_stream, c->side_hi})
        if (st) {
            (void)hipStreamSynchronize(st);
            (void)hipStreamDestroy(st);
        }
    if (c->ev_front) (void)hipEventDestroy(c->ev_front);
    if (c->ev_side) (void)hipEventDestroy(c->ev_side);
    if (c->d2h_stream) {
        (void)hipStreamSynchronize(c->d2h_stream);
        (void)hipStreamDestroy(c->d2h_stream);
    }
    if (c->ev_dl_ready) (void)hipEventDestroy(c->ev_dl_ready);
    if (c->ev_dl_done) (void)hipEventDestroy(c->ev_dl_done);
    if (c->sdma_inited) {
        (void)hsa_signal_destroy(c->dl_sig);
        (void)hsa_shut_down();                      // (balances sdma_setup's hsa_init)
    }
    if (c->h_misc) (void)hipHostFree(c->h_misc);
    if (c->h_tot) (void)hipHostFree(c->h_tot);
    if (c->own_stream) (void)hipStreamDestroy(c->own_stream);
    delete c;
}

int kdtn_set_stream(kdtn_ctx* c, void* s) {
    if (!c) return KDTN_EINVAL;
    c->stream = s ? static_cast<hipStream_t>(s) : c->own_stream;
    return KDTN_OK;
}

int kdtn_epoch_upload(kdtn_ctx* c, const kdtn_epoch_in* in) {
    if (!c || !in) return KDTN_EINVAL;
    HIP_TRY(hipSetDevice(c->device));
    g_last_error[0] = 0;
    end_shard_ingest(c);
    TRY(check_strtab(in->kdict, "kdict", in->kdict_keep));
    TRY(check_strtab(in->pdict, "pdict", in->pdict_keep));
    const kdtn_topo_table& T = in->topos;
    const uint32_t D = in->kdict.n, P = in->pdict.n;
    TRY(check_offsets(T.real_off, T.n, in->realised.n, "topos.real_off"));
    TRY(check_offsets(T.des_off, T.n, in->desired.n, "topos.des_off"));
    if (T.n && (!T.flags)) return KDTN_EINVAL;
    TRY(check_ids(T.ns, T.n, D, "topos.ns"));
    TRY(check_ids(T.name, T.n, D, "topos.name"));
    TRY(check_ids(T.src_ip, T.n, D, "topos.src_ip"));
    TRY(check_ids(T.net_ns, T.n, D, "topos.net_ns"));
    for (uint32_t t = 0; t < T.n; ++t) {
        if ((T.flags[t] & KDTN_TOPO_STATUS_NIL) && T.real_off[t + 1] != T.real_off[t]) {
            std::snprintf(g_last_error, sizeof(g_last_error), "topology %u: status.links nil but non-empty", t);
            return KDTN_EINVAL;
        }
        if ((T.flags[t] & KDTN_TOPO_SPEC_NIL) && T.des_off[t + 1] != T.des_off[t]) {
            std::snprintf(g_last_error, sizeof(g_last_error), "topology %u: spec.links nil but non-empty", t);
            return KDTN_EINVAL;
        }
    }
    TRY(check_vnis(c, in->vnis, D, in->kdict_keep));
    const uint32_t slice = in->pod_slice ? in->pod_slice : T.n;
    if (slice < T.n) return KDTN_EINVAL;

    TRY(check_keep(c, in->kdict, in->pdict, in->kdict_keep, in->pdict_keep));
    c->uploaded = false;                            // a failure from here on leaves no usable epoch
    c->T = T.n;
    TRY(upload_dicts(c, in->kdict, in->pdict, in->kdict_keep, in->pdict_keep));

    TRY(upload(c, c->t_ns, T.ns, (size_t)T.n * 4));
    TRY(upload(c, c->t_name, T.name, (size_t)T.n * 4));
    TRY(upload(c, c->t_src, T.src_ip, (size_t)T.n * 4));
    TRY(upload(c, c->t_netns, T.net_ns, (size_t)T.n * 4));
    TRY(upload(c, c->t_flags, T.flags, (size_t)T.n));
    TRY(upload(c, c->t_roff, T.real_off, (size_t)(T.n + 1) * 4));
    TRY(upload(c, c->t_noff, T.des_off, (size_t)(T.n + 1) * 4));

    TRY(upload_links(c, c->real, in->realised, D, P, "realised"));
    TRY(upload_links(c, c->des, in->desired, D, P, "desired"));

    c->pods_rank_major = true;
    TRY(prepare_epoch(c, in->vnis, slice, in->realised.n, in->desired.n));
    HIP_TRY(hipStreamSynchronize(c->stream));   // host arrays may be released after return
    c->uploaded = true;
    c->ran = false;
    c->pods_imported = false;
    c->j_done = false;                             // the tables are no ingest's any more
    c->tables_cur = false;
    c->pods_ready = false;                         // new rows: the next run builds the pod tables
    c->pods_delta = false;
    return KDTN_OK;
}

// The VxlanManager snapshot's lookup table on the context stream (k_vni_pack / _ht_build / _fill).
static int build_vni_table(kdtn_ctx* c) {
    hipStream_t s = c->stream;
    const size_t vcap = (size_t)c->vni_mask + 1;
    HIP_TRY(hipMemsetAsync(c->v_slots.p, 0xFF, vcap * 4, s));
    k_vni_pack<<<nblocks(c->V), BLOCK, 0, s>>>(dp<uint32_t>(c->v_node), dp<int32_t>(c->v_vni),
                                              dp<uint32_t>(c->v_netns), c->V, dp<uint4>(c->v_ents));
    k_vni_ht_build<<<nblocks(c->V), BLOCK, 0, s>>>(dp<uint4>(c->v_ents), c->V, dp<uint32_t>(c->v_slots),
                                                  c->vni_mask);
    k_vni_fill<<<nblocks(vcap), BLOCK, 0, s>>>(dp<uint4>(c->v_ents), dp<uint32_t>(c->v_slots), (uint32_t)vcap,
                                               dp<uint4>(c->v_table));
    return KDTN_OK;
}

int kdtn_epoch_run(kdtn_ctx* c, uint32_t stages) {
    if (!c || !c->uploaded) return KDTN_EINVAL;
    HIP_TRY(hipSetDevice(c->device));
    stages |= KDTN_STAGE_DIFF;
    c->last_stages = stages;
    c->n_ev = 0;
    hipStream_t s = c->stream;
    const DevTopos T = topo_view(c);
    const bool resolve = stages & KDTN_STAGE_RESOLVE;
    // pod tables already current (patched by kdtn_epoch_upload_delta): no fill, exchange or build
    const bool pods_cur = resolve && c->pods_delta && c->pods_ready;
    const bool host_xchg = resolve && !pods_cur && c->nranks > 1 && !c->comm;   // rows imported by the caller
    const bool exchange = resolve && !pods_cur && c->comm;                       // RCCL (a 1-rank comm too)
    if (host_xchg && !c->pods_imported) {
        std::snprintf(g_last_error, sizeof(g_last_error),
                      "host transport: kdtn_pods_import the gathered pod table before kdtn_epoch_run");
        return KDTN_EINVAL;
    }
    if (c->dl_pending) {                                          // outputs still being copied out
        if (c->dl_sdma) TRY(kdtn_epoch_download_wait(c));
        else HIP_TRY(hipStreamWaitEvent(s, c->ev_dl_done, 0));
    }
    // the previous epoch's kernels are done once its sync returned, so these host stores cannot
    // race a device write; an epoch without topologies leaves them zero
    for (int i = 0; i < 4; ++i) __atomic_store_n(c->h_tot + i, 0u, __ATOMIC_RELAXED);
    if (c->timing >= 2) (void)hipEventRecord(c->ev[0], s);
    uint32_t* sync = dp<uint32_t>(c->sync);
    // Epoch front: first launch (sync header, look-back area, pod-status rows) + RCCL
    // all-gather, the dictionary parses, the pod lookup tables, in sequence. The tables need
    // nothing from the parses, but running them beside a long key-string parse did not shorten
    // the epoch (config 2): on a side stream 0.791-0.796 vs 0.789 ms (profiles/r03u_side_ab.json),
    // fused into the parse launches 0.804 vs 0.793 ms (profiles/r06ae_fuse_ab.json). When the key
    // strings to parse are few (a churn epoch's appended strings, configs 1 and 4) the five
    // launches are the cost, and one local rank fuses them into two: k_epoch_front (sync header,
    // pod rows and their lookup slots, key strings) and k_pdict_verify (slot verify, full-prefix
    // scan, property strings): config-3 churn epochs 0.762 -> 0.741 ms, config 4 0.246 -> 0.240,
    // config 1 0.223 -> 0.206 (profiles/r06ad_fuse_churn.json, r06ae_fuse_ab.json).
    constexpr uint32_t FUSE_MAX_KSTRINGS = 4u << 20;
    int fuse_mode = (c->D - std::min(c->D, c->kd_from & ~63u)) < FUSE_MAX_KSTRINGS ? 1 : 0;
#if KDTN_PROFILING
    if (const char* ev = std::getenv("KDTN_FUSE")) fuse_mode = std::atoi(ev);
#endif
    const bool fused = fuse_mode && resolve && !pods_cur && c->nranks == 1 && !c->comm && c->pod_total &&
                       c->pod_total == c->slice && !c->n_late;
    const uint32_t pod_rows = c->pod_total + c->n_late;             // gathered table + late pods
    uint32_t* special = dp<uint32_t>(c->kd_special);
    const uint32_t n16 = (uint32_t)(sync_bytes(c->nwg) / 16);
    const uint32_t nbz = std::min<uint32_t>(nblocks(n16), 256);
    // the pod lookup tables (scatter, then verify fused with the full-prefix scan) on a side
    // stream beside the dictionary parses, which they do not need (the PHYSICAL bit of a pod's
    // name comes from its bytes): the comm stream right after the RCCL all-gather, else
    // side_stream after the first launch; k_reconcile waits for them
#if KDTN_PROFILING
    int side_mode = KDTN_LOOKUP_SIDE_DEFAULT;
    if (const char* ev = std::getenv("KDTN_LOOKUP_SIDE")) side_mode = std::atoi(ev);
#else
    constexpr int side_mode = KDTN_LOOKUP_SIDE_DEFAULT;
#endif
    hipStream_t ls = exchange ? c->comm_stream : (side_mode == 2 && c->side_hi ? c->side_hi : c->side_stream);
    const bool side = side_mode && !fused && resolve && pod_rows && !pods_cur && c->T && ls && c->ev_front && c->ev_side;
    // 4 pod rows per thread in the lookup build (every row load issued before the dependent
    // accesses): rank of 8 0.1761 / 0.1770 → 0.1735 / 0.1744 ms, N = 1 0.7895 → 0.7883 ms
    // (profiles/r05h_pod_per_ab_*)
#if KDTN_PROFILING
    int pod_per = 4;                                                 // (A/B: KDTN_POD_PER = 1, 2, 4)
    if (const char* ev = std::getenv("KDTN_POD_PER")) pod_per = std::atoi(ev);
#else
    constexpr int pod_per = 4;
#endif
    auto lookup_build = [&](hipStream_t q, bool parsed) -> int {
        if (++c->pod_stamp >= 0x7FFFFFFFu) {                             // stamp wrap: clear once
            HIP_TRY(hipMemsetAsync(c->pod_direct.p, 0, c->pod_direct.cap, q));
            HIP_TRY(hipMemsetAsync(c->pod_ovf.p, 0, c->pod_ovf.cap, q));
            c->pod_stamp = 1;
        }
        auto kern = pod_per == 4 ? k_pod_direct_scatter<4> : k_pod_direct_scatter<1>;
#if KDTN_PROFILING
        if (pod_per == 2) kern = k_pod_direct_scatter<2>;
#endif
        kern<<<nblocks(pod_rows, BLOCK * pod_per), BLOCK, 0, q>>>(
            dp<uint4>(c->pods), pod_rows, parsed ? dp<uint32_t>(c->kd_bits) + (size_t)KB_PHYSICAL * c->kb_words : nullptr,
            dp<uint8_t>(c->kd_bytes), dp<uint32_t>(c->kd_offs), dp<uint4>(c->pod_direct), c->pod_stamp, c->D,
            c->pods_rank_major ? (uint32_t)c->nranks : 1u, c->pod_total);
        return KDTN_OK;
    };
    auto verify_prefix = [&](hipStream_t q) {
        const uint32_t nbv = nblocks(pod_rows, BLOCK * pod_per);
        const uint32_t nbp = (uint32_t)std::min<uint64_t>(4 * FP_GRID, (c->T + 4 * BLOCK - 1) / (4 * BLOCK));
        auto kern = pod_per == 4 ? k_pod_verify_prefix<4> : k_pod_verify_prefix<1>;
#if KDTN_PROFILING
        if (pod_per == 2) kern = k_pod_verify_prefix<2>;
#endif
        kern<<<nbv + std::max<uint32_t>(nbp, 1), BLOCK, 0, q>>>(
            dp<uint4>(c->pods), pod_rows, dp<uint4>(c->pod_direct), c->pod_stamp,
            dp<unsigned long long>(c->pod_ovf), c->ovf_mask, c->D, T, sync + SYNC_FIRST_PARTIAL_INV, nbv,
            c->pods_rank_major ? (uint32_t)c->nranks : 1u, c->pod_total);
    };
    if (fused) {
        if (++c->pod_stamp >= 0x7FFFFFFFu) {                             // stamp wrap: clear once
            HIP_TRY(hipMemsetAsync(c->pod_direct.p, 0, c->pod_direct.cap, s));
            HIP_TRY(hipMemsetAsync(c->pod_ovf.p, 0, c->pod_ovf.cap, s));
            c->pod_stamp = 1;
        }
        const uint32_t k0 = c->kd_from & ~63u, p0 = c->pd_from & ~63u;  // (clip_specials ran at upload)
        const uint32_t nbs = nblocks(c->slice);
        const uint32_t nbk = c->D > k0 ? nblocks(c->D - k0) : 0u;
        k_epoch_front<<<nbz + nbs + nbk, BLOCK, 0, s>>>(
            reinterpret_cast<uint4*>(sync), n16, nbz, nbs, T, c->slice, dp<uint4>(c->pods), dp<uint4>(c->pod_direct),
            c->pod_stamp, dp<uint8_t>(c->kd_bytes), dp<uint32_t>(c->kd_offs), k0, c->D, dp<uint32_t>(c->kd_bits),
            c->kb_words, special);
        timer_mark(c, "epoch_front", 2);
        if (c->V) {
            TRY(build_vni_table(c));
            timer_mark(c, "hash_build", 2);
        }
        const uint32_t nbv = nblocks(c->pod_total);
        const uint32_t nbp = std::max<uint32_t>(1, (uint32_t)std::min<uint64_t>(4 * FP_GRID, (c->T + 4 * BLOCK - 1) / (4 * BLOCK)));
        const uint32_t nbd = c->P > p0 ? nblocks(c->P - p0) : 0u;
        k_pdict_verify<<<nbv + nbp + 3 * nbd, BLOCK, 0, s>>>(
            dp<uint4>(c->pods), c->pod_total, dp<uint4>(c->pod_direct), c->pod_stamp, dp<unsigned long long>(c->pod_ovf),
            c->ovf_mask, c->D, T, sync + SYNC_FIRST_PARTIAL_INV, nbv, nbp, dp<uint8_t>(c->pd_bytes),
            dp<uint32_t>(c->pd_offs), p0, c->P, nbd, c->cfg.tick_in_usec, dp<uint32_t>(c->pd_pct), dp<uint2>(c->pd_dur),
            dp<uint2>(c->pd_rate), dp<uint32_t>(c->pd_rerr));
        timer_mark(c, "pdict_verify", 2);
    } else {
        // k_epoch_begin zeroes the sync header (SYNC_*) and look-back area and fills this rank's
        // pod-status rows. With RCCL it runs on the comm stream, followed there by the
        // all-gather, beside this stream's dictionary parses; otherwise it follows the parses on
        // this stream, so the epoch's first launch is a long one and the host's later launches
        // are queued while it runs (a 2.5-µs first kernel left the GPU idle ≈ 5 µs for the next
        // launch, profiles/r05c_shardstats_trace.csv)
        const uint32_t fill = (resolve && !host_xchg && !pods_cur) ? c->slice : 0u;
        const uint32_t rank_base = c->slice * (uint32_t)c->rank;
        auto begin = [&](hipStream_t q) {
            k_epoch_begin<<<nbz + nblocks(fill), BLOCK, 0, q>>>(reinterpret_cast<uint4*>(sync), n16, nbz, T, fill,
                                                                rank_base, dp<uint4>(c->pods));
        };
        const bool begin_first = side && !exchange;                 // (A/B: the lookup build waits for it)
        if (exchange) {
            HIP_TRY(hipEventRecord(c->ev_fill, s));                   // after the previous epoch's kernels
            HIP_TRY(hipStreamWaitEvent(c->comm_stream, c->ev_fill, 0));
            begin(c->comm_stream);
            uint4* pods = dp<uint4>(c->pods);
            ncclResult_t r = ncclAllGather(pods + rank_base, pods, (size_t)c->slice * 4, ncclUint32, c->comm,
                                           c->comm_stream);
            if (r != ncclSuccess) {
                std::snprintf(g_last_error, sizeof(g_last_error), "ncclAllGather: %s", ncclGetErrorString(r));
                return KDTN_EIO;
            }
            HIP_TRY(hipEventRecord(c->ev_ag, c->comm_stream));
        } else if (begin_first) {
            begin(s);
            timer_mark(c, "pods_fill", 2);
        }
        if (side) {
            if (!exchange) {
                HIP_TRY(hipEventRecord(c->ev_front, s));
                HIP_TRY(hipStreamWaitEvent(ls, c->ev_front, 0));
            }
            TRY(lookup_build(ls, false));
            verify_prefix(ls);
            HIP_TRY(hipEventRecord(c->ev_side, ls));
        }
        // dictionaries: the strings this upload added (all of them unless kdict_keep /
        // pdict_keep), from a multiple of 64 so every wave writes whole predicate words
        uint32_t* special = dp<uint32_t>(c->kd_special);
#if KDTN_PROFILING
        int dict_fuse = KDTN_DICT_FUSE_DEFAULT ? 1 : 0;
        if (const char* ev = std::getenv("KDTN_DICT_FUSE")) dict_fuse = std::atoi(ev);
#else
        constexpr int dict_fuse = KDTN_DICT_FUSE_DEFAULT ? 1 : 0;
#endif
        const uint32_t k0f = c->kd_from & ~63u, p0f = c->pd_from & ~63u;
        if (dict_fuse && c->D > k0f && c->P > p0f) {              // both parses in one launch
            const uint32_t nbk = nblocks(c->D - k0f), nbp = nblocks(c->P - p0f);
            auto kern = k_dict_parse;
#if KDTN_PROFILING
            if (dict_fuse >= 3) kern = k_dict_parse_w7;                  // (3: values first, 4: keys first)
#endif
            kern<<<3 * nbp + nbk, BLOCK, 0, s>>>(
                dp<uint8_t>(c->kd_bytes), dp<uint32_t>(c->kd_offs), k0f, c->D, dp<uint32_t>(c->kd_bits), c->kb_words,
                special, dp<uint8_t>(c->pd_bytes), dp<uint32_t>(c->pd_offs), p0f, c->P, nbp, c->cfg.tick_in_usec,
                dp<uint32_t>(c->pd_pct), dp<uint2>(c->pd_dur), dp<uint2>(c->pd_rate), dp<uint32_t>(c->pd_rerr),
                (dict_fuse == 2 || dict_fuse == 4) ? nbk : 0u);
            timer_mark(c, "dict_parse", 2);
        } else {
        {
            const uint32_t k0 = c->kd_from & ~63u;                        // (clip_specials ran at upload)
            if (c->D > k0) {
                const uint8_t* kb = dp<uint8_t>(c->kd_bytes);
                const uint32_t* ko = dp<uint32_t>(c->kd_offs);
                uint32_t* bits = dp<uint32_t>(c->kd_bits);
                const uint32_t nk = c->D - k0;
    #if KDTN_PROFILING
                int sub = 1;                                               // strings per thread (2, 4: slower)
                if (const char* ev = std::getenv("KDTN_KD_SUB")) sub = std::atoi(ev);
                if (sub == 4) k_kdict_flags<4, false, BLOCK><<<nblocks(nk, BLOCK * 4), BLOCK, 0, s>>>(kb, ko, k0, c->D, bits, c->kb_words, special);
                else if (sub == 2) k_kdict_flags<2, false, BLOCK><<<nblocks(nk, BLOCK * 2), BLOCK, 0, s>>>(kb, ko, k0, c->D, bits, c->kb_words, special);
                else if (sub == 8) k_kdict_flags<1, true, BLOCK><<<nblocks(nk), BLOCK, 0, s>>>(kb, ko, k0, c->D, bits, c->kb_words, special);
                else if (sub == 16) k_kdict_flags_ws<<<nblocks(nk), BLOCK, 0, s>>>(kb, ko, k0, c->D, bits, c->kb_words, special);
                else if (sub >= 32 && sub < 40) {
                    const uint32_t nb = std::min(nblocks(nk), (uint32_t)(c->n_cus * 8 * (sub - 31)));
                    k_kdict_flags_pp<<<nb, BLOCK, 0, s>>>(kb, ko, k0, c->D, bits, c->kb_words, special);
                }
                else if (sub == 40) k_kdict_null<<<nblocks(nk), BLOCK, 0, s>>>(kb, ko, k0, c->D, bits, c->kb_words, special);
                else if (sub == 42) k_kdict_flags_v1<<<nblocks(nk), BLOCK, 0, s>>>(kb, ko, k0, c->D, bits, c->kb_words, special);
                else if (sub == 41) k_kdict_loadonly<<<nblocks(nk), BLOCK, 0, s>>>(kb, ko, k0, c->D, bits, c->kb_words, special);
                else if (sub == 64) k_kdict_flags<1, false, 64><<<nblocks(nk, 64), 64, 0, s>>>(kb, ko, k0, c->D, bits, c->kb_words, special);
                else if (sub == 1024) k_kdict_flags<1, false, 1024><<<nblocks(nk, 1024), 1024, 0, s>>>(kb, ko, k0, c->D, bits, c->kb_words, special);
                else
    #endif
                k_kdict_flags<1, false, BLOCK><<<nblocks(nk), BLOCK, 0, s>>>(kb, ko, k0, c->D, bits, c->kb_words, special);
            }
        }
        timer_mark(c, "kdict_parse", 2);
        {
            const uint32_t p0 = c->pd_from & ~63u;
            if (c->P > p0) launch_pdict(c, p0, c->P);
        }
        timer_mark(c, "pdict_parse", 2);
        }
        if (!exchange && !begin_first) {
            begin(s);
            timer_mark(c, "pods_fill", 2);
        }
        if (resolve) {
            if (side) {
                if (c->V) TRY(build_vni_table(c));
                HIP_TRY(hipStreamWaitEvent(s, c->ev_side, 0));             // lookup tables not hidden by the parses
                timer_mark(c, "lookup_wait", 2);
            } else {
                if (exchange) HIP_TRY(hipStreamWaitEvent(s, c->ev_ag, 0));   // exchange not hidden by the parses
                timer_mark(c, "pods_allgather", 2);
                if (pod_rows && !pods_cur) TRY(lookup_build(s, true));
                else if (!pods_cur && ++c->pod_stamp >= 0x7FFFFFFFu) {     // (no rows: the stamp still moves)
                    HIP_TRY(hipMemsetAsync(c->pod_direct.p, 0, c->pod_direct.cap, s));
                    HIP_TRY(hipMemsetAsync(c->pod_ovf.p, 0, c->pod_ovf.cap, s));
                    c->pod_stamp = 1;
                }
                if (c->V) TRY(build_vni_table(c));
                timer_mark(c, "hash_build", 2);
            }
        }
    }
    c->kd_valid = c->D;
    c->pd_valid = c->P;
    if (c->T) {
        DevTables tb{};
        tb.kbits = dp<uint32_t>(c->kd_bits);
        tb.kb_words = c->kb_words;
        tb.ppct = dp<uint32_t>(c->pd_pct);
        tb.pdur = dp<uint2>(c->pd_dur);
        tb.prate = dp<uint2>(c->pd_rate);
        tb.rate_err = dp<uint32_t>(c->pd_rerr);
        tb.pods = dp<uint4>(c->pods);
        tb.pod_direct = dp<uint4>(c->pod_direct);
        tb.pod_stamp = c->pod_stamp;
        tb.pod_ovf = dp<unsigned long long>(c->pod_ovf);
        tb.ovf_mask = c->ovf_mask;
        tb.vnis = dp<uint4>(c->v_table);
        tb.vni_slots = dp<uint32_t>(c->v_slots);
        tb.vni_mask = c->V ? c->vni_mask : 0;
        tb.special = special;
        tb.vxlan_base = c->cfg.vxlan_base;
        RecOut o;
        o.action = dp<uint8_t>(c->action);
        o.del_off = dp<uint32_t>(c->del_off);
        o.add_off = dp<uint32_t>(c->add_off);
        o.upd_off = dp<uint32_t>(c->upd_off);
        o.del_idx = dp<uint32_t>(c->del_idx);
        o.add_idx = dp<uint32_t>(c->add_idx);
        o.upd_idx = dp<uint32_t>(c->upd_idx);
        o.del_res = dp<uint4>(c->del_res);
        o.add_res = dp<uint4>(c->add_res);
        o.upd_res = dp<uint4>(c->upd_res);
        o.add_qdisc = dp<uint2>(c->add_qdisc);
        o.upd_qdisc = dp<uint2>(c->upd_qdisc);
        o.add_qerr = dp<uint8_t>(c->add_qerr);
        o.totals = sync + SYNC_TOTALS;
        o.htotals = c->h_tot;
        o.stages = stages;
        RecWork w;
        w.sync = sync;
        w.herr = c->h_tot + 3;
        w.status = reinterpret_cast<unsigned long long*>(static_cast<char*>(c->sync.p) + SYNC_HEADER_BYTES);
        w.hscratch = dp<uint32_t>(c->hscratch);
        w.fscratch = dp<uint8_t>(c->fscratch);
        w.otarget = dp<uint32_t>(c->otarget);
        w.nwg = c->nwg;
        w.trace = nullptr;
        w.first_partial_inv = sync + SYNC_FIRST_PARTIAL_INV;         // 0 (none) from the memset
        w.wcount = reinterpret_cast<uint32_t*>(static_cast<char*>(c->sync.p) + sync_counts_at(c->nwg));
        w.m_cap = c->real.n;
        w.n_cap = c->des.n;
        uint32_t* wbase = reinterpret_cast<uint32_t*>(reinterpret_cast<char*>(w.wcount) + align_up((size_t)c->nwg * 12, 16));
        bool placed = false;                                        // VAR_DIFF: k_place_scan + k_place
        // several workgroups per chunk when the chunks would not fill the chip about six times
        // over (4 resident k_reconcile workgroups per CU): they share a bulk chunk's records,
        // at least ~300 records per part (measured: 125k-pod config 2, 640 records per chunk:
        // split 2 0.097 ms, 3 0.106, 4 0.115; 100k-site config 4, 1267 per chunk: split 2 / 3 /
        // 4 / 6 / 8 0.156 / 0.158 / 0.150 / 0.174 / 0.166 ms, profiles/r06v_split_sweep.json)
        // Only bulk chunks share their records; in a chunk with comparisons the other parts
        // return at once, so an epoch whose realised lists are a large share of the records
        // runs one workgroup per chunk (config 1, 1274 records per chunk: split 1 / 2 / 4
        // 0.185 / 0.186 / 0.205 ms, the same record)
        const uint64_t per_chunk = ((uint64_t)c->real.n + c->des.n) / std::max<uint32_t>(c->nwg, 1);
        const bool cmp_heavy = (uint64_t)c->real.n * 4 > c->des.n;
        w.split = cmp_heavy ? 1u
                            : std::max<uint32_t>(1, std::min<uint32_t>({4u, (6 * 4 * c->n_cus + c->nwg - 1) / c->nwg,
                                                                        (uint32_t)std::max<uint64_t>(1, per_chunk / 300)}));
#if KDTN_PROFILING
        if (const char* ev = std::getenv("KDTN_SPLIT")) if (std::atoi(ev) > 0) w.split = (uint32_t)std::atoi(ev);
#endif
        if (fused || side) {                            // verify + prefix ran in k_pdict_verify / on the side stream
        } else if (resolve && pod_rows && !pods_cur) {   // the pod-table verify with the full-prefix scan
            verify_prefix(s);
            timer_mark(c, "verify_prefix", 2);
        } else {
            k_full_prefix<<<(unsigned)std::min<uint64_t>(FP_GRID, (c->T + 4 * FP_BLOCK - 1) / (4 * FP_BLOCK)), FP_BLOCK, 0, s>>>(
                T, sync + SYNC_FIRST_PARTIAL_INV);
            timer_mark(c, "full_prefix", 2);
        }
        if (c->timing == 1) (void)hipEventRecord(c->ev[0], s);
#if KDTN_PROFILING
        int variant = DEFAULT_VARIANT;
        if (const char* ev = std::getenv("KDTN_VARIANT")) variant = std::atoi(ev);
        if (variant & VAR_TRACE) {
            w.split = 1;                                           // trace slots per chunk
            TRY(ensure(c->trace, (size_t)c->nwg * TRACE_WORDS * 8));
            w.trace = reinterpret_cast<unsigned long long*>(c->trace.p);
            c->traced = true;
        }
        switch (variant) {
#define KDTN_VARIANT_CASE(V) \
        case V: k_reconcile<V><<<c->nwg * w.split, BLOCK, 0, s>>>(T, c->real.view, c->des.view, tb, o, w); placed = (V & VAR_DIFF) != 0; break;
        KDTN_PROFILING_VARIANTS(KDTN_VARIANT_CASE)
        KDTN_VARIANT_CASE(DIFF_VARIANT)
#undef KDTN_VARIANT_CASE
        default:
            k_reconcile<DEFAULT_VARIANT><<<c->nwg * w.split, BLOCK, 0, s>>>(T, c->real.view, c->des.view, tb, o, w);
            break;
        }
#else
        if (c->real.n && c->des.n) {             // CalcDiff windows: the comparison-heavy build
            k_reconcile<DIFF_VARIANT><<<c->nwg * w.split, BLOCK, 0, s>>>(T, c->real.view, c->des.view, tb, o, w);
            placed = true;
        } else {
            k_reconcile<DEFAULT_VARIANT><<<c->nwg * w.split, BLOCK, 0, s>>>(T, c->real.view, c->des.view, tb, o, w);
        }
#endif
        timer_mark(c, "reconcile", 1);
        if (placed) {
            if ((size_t)c->real.n * 2 > c->del_idx.cap / 4 || (size_t)c->des.n * 2 > c->add_idx.cap / 4) {
                std::snprintf(g_last_error, sizeof(g_last_error), "deferred placement without upper halves");
                return KDTN_EINVAL;
            }
            k_place_scan<<<1, PLACE_SCAN_BLOCK, 0, s>>>(w.wcount, c->nwg, wbase, o, c->T);
            timer_mark(c, "place_scan", 1);
            if (c->nwg >= 4u * c->n_cus) {               // enough chunks for a wave each
                k_place<true><<<(c->nwg + BLOCK / 64 - 1) / (BLOCK / 64), BLOCK, 0, s>>>(
                    T, w.wcount, wbase, w.first_partial_inv, o, w.m_cap, w.n_cap, c->nwg, 1u);
            } else {                                      // workgroups per chunk to fill the chip
                const uint32_t parts = std::min<uint32_t>(16u, std::max<uint32_t>(1u, 4u * c->n_cus / std::max<uint32_t>(c->nwg, 1u)));
                k_place<false><<<c->nwg * parts, BLOCK, 0, s>>>(T, w.wcount, wbase, w.first_partial_inv, o, w.m_cap,
                                                                w.n_cap, c->nwg, parts);
            }
            timer_mark(c, "place", 1);
        }
    } else {
        HIP_TRY(hipMemsetAsync(c->h_tot, 0, 16, s));   // (an earlier run may not have been synced)
        HIP_TRY(hipMemsetAsync(c->del_off.p, 0, 4, s));
        HIP_TRY(hipMemsetAsync(c->add_off.p, 0, 4, s));
        HIP_TRY(hipMemsetAsync(c->upd_off.p, 0, 4, s));
    }
    HIP_TRY(hipGetLastError());
    if (c->ev_done) HIP_TRY(hipEventRecord(c->ev_done, s));
    if (resolve && !pods_cur) c->pods_ready = true;           // the full build of this upload's rows
    c->ran = true;
    c->synced = false;
    c->encoded = false;
    c->tc_done = false;
    c->fan_valid = false;
    c->lc_valid = false;
    c->si_run = false;
    c->rp_done = false;
    c->vx_imported = false;
    c->vx_contest_ok = false;
    return KDTN_OK;
}

int kdtn_epoch_sync(kdtn_ctx* c, kdtn_counts* counts) {
    if (!c || !c->ran) return KDTN_EINVAL;
    HIP_TRY(hipSetDevice(c->device));
    // poll the epoch's completion event (a host-memory signal) for a bounded time before the
    // blocking stream sync: a sub-millisecond epoch is seen ending sooner than from a sleeping
    // wait, and a long one (or a hung GPU) does not hold a host core
    if (c->ev_done) {
        const auto t0 = std::chrono::steady_clock::now();
        while (hipEventQuery(c->ev_done) == hipErrorNotReady &&
               std::chrono::steady_clock::now() - t0 < std::chrono::microseconds(kSyncSpinUs)) {
        }
    }
    HIP_TRY(hipStreamSynchronize(c->stream));
    TRY(read_totals(c));
    if (counts) {
        counts->n_del = c->h_misc[1];
        counts->n_upd = c->h_misc[2];
        counts->n_add = c->h_misc[3];
        counts->n_topos = c->T;
    }
    for (int i = 0; i < c->n_ev; ++i) {                 // this epoch's marks into the totals
        float t = 0.f;
        (void)hipEventElapsedTime(&t, c->ev[i], c->ev[i + 1]);
        int k = 0;
        while (k < c->n_acc && std::strcmp(c->acc_name[k], c->ev_name[i]) != 0) ++k;
        if (k == c->n_acc) {
            if (k == kMaxTimers) continue;
            c->acc_name[k] = c->ev_name[i];
            c->acc_ms[k] = 0.0;
            c->acc_n[k] = 0;
            ++c->n_acc;
        }
        c->acc_ms[k] += t;
        bool first = true;                              // a stage marked in pieces counts once
        for (int j = 0; j < i; ++j) first &= std::strcmp(c->ev_name[j], c->ev_name[i]) != 0;
        if (first) ++c->acc_n[k];
    }
    return KDTN_OK;
}

int kdtn_timer_totals(kdtn_ctx* c, const char** names, double* ms, uint32_t* epochs, int cap, int reset) {
    if (!c || cap < 0) return KDTN_EINVAL;
    const int n = std::min(cap, c->n_acc);
    for (int i = 0; i < n; ++i) {
        if (names) names[i] = c->acc_name[i];
        if (ms) ms[i] = c->acc_ms[i];
        if (epochs) epochs[i] = c->acc_n[i];
    }
    if (reset) c->n_acc = 0;
    return n;
}

// the output copies of kdtn_epoch_download(_async) on stream `hs`
static int download_enqueue(kdtn_ctx* c, kdtn_batches* o, hipStream_t hs) {
    const uint32_t nd = c->h_misc[1], nu = c->h_misc[2], na = c->h_misc[3];
    o->n_del = nd;
    o->n_upd = nu;
    o->n_add = na;
    if (nd > o->del_cap || nu > o->upd_cap || na > o->add_cap) return KDTN_ENOSPC;
    auto d2h = [&](void* dst, DevBuf& b, size_t bytes) -> int {
        if (dst && bytes) HIP_TRY(hipMemcpyAsync(dst, b.p, bytes, hipMemcpyDeviceToHost, hs));
        return KDTN_OK;
    };
    const bool res = c->last_stages & KDTN_STAGE_RESOLVE, q = c->last_stages & KDTN_STAGE_QDISC;
    TRY(d2h(o->action, c->action, c->T));
    TRY(d2h(o->del_off, c->del_off, (size_t)(c->T + 1) * 4));
    TRY(d2h(o->add_off, c->add_off, (size_t)(c->T + 1) * 4));
    TRY(d2h(o->upd_off, c->upd_off, (size_t)(c->T + 1) * 4));
    TRY(d2h(o->del_idx, c->del_idx, (size_t)nd * 4));
    TRY(d2h(o->add_idx, c->add_idx, (size_t)na * 4));
    TRY(d2h(o->upd_idx, c->upd_idx, (size_t)nu * 4));
    if (res) {
        TRY(d2h(o->del_res, c->del_res, (size_t)nd * 16));
        TRY(d2h(o->add_res, c->add_res, (size_t)na * 16));
        TRY(d2h(o->upd_res, c->upd_res, (size_t)nu * 16));
    }
    if (q) {
        TRY(d2h(o->add_qdisc, c->add_qdisc, (size_t)na * 72));
        TRY(d2h(o->upd_qdisc, c->upd_qdisc, (size_t)nu * 72));
    }
    return KDTN_OK;
}

// HSA agents and the SDMA engine for device-to-host copies, once per context
static bool sdma_setup(kdtn_ctx* c) {
    if (c->sdma_tried) return c->sdma_ok;
    c->sdma_tried = true;
    if (hsa_init() != HSA_STATUS_SUCCESS) return false;
    hsa_amd_pointer_info_t dv{}, hv{};
    dv.size = hv.size = sizeof(hsa_amd_pointer_info_t);
    uint32_t mask = 0, pref = 0;
    bool ok = c->sync.p && hsa_amd_pointer_info(c->sync.p, &dv, nullptr, nullptr, nullptr) == HSA_STATUS_SUCCESS &&
              dv.type == HSA_EXT_POINTER_TYPE_HSA &&
              hsa_amd_pointer_info(c->h_misc, &hv, nullptr, nullptr, nullptr) == HSA_STATUS_SUCCESS &&
              hv.type == HSA_EXT_POINTER_TYPE_HSA;
    if (ok) {
        hsa_device_type_t tg = HSA_DEVICE_TYPE_CPU, th = HSA_DEVICE_TYPE_GPU;
        ok = hsa_agent_get_info(dv.agentOwner, HSA_AGENT_INFO_DEVICE, &tg) == HSA_STATUS_SUCCESS &&
             hsa_agent_get_info(hv.agentOwner, HSA_AGENT_INFO_DEVICE, &th) == HSA_STATUS_SUCCESS &&
             tg == HSA_DEVICE_TYPE_GPU && th == HSA_DEVICE_TYPE_CPU &&
             hsa_amd_memory_copy_engine_status(hv.agentOwner, dv.agentOwner, &mask) == HSA_STATUS_SUCCESS && mask;
    }
    if (ok) {
        (void)hsa_amd_memory_get_preferred_copy_engine(hv.agentOwner, dv.agentOwner, &pref);
        const uint32_t pick = (pref & mask) ? (pref & mask) : mask;
        // one engine, the lowest preferred one: beside the runtime's host-to-device copies it
        // keeps 48 GB/s where the H2D-preferred engine falls to 28 (tools/sdma_probe.cpp,
        // profiles/r06c_sdma_probe.jsonl). The download's pieces split over two engines measured
        // no faster (profiles/r06f_resident_engines.jsonl); the profiling build can still ask
        // for two (KDTN_SDMA_ENGINE = two engine bits)
        c->sdma_engine[0] = pick & (~pick + 1u);
        c->sdma_engine[1] = 0;
#if KDTN_PROFILING
        if (const char* ev = std::getenv("KDTN_SDMA_ENGINE")) {        // (A/B) engine bits of the mask
            const uint32_t e = (uint32_t)std::atoi(ev) & mask;
            if (e) {
                c->sdma_engine[0] = e & (~e + 1u);
                const uint32_t r2 = e & ~c->sdma_engine[0];
                c->sdma_engine[1] = r2 & (~r2 + 1u);
            }
        }
#endif
        c->sdma_gpu = dv.agentOwner;
        c->sdma_cpu = hv.agentOwner;
        ok = hsa_signal_create(0, 0, nullptr, &c->dl_sig) == HSA_STATUS_SUCCESS;
    }
    if (!ok) (void)hsa_shut_down();
    c->sdma_ok = c->sdma_inited = ok;
    return ok;
}

// The download's copies on the context's SDMA engine, completion on dl_sig. false (nothing
// issued) when a destination is not page-locked host memory the engine can write, or the
// setup failed: the caller takes the HIP copies. The epoch's kernels have completed (after
// kdtn_epoch_sync, whose completion event carries the system-scope release).
static bool sdma_download(kdtn_ctx* c, kdtn_batches* o) {
    if (!sdma_setup(c)) return false;
    const uint32_t nd = c->h_misc[1], nu = c->h_misc[2], na = c->h_misc[3];
    o->n_del = nd;
    o->n_upd = nu;
    o->n_add = na;
    if (nd > o->del_cap || nu > o->upd_cap || na > o->add_cap) return false;   // (the HIP path reports it)
    struct Piece { void* dst; const void* src; size_t bytes; };
    Piece pc[12];
    int n = 0;
    auto add = [&](void* dst, DevBuf& b, size_t bytes) {
        if (dst && bytes) pc[n++] = Piece{dst, b.p, bytes};
    };
    const bool res = c->last_stages & KDTN_STAGE_RESOLVE, q = c->last_stages & KDTN_STAGE_QDISC;
    add(o->action, c->action, c->T);
    add(o->del_off, c->del_off, (size_t)(c->T + 1) * 4);
    add(o->add_off, c->add_off, (size_t)(c->T + 1) * 4);
    add(o->upd_off, c->upd_off, (size_t)(c->T + 1) * 4);
    add(o->del_idx, c->del_idx, (size_t)nd * 4);
    add(o->add_idx, c->add_idx, (size_t)na * 4);
    add(o->upd_idx, c->upd_idx, (size_t)nu * 4);
    if (res) {
        add(o->del_res, c->del_res, (size_t)nd * 16);
        add(o->add_res, c->add_res, (size_t)na * 16);
        add(o->upd_res, c->upd_res, (size_t)nu * 16);
    }
    if (q) {
        add(o->add_qdisc, c->add_qdisc, (size_t)na * 72);
        add(o->upd_qdisc, c->upd_qdisc, (size_t)nu * 72);
    }
    for (int i = 0; i < n; ++i) {                   // page-locked, and the whole range inside it
        hsa_amd_pointer_info_t pi{};
        pi.size = sizeof pi;
        if (hsa_amd_pointer_info(pc[i].dst, &pi, nullptr, nullptr, nullptr) != HSA_STATUS_SUCCESS) return false;
        if (pi.type != HSA_EXT_POINTER_TYPE_HSA && pi.type != HSA_EXT_POINTER_TYPE_LOCKED) return false;
        uint8_t* b = static_cast<uint8_t*>(pi.hostBaseAddress);
        uint8_t* d = static_cast<uint8_t*>(pc[i].dst);
        if (!b || d < b || d + pc[i].bytes > b + pi.sizeInBytes) return false;
        // Memory registered with hipHostRegister / hsa_amd_memory_lock is reached by the copy
        // engine through its agent address, which need not equal the host address: the
        // engine writes agentBaseAddress + (d - hostBaseAddress). HSA allocations map both alike.
        if (pi.type == HSA_EXT_POINTER_TYPE_LOCKED) {
            if (!pi.agentBaseAddress) return false;
            pc[i].dst = static_cast<uint8_t*>(pi.agentBaseAddress) + (d - b);
        }
    }
    if (!n) return true;
    hsa_signal_store_screlease(c->dl_sig, n);
    {
        SdmaInflight& f = sdma_inflight();
        std::lock_guard<std::mutex> lk(f.m);
        f.sig.push_back(c->dl_sig.handle);
    }
    c->dl_sdma = c->dl_pending = true;
    // pieces to the engine with fewer bytes queued, largest first (one signal counts them all)
    int order[12];
    for (int i = 0; i < n; ++i) order[i] = i;
    std::sort(order, order + n, [&](int a, int b) { return pc[a].bytes > pc[b].bytes; });
    size_t queued[2] = {0, 0};
    for (int k = 0; k < n; ++k) {
        const int i = order[k];
        const int e = (c->sdma_engine[1] && queued[1] < queued[0]) ? 1 : 0;
        queued[e] += pc[i].bytes;
        if (hsa_amd_memory_async_copy_on_engine(pc[i].dst, c->sdma_cpu, pc[i].src, c->sdma_gpu, pc[i].bytes, 0, nullptr,
                                                c->dl_sig, (hsa_amd_sdma_engine_id_t)c->sdma_engine[e],
                                                true) != HSA_STATUS_SUCCESS) {
            hsa_signal_subtract_screlease(c->dl_sig, n - k);       // the pieces never issued
            (void)kdtn_epoch_download_wait(c);
            c->sdma_ok = false;                                    // HIP copies from now on
            return false;
        }
    }
    return true;
}

int kdtn_epoch_download(kdtn_ctx* c, kdtn_batches* o) {
    if (!c || !o || !c->ran) return KDTN_EINVAL;
    HIP_TRY(hipSetDevice(c->device));
    TRY(counts_fresh(c));
    HIP_TRY(hipStreamSynchronize(c->stream));
    TRY(kdtn_epoch_download_wait(c));
    if (sdma_download(c, o)) return kdtn_epoch_download_wait(c);
    TRY(download_enqueue(c, o, c->stream));
    HIP_TRY(hipStreamSynchronize(c->stream));
    return KDTN_OK;
}

// Asynchronous form: the copies run on a stream of their own after the epoch, beside whatever
// the caller enqueues next (commit, the next delta upload's host-to-device copies: the link is
// full duplex); the next kdtn_epoch_run waits for them on the GPU before it overwrites the
// outputs. The host buffers (page-locked, kdtn_host_alloc) hold the outputs once
// kdtn_epoch_download_wait returns. Counts are known at return (after kdtn_epoch_sync).
int kdtn_epoch_download_async(kdtn_ctx* c, kdtn_batches* o) {
    if (!c || !o || !c->ran) return KDTN_EINVAL;
    HIP_TRY(hipSetDevice(c->device));
    TRY(counts_fresh(c));
    TRY(kdtn_epoch_download_wait(c));
    HIP_TRY(hipStreamSynchronize(c->stream));       // (idle after kdtn_epoch_sync: returns at once)
    if (sdma_download(c, o)) return KDTN_OK;
    hipStream_t hs = c->d2h_stream ? c->d2h_stream : c->stream;
    HIP_TRY(hipEventRecord(c->ev_dl_ready, c->stream));
    HIP_TRY(hipStreamWaitEvent(hs, c->ev_dl_ready, 0));
    TRY(download_enqueue(c, o, hs));
    HIP_TRY(hipEventRecord(c->ev_dl_done, hs));
    c->dl_pending = true;
    return KDTN_OK;
}

int kdtn_epoch_download_wait(kdtn_ctx* c) {
    if (!c) return KDTN_EINVAL;
    if (!c->dl_pending) return KDTN_OK;
    if (c->dl_sdma) {
        sdma_wait(c->dl_sig);
        SdmaInflight& f = sdma_inflight();
        std::lock_guard<std::mutex> lk(f.m);
        f.sig.erase(std::remove(f.sig.begin(), f.sig.end(), c->dl_sig.handle), f.sig.end());
        c->dl_sdma = c->dl_pending = false;
        return KDTN_OK;
    }
    HIP_TRY(hipEventSynchronize(c->ev_dl_done));
    c->dl_pending = false;
    return KDTN_OK;
}

int kdtn_reconcile_epoch(kdtn_ctx* c, const kdtn_epoch_in* in, kdtn_batches* out) {
    TRY(kdtn_epoch_upload(c, in));
    TRY(kdtn_epoch_run(c, KDTN_STAGE_ALL));
    TRY(kdtn_epoch_sync(c, nullptr));
    return kdtn_epoch_download(c, out);
}

int kdtn_diff(kdtn_ctx* c, const kdtn_epoch_in* in, kdtn_batches* out) {
    TRY(kdtn_epoch_upload(c, in));
    TRY(kdtn_epoch_run(c, KDTN_STAGE_DIFF));
    TRY(kdtn_epoch_sync(c, nullptr));
    return kdtn_epoch_download(c, out);
}

// One daemon batch as a one-topology epoch: the pods become the topology table (so peer
// lookups see the informer's pods), the batch's links are the local pod's desired list
// (AddLinks: realised non-nil and empty, so every link is an add in query order) or its
// realised list (DelLinks: spec nil, so every link is a delete in query order).
int kdtn_resolve(kdtn_ctx* c, const kdtn_strtab* kdict, const kdtn_strtab* pdict, const kdtn_pod_table* pods,
                 uint32_t local, const kdtn_link_table* links, int batch_kind, const kdtn_vni_table* vnis,
                 kdtn_resolved* out, kdtn_qdisc* qout) {
    if (!c || !kdict || !pdict || !pods || !links || (links->n && !out)) return KDTN_EINVAL;
    if (local >= pods->n || (batch_kind != KDTN_BATCH_ADD && batch_kind != KDTN_BATCH_DEL)) return KDTN_EINVAL;
    if (!pods->ns || !pods->name || !pods->src_ip || !pods->net_ns || !pods->flags) return KDTN_EINVAL;
    const uint32_t P = pods->n, n = links->n;
    const bool add = batch_kind == KDTN_BATCH_ADD;
    std::vector<uint8_t> flags(pods->flags, pods->flags + P);
    std::vector<uint32_t> roff(P + 1, 0), noff(P + 1, 0);
    for (uint32_t t = 0; t < P; ++t) {
        if (t != local) flags[t] |= KDTN_TOPO_STATUS_NIL;             // no entries of their own
        else flags[t] = add ? 0u : (uint8_t)KDTN_TOPO_SPEC_NIL;
        roff[t + 1] = roff[t] + (!add && t == local ? n : 0);
        noff[t + 1] = noff[t] + (add && t == local ? n : 0);
    }
    kdtn_epoch_in in{};
    in.kdict = *kdict;
    in.pdict = *pdict;
    in.topos = kdtn_topo_table{P, pods->ns, pods->name, pods->src_ip, pods->net_ns, flags.data(), roff.data(),
                               noff.data()};
    kdtn_link_table empty{};
    in.realised = add ? empty : *links;
    in.desired = add ? *links : empty;
    if (vnis) in.vnis = *vnis;
    TRY(kdtn_epoch_upload(c, &in));
    TRY(kdtn_epoch_run(c, add ? KDTN_STAGE_ALL : (KDTN_STAGE_DIFF | KDTN_STAGE_RESOLVE)));
    kdtn_counts cnt{};
    TRY(kdtn_epoch_sync(c, &cnt));
    if ((add ? cnt.n_add : cnt.n_del) != n) {
        std::snprintf(g_last_error, sizeof(g_last_error), "kdtn_resolve: %u of %u links planned",
                      add ? cnt.n_add : cnt.n_del, n);
        return KDTN_EIO;
    }
    HIP_TRY(hipSetDevice(c->device));
    if (n) {
        HIP_TRY(hipMemcpyAsync(out, add ? c->add_res.p : c->del_res.p, (size_t)n * 16, hipMemcpyDeviceToHost,
                               c->stream));
        if (add && qout)
            HIP_TRY(hipMemcpyAsync(qout, c->add_qdisc.p, (size_t)n * 72, hipMemcpyDeviceToHost, c->stream));
    }
    HIP_TRY(hipStreamSynchronize(c->stream));
    return KDTN_OK;
}

void* kdtn_host_alloc(uint64_t bytes) {
    void* p = nullptr;
    if (hipHostMalloc(&p, bytes ? bytes : 1, hipHostMallocDefault) != hipSuccess) return nullptr;
    return p;
}

void kdtn_host_free(void* p) {
    if (p) (void)hipHostFree(p);
}

int kdtn_make_qdiscs(kdtn_ctx* c, const kdtn_strtab* pdict, const kdtn_props_table* props,
                     kdtn_qdisc* out) {
    if (!c || !pdict || !props || (!out && props->n)) return KDTN_EINVAL;
    HIP_TRY(hipSetDevice(c->device));
    g_last_error[0] = 0;
    TRY(check_strtab(*pdict, "pdict"));
    const uint32_t P = pdict->n, n = props->n;
    for (int k = 0; k < KDTN_NPROP; ++k) TRY(check_ids(props->prop[k], n, P, "props"));
    if (n && !props->gap) return KDTN_EINVAL;
    c->pd_valid = c->pd_from = c->si_p = 0;                // this call owns the property tables now
    c->ix_p.n = c->ix_p.mask = 0;
    c->uploaded = false;
    TRY(upload_arena(c, c->pd_bytes, pdict->bytes, pdict->offs[P]));
    TRY(upload(c, c->pd_offs, pdict->offs, (size_t)(P + 1) * 4));
    TRY(ensure(c->pd_pct, (size_t)P * 4));
    TRY(ensure(c->pd_dur, (size_t)P * 8));
    TRY(ensure(c->pd_rate, (size_t)P * 8));
    TRY(ensure(c->pd_rerr, (size_t)nblocks(P) * BLOCK / 8));
    // reuse the desired-link store for the property columns
    kdtn_link_table L{};
    L.n = n;
    std::vector<uint32_t> zeros((size_t)std::max<uint32_t>(n, 1), 0u);
    std::vector<int64_t> zuid((size_t)std::max<uint32_t>(n, 1), 0);
    for (int k = 0; k < KDTN_NKEY; ++k) L.key[k] = zeros.data();
    L.uid = zuid.data();
    for (int k = 0; k < KDTN_NPROP; ++k) L.prop[k] = props->prop[k];
    L.gap = props->gap;
    TRY(upload_links(c, c->des, L, 1, P, "props"));
    TRY(ensure(c->add_qdisc, (size_t)std::max<uint32_t>(n, 1) * 72));
    hipStream_t s = c->stream;
    if (P) launch_pdict(c, 0u, P);
    DevTables tb{};
    tb.ppct = dp<uint32_t>(c->pd_pct);
    tb.pdur = dp<uint2>(c->pd_dur);
    tb.prate = dp<uint2>(c->pd_rate);
    tb.rate_err = dp<uint32_t>(c->pd_rerr);
    if (n) k_qdisc_batch<<<nblocks(n), BLOCK, 0, s>>>(c->des.view, tb, dp<uint2>(c->add_qdisc));
    HIP_TRY(hipGetLastError());
    if (n) HIP_TRY(hipMemcpyAsync(out, c->add_qdisc.p, (size_t)n * 72, hipMemcpyDeviceToHost, s));
    HIP_TRY(hipStreamSynchronize(s));
    c->uploaded = false;   // the desired store was reused
    return KDTN_OK;
}

int kdtn_epoch_encode(kdtn_ctx* c, uint64_t* n_bytes) {
    if (!c || !c->ran) return KDTN_EINVAL;
    HIP_TRY(hipSetDevice(c->device));
    HIP_TRY(hipStreamSynchronize(c->stream));
    TRY(counts_fresh(c));
    hipStream_t s = c->stream;
    const uint32_t nd = c->h_misc[1], nu = c->h_misc[2], na = c->h_misc[3];
    const uint32_t T = c->T;
    const uint64_t ne = (uint64_t)nd + na + nu;
    if (ne > 0xFFFFFFFFull || 3ull * T + 1 > 0xFFFFFFFFull) return KDTN_EINVAL;
    TRY(ensure(c->w_rel, (size_t)ne * 4 + 16));                 // entry sizes
    TRY(ensure(c->w_topo, (size_t)ne * 4 + 16));
    TRY(ensure(c->w_size, ((size_t)ne + 1) * 8));                // entry offsets (u64)
    const size_t err_bytes = align_up(((size_t)T + 1) * 4, 16);  // err[T]: a batch over 4 GiB
    TRY(ensure(c->w_err, err_bytes));
    TRY(ensure(c->w_off, ((size_t)3 * T + 1) * 8));
    const uint32_t nb = nblocks(ne + 1, SCAN_CHUNK);
    TRY(ensure(c->w_part, (size_t)nb * 8 + 16));
    c->n_ev = 0;
    (void)hipEventRecord(c->ev[0], s);
    TRY(str_tables(c));
    timer_mark(c, "wire_strtab");
    HIP_TRY(hipMemsetAsync(c->w_err.p, 0, err_bytes, s));
    WireIn w{};
    w.kd = str_tab_kd(c);
    w.pd = str_tab_pd(c);
    TRY(list_coarse(c));
    for (int l = 0; l < 3; ++l) w.coarse[l] = dp<uint32_t>(c->lc[l]);
    w.t_name = dp<uint32_t>(c->t_name);
    w.t_src = dp<uint32_t>(c->t_src);
    w.t_netns = dp<uint32_t>(c->t_netns);
    w.t_ns = dp<uint32_t>(c->t_ns);
    w.list_off[0] = dp<uint32_t>(c->del_off);
    w.list_off[1] = dp<uint32_t>(c->add_off);
    w.list_off[2] = dp<uint32_t>(c->upd_off);
    w.list_idx[0] = dp<uint32_t>(c->del_idx);
    w.list_idx[1] = dp<uint32_t>(c->add_idx);
    w.list_idx[2] = dp<uint32_t>(c->upd_idx);
    w.list_base[0] = 0;
    w.list_base[1] = nd;
    w.list_base[2] = nd + na;
    w.n_entries = (uint32_t)ne;
    w.T = T;
    TRY(ensure(c->w_pinfo, (size_t)na * 8 + 16));
    WireWork wk{dp<uint32_t>(c->w_rel), dp<uint32_t>(c->w_topo), dp<uint64_t>(c->w_size), dp<uint32_t>(c->w_err),
                dp<uint64_t>(c->w_off), dp<uint64_t>(c->w_pinfo)};
    uint64_t total = 0;
    uint32_t big = 0;
    {   // sizes, one scan, then the writer (a single pass with a look-back scan measured slower:
        // 2.85 ms vs 0.79 + 0.14 + 1.78 ms on config 2, profiles/r03g_stages.json)
        if (ne) k_wire_entry_sizes<<<nblocks(ne), BLOCK, 0, s>>>(w, c->real.view, c->des.view, wk);
        timer_mark(c, "wire_sizes");
        k_wire_scan_partial<<<nb, BLOCK, 0, s>>>(w, wk, dp<uint64_t>(c->w_part));
        k_scan_top<<<1, SCAN_TOP_BLOCK, 0, s>>>(dp<uint64_t>(c->w_part), nb);
        k_wire_scan_final<<<nb, BLOCK, 0, s>>>(w, wk, dp<uint64_t>(c->w_part));
        k_wire_batch_off<<<nblocks((uint64_t)3 * T + 1), BLOCK, 0, s>>>(w, wk);
        timer_mark(c, "wire_scan");
        HIP_TRY(hipGetLastError());
        HIP_TRY(hipMemcpyAsync(&total, dp<uint64_t>(c->w_size) + ne, 8, hipMemcpyDeviceToHost, s));
        HIP_TRY(hipMemcpyAsync(&big, dp<uint32_t>(c->w_err) + T, 4, hipMemcpyDeviceToHost, s));
        HIP_TRY(hipStreamSynchronize(s));
        if (!big) TRY(ensure(c->w_arena, (size_t)total + 64));   // (WSink::copy reads past a range)
        timer_mark(c, "wire_host_sync");                // the arena size crosses to the host
        if (ne && !big) k_wire_write<<<nblocks(ne), BLOCK, 0, s>>>(w, c->real.view, c->des.view, wk, dp<uint8_t>(c->w_arena));
        timer_mark(c, "wire_write");
    }
    if (big) {
        std::snprintf(g_last_error, sizeof(g_last_error), "a LinksBatchQuery of more than 4 GiB");
        return KDTN_EINVAL;
    }
    HIP_TRY(hipGetLastError());
    HIP_TRY(hipStreamSynchronize(s));
    c->w_bytes = total;
    c->encoded = true;
    if (n_bytes) *n_bytes = total;
    return KDTN_OK;
}

int kdtn_epoch_download_wire(kdtn_ctx* c, kdtn_wire* o) {
    if (!c || !o || !c->encoded) return KDTN_EINVAL;
    HIP_TRY(hipSetDevice(c->device));
    o->n_bytes = c->w_bytes;
    if (o->bytes && c->w_bytes > o->cap) return KDTN_ENOSPC;
    hipStream_t s = c->stream;
    if (o->bytes && c->w_bytes)
        HIP_TRY(hipMemcpyAsync(o->bytes, c->w_arena.p, c->w_bytes, hipMemcpyDeviceToHost, s));
    if (o->off) HIP_TRY(hipMemcpyAsync(o->off, c->w_off.p, ((size_t)3 * c->T + 1) * 8, hipMemcpyDeviceToHost, s));
    if (o->err && c->T) HIP_TRY(hipMemcpyAsync(o->err, c->w_err.p, (size_t)c->T * 4, hipMemcpyDeviceToHost, s));
    HIP_TRY(hipStreamSynchronize(s));
    return KDTN_OK;
}

}  // extern "C"

namespace {

// The RemotePod fan-out of the last run (k_reach, node compaction, stable grouping) into
// f_nodes / f_idx / f_base; cached until the next run.
int fanout_compute(kdtn_ctx* c) {
    if (c->fan_valid) return KDTN_OK;
    HIP_TRY(hipStreamSynchronize(c->stream));
    TRY(counts_fresh(c));
    hipStream_t s = c->stream;
    const uint32_t na = c->h_misc[3], D = c->D;
    const uint32_t nw = (D + 3) / 4;                          // destination-daemon flag bytes (words of 4)
    TRY(ensure(c->f_mark, (size_t)nw * 4 + 16));
    HIP_TRY(hipMemsetAsync(c->f_mark.p, 0, (size_t)nw * 4, s));
    const uint32_t nchunks = nblocks(na, FAN_CHUNK);
    const uint32_t nbd = nblocks(nw, SCAN_CHUNK);
    TRY(ensure(c->f_node_idx, (size_t)D * 4));
    TRY(ensure(c->f_nodes, (size_t)FAN_NODE_CAP * 4 + 16));
    TRY(ensure(c->f_part, (size_t)nbd * 8 + 16));
    TRY(ensure(c->f_idx, (size_t)na * 4 + 16));
    TRY(ensure(c->f_inv, (size_t)na * 4 + 16));
    uint32_t* misc = dp<uint32_t>(c->misc);
    uint32_t* n_nodes = misc + MISC_FAN_NODES;
    TRY(run_reach(c, dp<uint32_t>(c->f_mark), 0));
    const FanIn f{dp<uint32_t>(c->add_off), dp<uint4>(c->add_res), dp<uint2>(c->add_qdisc), c->T, na, 0u,
                  dp<uint32_t>(c->f_node)};            // (after run_reach: it sizes f_node)
    k_fan_nodes_count<<<nbd, BLOCK, 0, s>>>(dp<uint32_t>(c->f_mark), nw, dp<uint64_t>(c->f_part));
    k_scan_top<<<1, SCAN_TOP_BLOCK, 0, s>>>(dp<uint64_t>(c->f_part), nbd);
    k_fan_nodes_write<<<nbd, BLOCK, 0, s>>>(dp<uint32_t>(c->f_mark), nw, dp<uint64_t>(c->f_part),
                                           dp<uint32_t>(c->f_node_idx), dp<uint32_t>(c->f_nodes), n_nodes);
    timer_mark(c, "fanout_nodes");
    uint32_t nn = 0;
    HIP_TRY(hipMemcpyAsync(&nn, n_nodes, 4, hipMemcpyDeviceToHost, s));
    HIP_TRY(hipStreamSynchronize(s));
    if (nn > (uint32_t)FAN_NODE_CAP) {
        std::snprintf(g_last_error, sizeof(g_last_error), "fan-out over %u daemons (cap %d)", nn, FAN_NODE_CAP);
        return KDTN_EINVAL;
    }
    timer_mark(c, "fanout_host_sync");
    const uint32_t ncells = nn * nchunks;
    TRY(ensure(c->f_counts, (size_t)ncells * 4 + 16));
    TRY(ensure(c->f_base, ((size_t)ncells + 1) * 8 + 16));
    uint32_t nsend = 0;
    if (na && nn) {
        const size_t lds = (size_t)nn * 4;
        k_fan_count<<<nchunks, 64, lds, s>>>(f, dp<uint8_t>(c->f_send), dp<uint32_t>(c->f_node_idx), n_nodes,
                                           dp<uint32_t>(c->f_counts), nchunks);
        TRY(scan_u32(c, dp<uint32_t>(c->f_counts), ncells, dp<uint64_t>(c->f_base)));
        k_fan_scatter<<<nchunks, 64, lds, s>>>(f, dp<uint8_t>(c->f_send), dp<uint32_t>(c->f_node_idx), n_nodes,
                                             dp<uint64_t>(c->f_base), nchunks, dp<uint32_t>(c->f_idx),
                                             dp<uint32_t>(c->f_inv));
        HIP_TRY(hipGetLastError());
        uint64_t tot = 0;
        HIP_TRY(hipMemcpyAsync(&tot, dp<uint64_t>(c->f_base) + ncells, 8, hipMemcpyDeviceToHost, s));
        HIP_TRY(hipStreamSynchronize(s));
        nsend = (uint32_t)tot;
    }
    timer_mark(c, "fanout_group");
    c->fan_nn = nn;
    c->fan_nsend = nsend;
    c->fan_valid = true;
    return KDTN_OK;
}

bool fanout_stages_ok(const kdtn_ctx* c) {
    return (c->last_stages & (KDTN_STAGE_RESOLVE | KDTN_STAGE_QDISC)) == (KDTN_STAGE_RESOLVE | KDTN_STAGE_QDISC);
}

}  // namespace

extern "C" {

int kdtn_epoch_fanout(kdtn_ctx* c, kdtn_fanout* o) {
    if (!c || !o || !c->ran) return KDTN_EINVAL;
    if (!fanout_stages_ok(c)) return KDTN_EINVAL;
    HIP_TRY(hipSetDevice(c->device));
    TRY(counts_fresh(c));
    hipStream_t s = c->stream;
    c->n_ev = 0;
    (void)hipEventRecord(c->ev[0], s);
    c->fan_valid = false;                                    // recomputed per call (timed stage)
    TRY(fanout_compute(c));
    const uint32_t nn = c->fan_nn, nsend = c->fan_nsend, na = c->h_misc[3];
    const uint32_t nchunks = nblocks(na, FAN_CHUNK);
    o->n_nodes = nn;
    o->n_send = nsend;
    if (nn > o->node_cap || nsend > o->idx_cap) return KDTN_ENOSPC;
    if (o->node && nn) HIP_TRY(hipMemcpyAsync(o->node, c->f_nodes.p, (size_t)nn * 4, hipMemcpyDeviceToHost, s));
    if (o->idx && nsend) HIP_TRY(hipMemcpyAsync(o->idx, c->f_idx.p, (size_t)nsend * 4, hipMemcpyDeviceToHost, s));
    if (o->off) {
        // off[k] = base of (node k, chunk 0): strided 8-B reads of the scanned (node, chunk) matrix
        std::vector<uint64_t> b(nn ? nn : 1);
        if (nn && na)
            HIP_TRY(hipMemcpy2DAsync(b.data(), 8, dp<uint64_t>(c->f_base), (size_t)nchunks * 8, 8, nn,
                                     hipMemcpyDeviceToHost, s));
        HIP_TRY(hipStreamSynchronize(s));
        for (uint32_t k = 0; k < nn; ++k) o->off[k] = na ? (uint32_t)b[k] : 0u;
        o->off[nn] = nsend;
    }
    HIP_TRY(hipStreamSynchronize(s));
    return KDTN_OK;
}

int kdtn_epoch_remote_encode(kdtn_ctx* c, kdtn_remote_info* info) {
    if (!c || !c->ran || !fanout_stages_ok(c)) return KDTN_EINVAL;
    HIP_TRY(hipSetDevice(c->device));
    TRY(counts_fresh(c));
    hipStream_t s = c->stream;
    c->n_ev = 0;
    (void)hipEventRecord(c->ev[0], s);
    TRY(fanout_compute(c));                                  // f_idx (fan-out order) and f_send (reach)
    const uint32_t na = c->h_misc[3], nr = c->fan_nsend;
    // physical peers' local Updates: reached PHYSICAL adds whose MakeVeth passed, add-list order
    TRY(ensure(c->rp_flag, (size_t)na * 4 + 16));
    TRY(ensure(c->rp_pos, ((size_t)na + 1) * 8));
    TRY(ensure(c->rp_phys, (size_t)na * 4 + 16));
    if (na) k_remote_phys_flags<<<nblocks(na), BLOCK, 0, s>>>(dp<uint8_t>(c->f_send), dp<uint4>(c->add_res), na,
                                                              dp<uint32_t>(c->rp_flag));
    TRY(scan_u32(c, dp<uint32_t>(c->rp_flag), na, dp<uint64_t>(c->rp_pos)));
    if (na) k_remote_phys_scatter<<<nblocks(na), BLOCK, 0, s>>>(dp<uint32_t>(c->rp_flag), dp<uint64_t>(c->rp_pos), na,
                                                                dp<uint32_t>(c->rp_phys));
    uint64_t nphys = 0;
    HIP_TRY(hipMemcpyAsync(&nphys, dp<uint64_t>(c->rp_pos) + na, 8, hipMemcpyDeviceToHost, s));
    // UTF-8 validity of every dictionary string (proto.Marshal fails on invalid strings)
    TRY(str_tables(c));

    HIP_TRY(hipStreamSynchronize(s));
    timer_mark(c, "remote_select");
    const uint64_t n = (uint64_t)nr + nphys;
    if (n >= 0xFFFFFFFFull) return KDTN_EINVAL;
    RemoteIn r{};
    r.kd = str_tab_kd(c);
    r.pd = str_tab_pd(c);
    r.kd_offs = dp<uint32_t>(c->kd_offs);
    if (c->encoded) {                        // the run's wire encoding: its properties fields
        r.w_pinfo = dp<uint64_t>(c->w_pinfo);
        r.w_pos = dp<uint64_t>(c->w_size);
        r.w_arena = dp<uint8_t>(c->w_arena);
        r.w_err = dp<uint32_t>(c->w_err);
        r.w_nd = c->h_misc[1];
    }
    TRY(list_coarse(c));
    r.add_coarse = dp<uint32_t>(c->lc[1]);
    r.t_ns = dp<uint32_t>(c->t_ns);
    r.t_src = dp<uint32_t>(c->t_src);
    r.t_netns = dp<uint32_t>(c->t_netns);
    r.add_off = dp<uint32_t>(c->add_off);
    r.add_idx = dp<uint32_t>(c->add_idx);
    r.add_res = dp<uint4>(c->add_res);
    r.add_qdisc = dp<uint2>(c->add_qdisc);
    r.pods = dp<uint4>(c->pods);
    r.rem_idx = dp<uint32_t>(c->f_idx);
    r.phys_idx = dp<uint32_t>(c->rp_phys);
    r.send = dp<uint8_t>(c->f_send);
    r.phys_flag = dp<uint32_t>(c->rp_flag);
    r.phys_pos = dp<uint64_t>(c->rp_pos);
    r.rem_inv = dp<uint32_t>(c->f_inv);
    r.N = c->des.view;
    r.n_msgs = (uint32_t)n;
    r.n_remote = nr;
    r.T = c->T;
    r.n_add = na;
    TRY(ensure(c->rp_msz, (size_t)n * 4 + 16));
    TRY(ensure(c->rp_tsz, (size_t)n * 4 + 16));
    TRY(ensure(c->rp_moff, (n + 1) * 8));
    TRY(ensure(c->rp_toff, (n + 1) * 8));
    // sizes per add entry (coalesced columns), stored at the message indices
    if (n) k_remote_sizes<<<nblocks(na), BLOCK, 0, s>>>(r, dp<uint32_t>(c->rp_msz), dp<uint32_t>(c->rp_tsz));
    TRY(scan_u32(c, dp<uint32_t>(c->rp_msz), (uint32_t)n, dp<uint64_t>(c->rp_moff)));   // message offsets
    TRY(scan_u32(c, dp<uint32_t>(c->rp_tsz), (uint32_t)n, dp<uint64_t>(c->rp_toff)));   // tc argv offsets
    timer_mark(c, "remote_sizes");
    HIP_TRY(hipGetLastError());
    uint64_t tot[2] = {0, 0};
    HIP_TRY(hipMemcpyAsync(tot, dp<uint64_t>(c->rp_moff) + n, 8, hipMemcpyDeviceToHost, s));
    HIP_TRY(hipMemcpyAsync(tot + 1, dp<uint64_t>(c->rp_toff) + n, 8, hipMemcpyDeviceToHost, s));
    HIP_TRY(hipStreamSynchronize(s));
    TRY(ensure(c->rp_arena, (size_t)tot[0] + 16));
    TRY(ensure(c->rp_tc, (size_t)tot[1] + 16));
    timer_mark(c, "remote_host_sync");
    if (n) {
        k_remote_write<<<nblocks(na), BLOCK, 0, s>>>(r, dp<uint64_t>(c->rp_moff), dp<uint8_t>(c->rp_arena));
        timer_mark(c, "remote_write");
        if (nr) k_tc_remote_write<<<nblocks(na), BLOCK, 0, s>>>(r, dp<uint64_t>(c->rp_toff), dp<uint8_t>(c->rp_tc));
        timer_mark(c, "remote_tc_write");
    }
    HIP_TRY(hipGetLastError());
    HIP_TRY(hipStreamSynchronize(s));
    c->rp_n = (uint32_t)n;
    c->rp_nr = nr;
    c->rp_bytes = tot[0];
    c->rp_tc_bytes = tot[1];
    c->rp_done = true;
    if (info) {
        info->n_msgs = c->rp_n;
        info->n_remote = nr;
        info->n_bytes = tot[0];
        info->n_tc_bytes = tot[1];
    }
    return KDTN_OK;
}

int kdtn_epoch_download_remote(kdtn_ctx* c, kdtn_remote_pods* o) {
    if (!c || !o || !c->rp_done) return KDTN_EINVAL;
    HIP_TRY(hipSetDevice(c->device));
    if ((o->bytes && c->rp_bytes > o->cap) || (o->tc_bytes && c->rp_tc_bytes > o->tc_cap) ||
        ((o->off || o->entry || o->tc_off) && c->rp_n > o->msg_cap))
        return KDTN_ENOSPC;
    hipStream_t s = c->stream;
    const size_t n = c->rp_n, nr = c->rp_nr;
    if (o->bytes && c->rp_bytes) HIP_TRY(hipMemcpyAsync(o->bytes, c->rp_arena.p, c->rp_bytes, hipMemcpyDeviceToHost, s));
    if (o->tc_bytes && c->rp_tc_bytes)
        HIP_TRY(hipMemcpyAsync(o->tc_bytes, c->rp_tc.p, c->rp_tc_bytes, hipMemcpyDeviceToHost, s));
    if (o->off) HIP_TRY(hipMemcpyAsync(o->off, c->rp_moff.p, (n + 1) * 8, hipMemcpyDeviceToHost, s));
    if (o->tc_off) HIP_TRY(hipMemcpyAsync(o->tc_off, c->rp_toff.p, (n + 1) * 8, hipMemcpyDeviceToHost, s));
    if (o->entry) {
        if (nr) HIP_TRY(hipMemcpyAsync(o->entry, c->f_idx.p, nr * 4, hipMemcpyDeviceToHost, s));
        if (n > nr) HIP_TRY(hipMemcpyAsync(o->entry + nr, c->rp_phys.p, (n - nr) * 4, hipMemcpyDeviceToHost, s));
    }
    HIP_TRY(hipStreamSynchronize(s));
    return KDTN_OK;
}

int kdtn_epoch_tc(kdtn_ctx* c, uint64_t* n_bytes) {
    if (!c || !c->ran) return KDTN_EINVAL;
    if ((c->last_stages & (KDTN_STAGE_RESOLVE | KDTN_STAGE_QDISC)) != (KDTN_STAGE_RESOLVE | KDTN_STAGE_QDISC))
        return KDTN_EINVAL;
    HIP_TRY(hipSetDevice(c->device));
    HIP_TRY(hipStreamSynchronize(c->stream));
    TRY(counts_fresh(c));
    hipStream_t s = c->stream;
    const uint32_t nu = c->h_misc[2], na = c->h_misc[3];
    const uint64_t n = 2ull * na + nu;                    // command slots: 2 per add entry, 1 per update
    if (n >= 0xFFFFFFFFull) return KDTN_EINVAL;
    const uint32_t nb = nblocks(n + 1, SCAN_CHUNK);
    TRY(ensure(c->tc_size, (size_t)n * 4 + 16));
    TRY(ensure(c->tc_off, ((size_t)n + 1) * 8));
    TRY(ensure(c->tc_part, (size_t)nb * 8 + 16));
    c->n_ev = 0;
    (void)hipEventRecord(c->ev[0], s);
    TRY(run_reach(c, nullptr, 0));
    TRY(str_tables(c));                                   // the interface names' entries
    timer_mark(c, "tc_reach");
    TcIn w{c->des.view, dp<uint8_t>(c->f_send), dp<uint8_t>(c->f_reach_upd), dp<uint32_t>(c->add_idx),
           dp<uint32_t>(c->upd_idx), dp<uint4>(c->add_res),
           dp<uint4>(c->upd_res), dp<uint2>(c->add_qdisc), dp<uint2>(c->upd_qdisc), str_tab_kd(c), na, nu};
    if (n) k_tc_sizes<<<nblocks(n), BLOCK, 0, s>>>(w, dp<uint32_t>(c->tc_size));
    TRY(scan_u32(c, dp<uint32_t>(c->tc_size), (uint32_t)n, dp<uint64_t>(c->tc_off)));
    timer_mark(c, "tc_sizes");
    HIP_TRY(hipGetLastError());
    uint64_t total = 0;
    HIP_TRY(hipMemcpyAsync(&total, dp<uint64_t>(c->tc_off) + n, 8, hipMemcpyDeviceToHost, s));
    HIP_TRY(hipStreamSynchronize(s));
    TRY(ensure(c->tc_arena, (size_t)total + 16));
    timer_mark(c, "tc_host_sync");
    if (n) k_tc_write<<<nblocks(n), BLOCK, 0, s>>>(w, dp<uint64_t>(c->tc_off), dp<uint8_t>(c->tc_arena));
    timer_mark(c, "tc_write");
    HIP_TRY(hipGetLastError());
    HIP_TRY(hipStreamSynchronize(s));
    c->tc_bytes = total;
    c->tc_n = (uint32_t)n;
    c->tc_done = true;
    if (n_bytes) *n_bytes = total;
    return KDTN_OK;
}

int kdtn_epoch_download_tc(kdtn_ctx* c, kdtn_tc_argv* o) {
    if (!c || !o || !c->tc_done) return KDTN_EINVAL;
    HIP_TRY(hipSetDevice(c->device));
    o->n_bytes = c->tc_bytes;
    if (o->bytes && c->tc_bytes > o->cap) return KDTN_ENOSPC;
    if (o->bytes && c->tc_bytes)
        HIP_TRY(hipMemcpyAsync(o->bytes, c->tc_arena.p, c->tc_bytes, hipMemcpyDeviceToHost, c->stream));
    if (o->off) HIP_TRY(hipMemcpyAsync(o->off, c->tc_off.p, ((size_t)c->tc_n + 1) * 8, hipMemcpyDeviceToHost, c->stream));
    HIP_TRY(hipStreamSynchronize(c->stream));
    return KDTN_OK;
}

}  // extern "C"

// ======================================================================================
// CR ingest: TopologyList JSON → device-resident epoch tables (kdtn_ingest.hip)
// ======================================================================================
namespace {

template <typename T>
int d2h(kdtn_ctx* c, T* host, const void* dev, size_t count = 1) {
    HIP_TRY(hipMemcpyAsync(host, dev, sizeof(T) * count, hipMemcpyDeviceToHost, c->stream));
    return KDTN_OK;
}

// where a decode writes its tables (the context's own, or an incremental ingest's scratch)
struct JsTargets {
    DevBuf *ns, *name, *src, *netns, *flags, *roff, *noff;
    DevLinkStore *des, *real;
    DevBuf *kd_bytes, *kd_offs, *pd_bytes, *pd_offs;
};
struct JsCounts {
    uint32_t T, N, M, D, P;
    uint64_t kbytes, pbytes;
};

// small control block: [0] syntax error, [1] decode error (pos << 8 | code, ~0 = none),
// [2] heap bytes used, [3] status | seen_root << 32, [4] kd fill | pd fill << 32
constexpr size_t J_SMALL = 64;

int json_reject(kdtn_ctx* c, kdtn_ingest_info* info, unsigned long long word) {
    c->j_info.json_err = (int32_t)(word & 0xFF);
    c->j_info.err_offset = word >> 8;
    if (info) *info = c->j_info;
    c->j_done = false;
    c->uploaded = false;
    std::snprintf(g_last_error, sizeof(g_last_error), "TopologyList rejected: json error %d at byte %llu",
                  c->j_info.json_err, (unsigned long long)c->j_info.err_offset);
    return KDTN_EBADMSG;
}

// ids of one dictionary in first-occurrence order, its arena and offsets
int json_dict(kdtn_ctx* c, const JsDict& dt, const JsIntern& in, uint32_t ntok, DevBuf& slot_id, DevBuf& bytes,
              DevBuf& offs, uint32_t* n_out, uint64_t* bytes_out) {
    hipStream_t s = c->stream;
    const uint32_t nw = (ntok + 31) / 32, cap = dt.mask + 1;
    TRY(ensure(c->j_bits, (size_t)nw * 4));
    TRY(ensure(c->j_bcnt, (size_t)nw * 4));
    TRY(ensure(c->j_wrank, ((size_t)nw + 1) * 8));
    HIP_TRY(hipMemsetAsync(c->j_bits.p, 0, (size_t)nw * 4, s));
    k_js_rep_mark<<<nblocks(cap), BLOCK, 0, s>>>(dt, dp<uint32_t>(c->j_bits));
    k_js_popc<<<nblocks(nw), BLOCK, 0, s>>>(dp<uint32_t>(c->j_bits), nw, dp<uint32_t>(c->j_bcnt));
    TRY(scan_u32(c, dp<uint32_t>(c->j_bcnt), nw, dp<uint64_t>(c->j_wrank)));
    timer_mark(c, "js_intern");
    uint64_t uniq = 0;
    TRY(d2h(c, &uniq, dp<uint64_t>(c->j_wrank) + nw));
    HIP_TRY(hipStreamSynchronize(s));
    timer_mark(c, "js_sync");
    const uint32_t n = (uint32_t)uniq + 1;                    // + id 0 = ""
    TRY(ensure(slot_id, (size_t)cap * 4));
    TRY(ensure(c->j_len, (size_t)n * 4));
    TRY(ensure(c->j_off64, ((size_t)n + 1) * 8));
    TRY(ensure(c->j_sofid, (size_t)n * 4));
    HIP_TRY(hipMemsetAsync(c->j_len.p, 0, (size_t)n * 4, s));
    k_js_ids<<<nblocks(cap), BLOCK, 0, s>>>(dt, dp<uint32_t>(c->j_bits), dp<uint64_t>(c->j_wrank),
                                            dp<uint32_t>(slot_id), dp<uint32_t>(c->j_len), dp<uint32_t>(c->j_sofid));
    TRY(scan_u32(c, dp<uint32_t>(c->j_len), n, dp<uint64_t>(c->j_off64)));
    timer_mark(c, "js_intern");
    uint64_t total = 0;
    TRY(d2h(c, &total, dp<uint64_t>(c->j_off64) + n));
    HIP_TRY(hipStreamSynchronize(s));
    timer_mark(c, "js_sync");
    if (total > 0xFFFFFF00ull) {
        std::snprintf(g_last_error, sizeof(g_last_error), "dictionary arena of %llu bytes exceeds 4 GiB",
                      (unsigned long long)total);
        return KDTN_EINVAL;
    }
    TRY(ensure(bytes, (size_t)total + 64));
    TRY(ensure(offs, ((size_t)n + 1) * 4));
    HIP_TRY(hipMemsetAsync(offs.p, 0, 4, s));
    HIP_TRY(hipMemsetD32Async(reinterpret_cast<hipDeviceptr_t>(dp<uint32_t>(offs) + n), (int)(uint32_t)total, 1, s));
    if (n > 1)
        k_js_dict_copy<<<nblocks(n - 1), BLOCK, 0, s>>>(dt, in, dp<uint32_t>(c->j_sofid), n, dp<uint64_t>(c->j_off64),
                                                        dp<uint32_t>(offs), dp<uint8_t>(bytes));
    *n_out = n;
    *bytes_out = total;
    return KDTN_OK;
}

int link_store_alloc(kdtn_ctx* c, DevLinkStore& st, uint32_t n) {
    const size_t tiles = ((size_t)std::max<uint32_t>(n, 1) + TILE_RECS - 1) / TILE_RECS;
    TRY(ensure(st.buf, tiles * TILE_WORDS * 4));
    st.view.base = dp<uint32_t>(st.buf);
    st.view.n = n;
    st.n = n;
    return KDTN_OK;
}

}  // namespace

extern "C" {

int kdtn_json_upload(kdtn_ctx* c, const uint8_t* doc, uint64_t n) {
    if (!c || (n && !doc)) return KDTN_EINVAL;
    if (n >= 0xFFFFFF00ull) {
        std::snprintf(g_last_error, sizeof(g_last_error), "document of %llu bytes: the GPU ingest takes < 4 GiB",
                      (unsigned long long)n);
        return KDTN_EINVAL;
    }
    HIP_TRY(hipSetDevice(c->device));
    const uint32_t nb = (uint32_t)((n + 63) / 64);
    const size_t padded = (size_t)nb * 64 + 128;             // whitespace tail: blocks and look-ahead
    TRY(ensure(c->j_doc, padded));
    if (n) HIP_TRY(hipMemcpyAsync(c->j_doc.p, doc, n, hipMemcpyHostToDevice, c->stream));
    HIP_TRY(hipMemsetAsync(dp<uint8_t>(c->j_doc) + n, ' ', padded - n, c->stream));
    HIP_TRY(hipStreamSynchronize(c->stream));
    c->j_n = n;
    c->j_nb = nb;
    c->j_loaded = true;
    c->j_done = false;
    return KDTN_OK;
}

// The decode of the uploaded document into `tg` (the context's own tables for a full ingest,
// scratch tables for an incremental one): topology columns, both link stores, first-occurrence
// dictionaries. Counts into `o`. A rejected document returns KDTN_EBADMSG (json_reject).
static int json_decode(kdtn_ctx* c, const JsTargets& tg, JsCounts* o, kdtn_ingest_info* info) {
    hipStream_t s = c->stream;
    c->j_info = kdtn_ingest_info{};
    c->n_ev = 0;
    (void)hipEventRecord(c->ev[0], s);
    const uint32_t nb = c->j_nb;
    if (nb == 0) return json_reject(c, info, (0ull << 8) | KDTN_JSON_SYNTAX);   // empty document

    TRY(ensure(c->j_small, J_SMALL));
    unsigned long long* small = dp<unsigned long long>(c->j_small);
    HIP_TRY(hipMemsetAsync(small, 0xFF, 16, s));
    HIP_TRY(hipMemsetAsync(small + 2, 0, J_SMALL - 16, s));
    // one word past the end: any_in reads the word after a string's first (its bits are masked)
    for (DevBuf* b : {&c->j_q, &c->j_bs, &c->j_hb, &c->j_esc, &c->j_tok, &c->j_open, &c->j_close}) TRY(ensure(*b, ((size_t)nb + 1) * 8));
    // per-workgroup counts (quotes; tokens, depth, opens, colons, scalars) and their offsets
    const uint32_t nwg = nblocks(nb);
    TRY(ensure(c->j_qcnt, (size_t)nwg * 4));
    TRY(ensure(c->j_qoff, ((size_t)nwg + 1) * 8));
    TRY(ensure(c->j_gcnt, (size_t)5 * nwg * 4));
    TRY(ensure(c->j_goff, (size_t)5 * (nwg + 1) * 8));
    JsDoc j{dp<uint8_t>(c->j_doc), (uint32_t)c->j_n, nb, dp<uint64_t>(c->j_q), dp<uint64_t>(c->j_bs),
            dp<uint64_t>(c->j_hb), dp<uint64_t>(c->j_esc), 0u};
#if KDTN_PROFILING
    j.variant = (uint32_t)std::strtoul(std::getenv("KDTN_JS_VARIANT") ? std::getenv("KDTN_JS_VARIANT") : "0", nullptr, 0);
#endif
    JsMasks m{dp<uint64_t>(c->j_tok), dp<uint64_t>(c->j_open), dp<uint64_t>(c->j_close), dp<uint32_t>(c->j_gcnt)};
    const uint64_t* goff = dp<uint64_t>(c->j_goff);
    auto gtotal = [&](int f) { return goff + (size_t)f * (nwg + 1) + nwg; };   // f: 0 tokens, 2 opens, 3 colons, 4 scalars

    // 1. block masks, string state, token counts, depth
    k_js_quotes<<<nblocks(nb), BLOCK, 0, s>>>(j, dp<uint64_t>(c->j_q), dp<uint64_t>(c->j_bs), dp<uint64_t>(c->j_hb),
                                              dp<uint64_t>(c->j_esc),
                                             dp<uint32_t>(c->j_qcnt));
    TRY(scan_u32(c, dp<uint32_t>(c->j_qcnt), nwg, dp<uint64_t>(c->j_qoff)));
    k_js_classify<<<nwg, BLOCK, 0, s>>>(j, dp<uint64_t>(c->j_qoff), m, nwg, small);
    for (int f = 0; f < 5; ++f)
        TRY(scan_u32(c, dp<uint32_t>(c->j_gcnt) + (size_t)f * nwg, nwg, dp<uint64_t>(c->j_goff) + (size_t)f * (nwg + 1)));
    timer_mark(c, "js_blocks");
    uint64_t quotes = 0, ntok64 = 0, nopen64 = 0;
    TRY(d2h(c, &nopen64, gtotal(2)));
    uint64_t nval64 = 0;
    TRY(d2h(c, &nval64, gtotal(3)));
    uint64_t nscal64 = 0;
    TRY(d2h(c, &nscal64, gtotal(4)));
    unsigned long long serr = 0;
    TRY(d2h(c, &quotes, dp<uint64_t>(c->j_qoff) + nwg));
    TRY(d2h(c, &ntok64, gtotal(0)));
    TRY(d2h(c, &serr, small));
    HIP_TRY(hipStreamSynchronize(s));
    timer_mark(c, "js_sync");                       // host round trips are timed apart
    HIP_TRY(hipGetLastError());
    if (quotes & 1) serr = std::min<unsigned long long>(serr, (c->j_n << 8) | KDTN_JSON_SYNTAX);   // unterminated
    if (ntok64 == 0) serr = std::min<unsigned long long>(serr, KDTN_JSON_SYNTAX);
    if (serr != ~0ull) return json_reject(c, info, serr);
    const uint32_t ntok = (uint32_t)ntok64;
    c->j_info.n_tokens = ntok64;

    // 2. token stream, parents, checkValid
    TRY(ensure(c->j_toks, (size_t)ntok * 8));
    TRY(ensure(c->j_par, (size_t)ntok * 4));
    TRY(ensure(c->j_role, (size_t)ntok));
    TRY(ensure(c->j_ecls, ((size_t)ntok + JS_TILE - 1) / JS_TILE * JS_TILE));   // whole tiles (uint4 reads)
    TRY(ensure(c->j_ord, (size_t)ntok * 4));
    const uint32_t nopen = (uint32_t)nopen64;
    TRY(ensure(c->j_olist, (size_t)nopen * 4));
    TRY(ensure(c->j_odep, (size_t)nopen));
    const uint32_t nval = (uint32_t)nval64;
    TRY(ensure(c->j_vlist, (size_t)nval * 4));
    const uint32_t nscal = (uint32_t)nscal64;
    TRY(ensure(c->j_slist, (size_t)nscal * 4 + 4));
    const JsToks tk{dp<uint32_t>(c->j_toks), dp<uint32_t>(c->j_toks) + ntok};   // offsets, then meta words
    uint32_t* par = dp<uint32_t>(c->j_par);
    k_js_tokens<<<nwg, BLOCK, 0, s>>>(j, m, goff, nwg, tk, dp<uint32_t>(c->j_olist), dp<uint8_t>(c->j_odep),
                                             dp<uint32_t>(c->j_vlist), dp<uint32_t>(c->j_slist), small);
    timer_mark(c, "js_tokens");
    const uint32_t ntiles = (ntok + JS_TILE - 1) / JS_TILE, ng = (ntiles + BLOCK - 1) / BLOCK;
    TRY(ensure(c->j_tagg, (size_t)ntiles * JS_PD * 4));
    TRY(ensure(c->j_gagg, (size_t)ng * JS_PD * 4));
    k_js_par_agg<<<ntiles, BLOCK, 0, s>>>(tk.meta, ntok, dp<uint32_t>(c->j_tagg));
    k_js_par_group<<<ng, BLOCK, 0, s>>>(dp<uint32_t>(c->j_tagg), ntiles, dp<uint32_t>(c->j_gagg));
    k_js_par_top<<<1, BLOCK, 0, s>>>(dp<uint32_t>(c->j_gagg), ng);
    k_js_par_tiles<<<ng, BLOCK, 0, s>>>(dp<uint32_t>(c->j_tagg), ntiles, dp<uint32_t>(c->j_gagg));
    uint32_t* deep = reinterpret_cast<uint32_t*>(small + 4);   // zeroed with the small words above
    k_js_par_apply<<<ntiles, BLOCK, 0, s>>>(tk.meta, ntok, dp<uint32_t>(c->j_tagg), par, deep);
    k_js_deep<<<std::min<uint32_t>(nblocks(ntok), 2048), BLOCK, 0, s>>>(tk.meta, ntok, par, deep);
    timer_mark(c, "js_parents");
    k_js_validate<<<nblocks(ntok), BLOCK, 0, s>>>(j, tk, ntok, par, dp<uint8_t>(c->j_ecls), small);
    k_js_tail<<<1, 64, 0, s>>>(j, tk, ntok, par, small);
    if (nscal) k_js_scalars<<<nblocks(nscal), BLOCK, 0, s>>>(j, tk.pos, dp<uint32_t>(c->j_slist), nscal, small);
    timer_mark(c, "js_validate");
    TRY(d2h(c, &serr, small));
    HIP_TRY(hipStreamSynchronize(s));
    timer_mark(c, "js_sync");
    HIP_TRY(hipGetLastError());
    if (serr != ~0ull) return json_reject(c, info, serr);

    // 3. schema roles, items / links ordinals
    uint8_t* role = dp<uint8_t>(c->j_role);
    uint32_t* ord = dp<uint32_t>(c->j_ord);
    HIP_TRY(hipMemsetAsync(role, 0, ntok, s));                  // R_NONE below the schema levels
    for (uint32_t level : {0u, 1u, 3u, 4u})            // levels 2 and 5: k_js_elems_count
        if (nopen) k_js_roles<<<nblocks(nopen), BLOCK, 0, s>>>(j, tk, dp<uint32_t>(c->j_olist), nopen, par, role,
                                                    dp<uint8_t>(c->j_odep), level);
    TRY(ensure(c->j_cnt3, (size_t)3 * ntiles * 4));
    TRY(ensure(c->j_coff3, (size_t)3 * (ntiles + 1) * 8));
    k_js_elems_count<<<ntiles, BLOCK, 0, s>>>(j, tk, ntok, par, role, dp<uint32_t>(c->j_cnt3),
                                              dp<uint8_t>(c->j_ecls), small + 1);
    if (nopen)                                          // properties objects, under the links elements
        k_js_roles<<<nblocks(nopen), BLOCK, 0, s>>>(j, tk, dp<uint32_t>(c->j_olist), nopen, par, role,
                                                    dp<uint8_t>(c->j_odep), 6u);
    for (int q = 0; q < 3; ++q)
        TRY(scan_u32(c, dp<uint32_t>(c->j_cnt3) + (size_t)q * ntiles, ntiles,
                     dp<uint64_t>(c->j_coff3) + (size_t)q * (ntiles + 1)));
    timer_mark(c, "js_elements");
    uint64_t tot[3];
    for (int q = 0; q < 3; ++q) TRY(d2h(c, tot + q, dp<uint64_t>(c->j_coff3) + (size_t)q * (ntiles + 1) + ntiles));
    unsigned long long derr = 0;
    TRY(d2h(c, &derr, small + 1));
    HIP_TRY(hipStreamSynchronize(s));
    timer_mark(c, "js_sync");
    HIP_TRY(hipGetLastError());
    if (derr != ~0ull) return json_reject(c, info, derr);
    const uint32_t T = (uint32_t)tot[0], N = (uint32_t)tot[1], M = (uint32_t)tot[2];

    // 4. output tables
    for (DevBuf* b : {tg.ns, tg.name, tg.src, tg.netns, &c->j_tflags}) TRY(ensure(*b, (size_t)T * 4));
    TRY(ensure(*tg.flags, (size_t)T));
    TRY(ensure(*tg.roff, ((size_t)T + 1) * 4));
    TRY(ensure(*tg.noff, ((size_t)T + 1) * 4));
    TRY(link_store_alloc(c, *tg.des, N));
    TRY(link_store_alloc(c, *tg.real, M));
    const uint64_t owners = 1 + 9ull * T + 22ull * ((uint64_t)N + M);
    if (owners >= JS_NONE) {
        std::snprintf(g_last_error, sizeof(g_last_error), "ingest: too many records for one document");
        return KDTN_EINVAL;
    }
    TRY(ensure(c->j_owner, (size_t)owners * 4));
    TRY(ensure(c->j_vown, (size_t)nval * 4));
    JsTopoOut to{dp<uint32_t>(*tg.ns), dp<uint32_t>(*tg.name), dp<uint32_t>(*tg.src), dp<uint32_t>(*tg.netns),
                 dp<uint32_t>(c->j_tflags), dp<uint32_t>(*tg.roff), dp<uint32_t>(*tg.noff)};
    k_js_elems_write<<<ntiles, BLOCK, 0, s>>>(dp<uint8_t>(c->j_ecls), ntok, dp<uint64_t>(c->j_coff3), ntiles, ord, to);
    HIP_TRY(hipMemsetD32Async(reinterpret_cast<hipDeviceptr_t>(to.real_off + T), (int)M, 1, s));
    HIP_TRY(hipMemsetD32Async(reinterpret_cast<hipDeviceptr_t>(to.des_off + T), (int)N, 1, s));
    // the values land in row-major staging (one record's 88 B written by the wave that decodes
    // it), whole tiles per side so the finalize pass reads full tiles; it writes the AoSoA tiles
    const uint64_t des_tiles = ((uint64_t)N + TILE_RECS - 1) / TILE_RECS, real_tiles = ((uint64_t)M + TILE_RECS - 1) / TILE_RECS;
    const size_t rows_bytes = (size_t)(des_tiles + real_tiles) * TILE_WORDS * 4;
    TRY(ensure(c->j_rows, std::max<size_t>(rows_bytes, 16)));
    JsStore des{dp<uint32_t>(c->j_rows)};
    JsStore real{dp<uint32_t>(c->j_rows) + (size_t)des_tiles * TILE_WORDS};

    // 5. schema values + interning; a table or heap that fills up is grown and the pass rerun
    // A table that fills up (or whose probe runs grow past JS_MAX_PROBE) is grown 4x and the
    // pass rerun. (Sized for fewer distinct strings — half a key string per record — the config-2
    // document, 12M distinct key strings, overflowed its first table after 217 ms of ever longer
    // probe runs; the decode time does not depend on the table's footprint at these sizes.)
    uint32_t kcap = std::max(c->j_kcap, next_pow2(std::max<uint64_t>(1024, 2ull * ((uint64_t)N + M) + 4ull * T)));
    uint32_t pcap = std::max(c->j_pcap, next_pow2(std::max<uint64_t>(1024, ((uint64_t)N + M) / 2 + 64)));
    uint64_t hcap = std::max<uint64_t>(1 << 20, c->j_n / 16);
    JsIntern in{};
    for (int attempt = 0;; ++attempt) {
        TRY(ensure(c->j_kslots, (size_t)kcap * sizeof(JsSlot)));
        TRY(ensure(c->j_krep, (size_t)kcap * 4));
        TRY(ensure(c->j_pslots, (size_t)pcap * sizeof(JsSlot)));
        TRY(ensure(c->j_prep, (size_t)pcap * 4));
        TRY(ensure(c->j_heap, (size_t)hcap + 64));
        TRY(ensure(c->j_kkeys, (size_t)kcap * 8));
        TRY(ensure(c->j_pkeys, (size_t)pcap * 8));
        HIP_TRY(hipMemsetAsync(c->j_kslots.p, 0, (size_t)kcap * sizeof(JsSlot), s));
        HIP_TRY(hipMemsetAsync(c->j_kkeys.p, 0, (size_t)kcap * 8, s));
        HIP_TRY(hipMemsetAsync(c->j_pkeys.p, 0, (size_t)pcap * 8, s));
        HIP_TRY(hipMemsetAsync(c->j_krep.p, 0xFF, (size_t)kcap * 4, s));
        HIP_TRY(hipMemsetAsync(c->j_pslots.p, 0, (size_t)pcap * sizeof(JsSlot), s));
        HIP_TRY(hipMemsetAsync(c->j_prep.p, 0xFF, (size_t)pcap * 4, s));
        HIP_TRY(hipMemsetAsync(small + 2, 0, J_SMALL - 16, s));
        HIP_TRY(hipMemsetAsync(small + 1, 0xFF, 8, s));
        for (DevBuf* b : {tg.ns, tg.name, tg.src, tg.netns})
            HIP_TRY(hipMemsetAsync(b->p, 0, (size_t)T * 4, s));
        HIP_TRY(hipMemsetD32Async(reinterpret_cast<hipDeviceptr_t>(to.flags), (int)(KDTN_TOPO_SPEC_NIL | KDTN_TOPO_STATUS_NIL),
                                  T, s));
        if (rows_bytes) HIP_TRY(hipMemsetAsync(c->j_rows.p, 0, rows_bytes, s));   // absent fields: id 0, uid 0
        in.doc = j.doc;
        in.heap = dp<uint8_t>(c->j_heap);
        in.heap_used = small + 2;
        in.heap_cap = hcap;
        in.status = reinterpret_cast<uint32_t*>(small + 3);
        in.owner = dp<uint32_t>(c->j_owner);
        in.vown = dp<uint32_t>(c->j_vown);
        in.own_des = 1 + 9 * T;
        in.own_real = in.own_des + 22 * N;
#if KDTN_PROFILING
        in.variant = (uint32_t)std::strtoul(std::getenv("KDTN_JS_VARIANT") ? std::getenv("KDTN_JS_VARIANT") : "0",
                                            nullptr, 0);
#else
        in.variant = 0;
#endif
        in.kd = JsDict{dp<JsSlot>(c->j_kslots), dp<unsigned long long>(c->j_kkeys), dp<uint32_t>(c->j_krep), kcap - 1};
        in.pd = JsDict{dp<JsSlot>(c->j_pslots), dp<unsigned long long>(c->j_pkeys), dp<uint32_t>(c->j_prep), pcap - 1};
        if (nval)
            k_js_values<<<nblocks(nval), BLOCK, 0, s>>>(j, tk, dp<uint32_t>(c->j_vlist), nval, par, role, ord, to,
                                                        des, real, in, small + 1);
        if (nval && !(KDTN_PROFILING && (in.variant & JSV_NO_SEEN))) {
            uint32_t* any_dup = reinterpret_cast<uint32_t*>(small + 5);   // zeroed with the small words
            k_js_dups<<<nblocks(nval), BLOCK, 0, s>>>(dp<uint32_t>(c->j_vlist), nval, dp<uint32_t>(c->j_vown),
                                                      dp<uint32_t>(c->j_owner), any_dup);
            k_js_dups_report<<<std::min<uint32_t>(nblocks(nval), 2048), BLOCK, 0, s>>>(
                tk.pos, dp<uint32_t>(c->j_vlist), nval, dp<uint32_t>(c->j_vown), dp<uint32_t>(c->j_owner), any_dup,
                small + 1);
        }
        timer_mark(c, "js_values");
        unsigned long long ctl[3];
        TRY(d2h(c, ctl, small + 1, 3));
        HIP_TRY(hipStreamSynchronize(s));
        timer_mark(c, "js_sync");
        HIP_TRY(hipGetLastError());
        const uint32_t status = (uint32_t)ctl[2];
        if (status & JS_ST_LONG) {
            std::snprintf(g_last_error, sizeof(g_last_error), "a schema string is longer than 16 MiB");
            return KDTN_EINVAL;
        }
        if (status & JS_ST_OVERFLOW) {                  // a table filled up or the heap ran out
            if (attempt >= 6) return KDTN_ENOMEM;
            if (ctl[1] > hcap) hcap = std::max<uint64_t>(hcap * 4, ctl[1] + (1 << 20));
            else { kcap = std::min<uint64_t>((uint64_t)kcap * 4, 1u << 31); pcap = std::min<uint64_t>((uint64_t)pcap * 4, 1u << 31); }
            continue;
        }
        if (ctl[0] != ~0ull) return json_reject(c, info, ctl[0]);
        break;
    }

    // 6. ids in first-occurrence order, dictionaries, id columns
    uint64_t kbytes = 0, pbytes = 0;
    uint32_t D = 0, P = 0;
    TRY(json_dict(c, in.kd, in, ntok, c->j_kslot_id, *tg.kd_bytes, *tg.kd_offs, &D, &kbytes));
    TRY(json_dict(c, in.pd, in, ntok, c->j_pslot_id, *tg.pd_bytes, *tg.pd_offs, &P, &pbytes));
    // keep the intern tables at most half full for the next document of this shape
    c->j_kcap = std::max(kcap, next_pow2(2ull * D));
    c->j_pcap = std::max(pcap, next_pow2(2ull * P));
    if (N) k_js_finalize_links<<<(uint32_t)des_tiles, BLOCK, 0, s>>>(des.base, dp<uint32_t>(tg.des->buf),
                                                                       dp<uint32_t>(c->j_kslot_id), dp<uint32_t>(c->j_pslot_id));
    if (M) k_js_finalize_links<<<(uint32_t)real_tiles, BLOCK, 0, s>>>(real.base, dp<uint32_t>(tg.real->buf),
                                                                        dp<uint32_t>(c->j_kslot_id), dp<uint32_t>(c->j_pslot_id));
    if (T) k_js_finalize_topos<<<nblocks(T), BLOCK, 0, s>>>(to, T, dp<uint32_t>(c->j_kslot_id), dp<uint8_t>(*tg.flags));
    timer_mark(c, "js_intern");
    HIP_TRY(hipGetLastError());
    *o = JsCounts{T, N, M, D, P, kbytes, pbytes};
    return KDTN_OK;
}

static int json_ingest_full(kdtn_ctx* c, const kdtn_vni_table* vnis, kdtn_ingest_info* info) {
    if (!c || !c->j_loaded) return KDTN_EINVAL;
    HIP_TRY(hipSetDevice(c->device));
    c->sh_T = 0;
    g_last_error[0] = 0;
    hipStream_t s = c->stream;
    c->uploaded = false;
    c->ran = false;
    c->kd_valid = c->pd_valid = c->kd_from = c->pd_from = 0;   // the document's dictionaries are new
    c->si_k = c->si_p = 0;
    c->ix_k.n = c->ix_k.mask = c->ix_p.n = c->ix_p.mask = 0;     // (their string indexes too)
    const JsTargets tg{&c->t_ns, &c->t_name, &c->t_src, &c->t_netns, &c->t_flags, &c->t_roff, &c->t_noff,
                       &c->des, &c->real, &c->kd_bytes, &c->kd_offs, &c->pd_bytes, &c->pd_offs};
    JsCounts k{};
    TRY(json_decode(c, tg, &k, info));
    const uint32_t T = k.T, N = k.N, M = k.M;
    const uint64_t kbytes = k.kbytes, pbytes = k.pbytes;
    c->T = T;
    c->D = k.D;
    c->P = k.P;

    // 7. the epoch inputs are in place: finish what kdtn_epoch_upload would set up
    TRY(prepare_dicts(c));
    const kdtn_vni_table none{0, nullptr, nullptr, nullptr};
    const kdtn_vni_table& vn = vnis ? *vnis : none;
    TRY(check_vnis(c, vn, c->D, 0u));             // the engine's own dictionary: no kept prefix
    TRY(prepare_epoch(c, vn, T, M, N));
    HIP_TRY(hipStreamSynchronize(s));
    c->j_info.n_topos = T;
    c->j_info.n_desired = N;
    c->j_info.n_realised = M;
    c->j_info.n_kdict = c->D;
    c->j_info.n_pdict = c->P;
    c->j_info.kdict_bytes = kbytes;
    c->j_info.pdict_bytes = pbytes;
    c->kd_arena = kbytes;
    c->pd_arena = pbytes;
    if (info) *info = c->j_info;
    c->j_done = true;
    c->uploaded = true;
    c->pods_ready = false;
    c->pods_delta = false;
    return KDTN_OK;
}

int kdtn_json_ingest(kdtn_ctx* c, const kdtn_vni_table* vnis, kdtn_ingest_info* info) {
    if (c) end_shard_ingest(c);
    if (c && c->nranks > 1) {
        std::snprintf(g_last_error, sizeof(g_last_error),
                      "kdtn_json_ingest: single-shard contexts (kdtn_json_ingest_shard for a rank of several)");
        return KDTN_EINVAL;
    }
    return json_ingest_full(c, vnis, info);
}

// The whole document decoded as for one GPU, then the epoch cut down to this shard's
// Topologies on the GPU: the full table fills the pod-status rows of every Topology (pod
// index = document index), the shard's topology rows and records are compacted into fresh
// tables that are swapped in, and the context is left as a rank whose pod table is in place.
int kdtn_json_ingest_shard(kdtn_ctx* c, const kdtn_vni_table* vnis, uint32_t nshards, uint32_t shard,
                           kdtn_ingest_info* info) {
    if (!c || nshards < 1 || shard >= nshards || nshards > 0x7FFFFFFFu) return KDTN_EINVAL;
    if (c->comm) {
        std::snprintf(g_last_error, sizeof(g_last_error),
                      "kdtn_json_ingest_shard: the context has an RCCL communicator (no exchange is needed)");
        return KDTN_EINVAL;
    }
    end_shard_ingest(c);
    const int saved_nranks = c->nranks, saved_rank = c->rank;
    c->nranks = 1;
    c->rank = 0;
    const int rc = json_ingest_full(c, vnis, info);
    if (rc != KDTN_OK || nshards == 1) {
        c->nranks = saved_nranks;
        c->rank = saved_rank;
        return rc;
    }
    HIP_TRY(hipSetDevice(c->device));
    hipStream_t s = c->stream;
    const uint32_t Tf = c->T, Mf = c->real.n, Nf = c->des.n;
    const DevTopos full = topo_view(c);
    // 1. selection and the shard's offsets
    for (DevBuf* b : {&c->sh_keep, &c->sh_kreal, &c->sh_kdes}) TRY(ensure(*b, ((size_t)Tf + 1) * 4));
    for (DevBuf* b : {&c->sh_tidx, &c->sh_roff64, &c->sh_noff64}) TRY(ensure(*b, ((size_t)Tf + 1) * 8));
    if (Tf)
        k_shard_mark<<<nblocks(Tf), BLOCK, 0, s>>>(full, dp<uint8_t>(c->kd_bytes), dp<uint32_t>(c->kd_offs), nshards,
                                                   shard, dp<uint32_t>(c->sh_keep), dp<uint32_t>(c->sh_kreal),
                                                   dp<uint32_t>(c->sh_kdes));
    TRY(scan_u32(c, dp<uint32_t>(c->sh_keep), Tf, dp<uint64_t>(c->sh_tidx)));
    TRY(scan_u32(c, dp<uint32_t>(c->sh_kreal), Tf, dp<uint64_t>(c->sh_roff64)));
    TRY(scan_u32(c, dp<uint32_t>(c->sh_kdes), Tf, dp<uint64_t>(c->sh_noff64)));
    uint64_t cnt[3] = {0, 0, 0};
    TRY(d2h(c, cnt, dp<uint64_t>(c->sh_tidx) + Tf));
    TRY(d2h(c, cnt + 1, dp<uint64_t>(c->sh_roff64) + Tf));
    TRY(d2h(c, cnt + 2, dp<uint64_t>(c->sh_noff64) + Tf));
    HIP_TRY(hipStreamSynchronize(s));
    HIP_TRY(hipGetLastError());
    const uint32_t Ts = (uint32_t)cnt[0], Ms = (uint32_t)cnt[1], Ns = (uint32_t)cnt[2];
    // 2. the shard's tables
    for (DevBuf* b : {&c->sh_ns, &c->sh_name, &c->sh_src, &c->sh_netns, &c->sh_doc}) TRY(ensure(*b, ((size_t)Ts + 1) * 4));
    TRY(ensure(c->sh_flags, (size_t)Ts + 1));
    TRY(ensure(c->sh_roff, ((size_t)Ts + 1) * 4));
    TRY(ensure(c->sh_noff, ((size_t)Ts + 1) * 4));
    TRY(link_store_alloc(c, c->sh_real, Ms));
    TRY(link_store_alloc(c, c->sh_des, Ns));
    HIP_TRY(hipMemsetAsync(c->sh_real.buf.p, 0, c->sh_real.buf.cap, s));   // tile padding as an upload leaves it
    HIP_TRY(hipMemsetAsync(c->sh_des.buf.p, 0, c->sh_des.buf.cap, s));
    DevTopos out{dp<uint32_t>(c->sh_ns), dp<uint32_t>(c->sh_name), dp<uint32_t>(c->sh_src), dp<uint32_t>(c->sh_netns),
                 dp<uint8_t>(c->sh_flags), dp<uint32_t>(c->sh_roff), dp<uint32_t>(c->sh_noff), Ts};
    k_shard_topos<<<nblocks((uint64_t)Tf + 1), BLOCK, 0, s>>>(full, dp<uint32_t>(c->sh_keep), dp<uint64_t>(c->sh_tidx),
                                                              dp<uint64_t>(c->sh_roff64), dp<uint64_t>(c->sh_noff64), out,
                                                              dp<uint32_t>(c->sh_doc));
    if (Mf)
        k_shard_links<<<nblocks(Mf), BLOCK, 0, s>>>(c->real.view, full.real_off, Tf, dp<uint32_t>(c->sh_keep),
                                                    dp<uint64_t>(c->sh_roff64), dp<uint32_t>(c->sh_real.buf));
    if (Nf)
        k_shard_links<<<nblocks(Nf), BLOCK, 0, s>>>(c->des.view, full.des_off, Tf, dp<uint32_t>(c->sh_keep),
                                                    dp<uint64_t>(c->sh_noff64), dp<uint32_t>(c->sh_des.buf));
    HIP_TRY(hipGetLastError());
    // 3. a rank of nshards with every Topology's pod-status row: pod index = document index
    const uint32_t slice = (Tf + nshards - 1) / nshards;
    c->sh_active = true;
    c->sh_saved_nranks = saved_nranks;
    c->sh_saved_rank = saved_rank;
    c->nranks = (int)nshards;
    c->pods_rank_major = false;                         // pod index = document index
    c->rank = (int)shard;
    c->T = Ts;
    const kdtn_vni_table none{0, nullptr, nullptr, nullptr};
    TRY(prepare_epoch(c, vnis ? *vnis : none, slice, Ms, Ns));
    if (c->pod_total)
        k_pods_fill<<<nblocks(c->pod_total), BLOCK, 0, s>>>(full, c->pod_total, 0u, dp<uint4>(c->pods));
    HIP_TRY(hipGetLastError());
    HIP_TRY(hipStreamSynchronize(s));                // the full tables are read until here
    std::swap(c->t_ns, c->sh_ns);
    std::swap(c->t_name, c->sh_name);
    std::swap(c->t_src, c->sh_src);
    std::swap(c->t_netns, c->sh_netns);
    std::swap(c->t_flags, c->sh_flags);
    std::swap(c->t_roff, c->sh_roff);
    std::swap(c->t_noff, c->sh_noff);
    std::swap(c->real, c->sh_real);
    std::swap(c->des, c->sh_des);
    c->sh_T = Ts;
    c->pods_imported = true;
    c->j_info.n_topos = Ts;
    c->j_info.n_desired = Ns;
    c->j_info.n_realised = Ms;
    if (info) *info = c->j_info;
    return KDTN_OK;
}

int kdtn_ingest_shard_topos(kdtn_ctx* c, uint32_t* doc_index) {
    if (!c || !c->j_done || (c->sh_T && !doc_index)) return KDTN_EINVAL;
    HIP_TRY(hipSetDevice(c->device));
    if (c->nranks == 1) {                            // unsharded: the identity
        for (uint32_t t = 0; t < c->T; ++t) doc_index[t] = t;
        return KDTN_OK;
    }
    if (c->sh_T)
        HIP_TRY(hipMemcpyAsync(doc_index, c->sh_doc.p, (size_t)c->sh_T * 4, hipMemcpyDeviceToHost, c->stream));
    HIP_TRY(hipStreamSynchronize(c->stream));
    return KDTN_OK;
}

int kdtn_ingest_download(kdtn_ctx* c, kdtn_ingest_tables* o) {
    if (!c || !o || !(c->j_done || c->tables_cur)) return KDTN_EINVAL;
    HIP_TRY(hipSetDevice(c->device));
    hipStream_t s = c->stream;
    const kdtn_ingest_info& I = c->j_info;
    auto get = [&](void* dst, const DevBuf& b, size_t bytes) -> int {
        if (dst && bytes) HIP_TRY(hipMemcpyAsync(dst, b.p, bytes, hipMemcpyDeviceToHost, s));
        return KDTN_OK;
    };
    TRY(get(o->kd_bytes, c->kd_bytes, I.kdict_bytes));
    TRY(get(o->kd_offs, c->kd_offs, ((size_t)I.n_kdict + 1) * 4));
    TRY(get(o->pd_bytes, c->pd_bytes, I.pdict_bytes));
    TRY(get(o->pd_offs, c->pd_offs, ((size_t)I.n_pdict + 1) * 4));
    const size_t T = I.n_topos;
    TRY(get(o->ns, c->t_ns, T * 4));
    TRY(get(o->name, c->t_name, T * 4));
    TRY(get(o->src_ip, c->t_src, T * 4));
    TRY(get(o->net_ns, c->t_netns, T * 4));
    TRY(get(o->flags, c->t_flags, T));
    TRY(get(o->real_off, c->t_roff, (T + 1) * 4));
    TRY(get(o->des_off, c->t_noff, (T + 1) * 4));
    // AoSoA tiles → SoA columns
    auto cols = [&](const DevLinkStore& st, uint32_t* key, uint32_t* prop, uint32_t* gap, int64_t* uid) -> int {
        const uint32_t n = st.n;
        if (!n) return KDTN_OK;
        const size_t full = n / TILE_RECS, tail = n % TILE_RECS, tile_bytes = (size_t)TILE_WORDS * 4;
        const uint8_t* base = reinterpret_cast<const uint8_t*>(st.view.base);   // (des may read real's buffer)
        auto col = [&](int cidx, void* dst, size_t esz) -> int {
            if (!dst) return KDTN_OK;
            const size_t run = TILE_RECS * esz;
            const uint8_t* src = base + (size_t)cidx * TILE_RECS * 4;
            if (full) HIP_TRY(hipMemcpy2DAsync(dst, run, src, tile_bytes, run, full, hipMemcpyDeviceToHost, s));
            if (tail)
                HIP_TRY(hipMemcpyAsync(static_cast<uint8_t*>(dst) + full * run, src + full * tile_bytes, tail * esz,
                                       hipMemcpyDeviceToHost, s));
            return KDTN_OK;
        };
        for (int k = 0; k < KDTN_NKEY; ++k) TRY(col(COL_KEY0 + k, key ? key + (size_t)k * n : nullptr, 4));
        for (int k = 0; k < KDTN_NPROP; ++k) TRY(col(COL_PROP0 + k, prop ? prop + (size_t)k * n : nullptr, 4));
        TRY(col(COL_GAP, gap, 4));
        TRY(col(COL_UID, uid, 8));
        return KDTN_OK;
    };
    TRY(cols(c->des, o->des_key, o->des_prop, o->des_gap, o->des_uid));
    TRY(cols(c->real, o->real_key, o->real_prop, o->real_gap, o->real_uid));
    HIP_TRY(hipStreamSynchronize(s));
    return KDTN_OK;
}

}  // extern "C"

extern "C" {

int kdtn_comm_unique_id(uint8_t out[128]) {
    ncclUniqueId id;
    if (ncclGetUniqueId(&id) != ncclSuccess) return KDTN_EIO;
    static_assert(sizeof(id) == 128, "ncclUniqueId is 128 bytes");
    std::memcpy(out, &id, 128);
    return KDTN_OK;
}

int kdtn_comm_init(kdtn_ctx* c, const uint8_t uid[128], int nranks, int rank) {
    if (!c || !uid || nranks < 1 || rank < 0 || rank >= nranks) return KDTN_EINVAL;
    HIP_TRY(hipSetDevice(c->device));
    if (c->comm) {
        (void)ncclCommDestroy(c->comm);
        c->comm = nullptr;
    }
    c->nranks = nranks;
    c->rank = rank;
    c->uploaded = false;
    c->sh_active = false;
    c->pods_rank_major = true;
    if (!c->comm_stream) {
        HIP_TRY(hipStreamCreateWithFlags(&c->comm_stream, hipStreamNonBlocking));
        HIP_TRY(hipEventCreateWithFlags(&c->ev_fill, hipEventDisableTiming));
        HIP_TRY(hipEventCreateWithFlags(&c->ev_ag, hipEventDisableTiming));
    }
    ncclUniqueId id;
    std::memcpy(&id, uid, 128);
    ncclResult_t r = ncclCommInitRank(&c->comm, nranks, id, rank);
    if (r != ncclSuccess) {
        std::snprintf(g_last_error, sizeof(g_last_error), "ncclCommInitRank: %s", ncclGetErrorString(r));
        c->comm = nullptr;
        c->nranks = 1;
        c->rank = 0;
        return KDTN_EIO;
    }
    return KDTN_OK;
}

int kdtn_comm_set_ranks(kdtn_ctx* c, int nranks, int rank) {
    if (!c || nranks < 1 || rank < 0 || rank >= nranks) return KDTN_EINVAL;
    HIP_TRY(hipSetDevice(c->device));
    if (c->comm) {
        (void)ncclCommDestroy(c->comm);
        c->comm = nullptr;
    }
    c->nranks = nranks;
    c->rank = rank;
    c->uploaded = false;
    c->pods_imported = false;
    c->sh_active = false;                 // a new rank setup replaces a sharded ingest's
    c->pods_rank_major = true;
    return KDTN_OK;
}

int kdtn_pods_export(kdtn_ctx* c, kdtn_pod_row* rows) {
    if (!c || !c->uploaded || (c->slice && !rows)) return KDTN_EINVAL;
    HIP_TRY(hipSetDevice(c->device));
    const uint32_t rank_base = c->slice * (uint32_t)c->rank;
    uint4* pods = dp<uint4>(c->pods);
    if (c->slice) {
        k_pods_fill<<<nblocks(c->slice), BLOCK, 0, c->stream>>>(topo_view(c), c->slice, rank_base, pods);
        HIP_TRY(hipGetLastError());
        HIP_TRY(hipMemcpyAsync(rows, pods + rank_base, (size_t)c->slice * 16, hipMemcpyDeviceToHost, c->stream));
    }
    HIP_TRY(hipStreamSynchronize(c->stream));
    return KDTN_OK;
}

int kdtn_pods_import(kdtn_ctx* c, const kdtn_pod_row* rows, uint64_t n) {
    if (!c || !c->uploaded || n != c->pod_total || (n && !rows)) {
        if (c) std::snprintf(g_last_error, sizeof(g_last_error), "kdtn_pods_import: %llu rows, expected pod_slice*nranks = %u",
                             (unsigned long long)n, c->pod_total);
        return KDTN_EINVAL;
    }
    HIP_TRY(hipSetDevice(c->device));
    if (n) HIP_TRY(hipMemcpyAsync(c->pods.p, rows, (size_t)n * 16, hipMemcpyHostToDevice, c->stream));
    HIP_TRY(hipStreamSynchronize(c->stream));
    c->pods_imported = true;
    return KDTN_OK;
}

// getPod's API-server fallback (include/kdtn.h): rows of Topologies the informer store missed,
// after the gathered pod table, in every following run's peer lookup
int kdtn_epoch_late_pods(kdtn_ctx* c, const kdtn_pod_row* rows, uint32_t n) {
    if (!c || !c->uploaded || (n && !rows)) return KDTN_EINVAL;
    HIP_TRY(hipSetDevice(c->device));
    g_last_error[0] = 0;
    const uint32_t D = c->D;
    for (uint32_t i = 0; i < n; ++i) {
        const kdtn_pod_row& r = rows[i];
        if (r.ns >= D || r.name >= D || r.src_ip >= D || (r.net_ns_nil & 0x7FFFFFFFu) >= D) {
            std::snprintf(g_last_error, sizeof(g_last_error),
                          "kdtn_epoch_late_pods: row %u names a string past the dictionary (%u strings)", i, D);
            return KDTN_EINVAL;
        }
    }
    const uint64_t all = (uint64_t)c->pod_total + n;
    if (all > POD_INDEX) {
        std::snprintf(g_last_error, sizeof(g_last_error), "kdtn_epoch_late_pods: pod table of %llu entries exceeds 2^30",
                      (unsigned long long)all);
        return KDTN_EINVAL;
    }
    hipStream_t s = c->stream;
    // the gathered rows stay (a host-transport import, a sharded ingest's fill)
    TRY(ensure_keep(c->pods, (size_t)all * 16, (size_t)c->pod_total * 16, s));
    c->ovf_mask = next_pow2(all * 2) - 1;
    if (c->pod_ovf.cap < (size_t)(c->ovf_mask + 1) * 8) {       // stamped slots start zeroed
        TRY(ensure(c->pod_ovf, (size_t)(c->ovf_mask + 1) * 8));
        HIP_TRY(hipMemsetAsync(c->pod_ovf.p, 0, c->pod_ovf.cap, s));
    }
    if (n) HIP_TRY(hipMemcpyAsync(dp<uint4>(c->pods) + c->pod_total, rows, (size_t)n * 16, hipMemcpyHostToDevice, s));
    HIP_TRY(hipStreamSynchronize(s));             // the caller's rows may be released on return
    c->n_late = n;
    c->pods_ready = false;                        // the next run builds the lookup over every row
    c->pods_delta = false;
    return KDTN_OK;
}

int kdtn_debug_wg_trace(kdtn_ctx* c, uint64_t* out, uint32_t cap) {
    if (!c || !c->traced) return KDTN_EINVAL;
    HIP_TRY(hipSetDevice(c->device));
    HIP_TRY(hipStreamSynchronize(c->stream));
    const uint32_t n = std::min<uint64_t>(cap, (uint64_t)c->nwg * TRACE_WORDS);
    HIP_TRY(hipMemcpy(out, c->trace.p, (size_t)n * 8, hipMemcpyDeviceToHost));
    return (int)n;
}

}  // extern "C"

namespace {

// this rank's VxlanManager ops of the last run into vx_ops: [n_del del slots][2 n_add add slots]
int vni_ops_compute(kdtn_ctx* c, uint32_t* nd_out, uint32_t* na_out) {
    const uint32_t need = KDTN_STAGE_RESOLVE | KDTN_STAGE_QDISC;
    if (!c->ran || (c->last_stages & need) != need) {
        std::snprintf(g_last_error, sizeof(g_last_error),
                      "VXLAN ops: need an epoch run with the resolve and qdisc stages");
        return KDTN_EINVAL;
    }
    hipStream_t s = c->stream;
    HIP_TRY(hipStreamSynchronize(s));                 // counts of the run (h_misc)
    TRY(counts_fresh(c));
    const uint32_t nd = c->h_misc[1], na = c->h_misc[3];
    if (2ull * na + nd + c->V >= 0x7FFFFFFFull) return KDTN_EINVAL;
    TRY(ensure(c->vx_ops, ((size_t)nd + 2ull * na) * 16));
    VniOpsIn f{ReachIn{dp<uint32_t>(c->del_off), dp<uint4>(c->del_res), dp<uint32_t>(c->add_off), dp<uint4>(c->add_res),
                       dp<uint2>(c->add_qdisc), dp<uint32_t>(c->upd_off), dp<uint4>(c->upd_res), c->T, 0u},
               dp<uint32_t>(c->t_src), dp<uint32_t>(c->t_netns), dp<uint4>(c->pods), nd, na};
    TRY(ensure(c->vx_cut, (size_t)c->T * 8 + 8));
    uint32_t* cut = dp<uint32_t>(c->vx_cut);
    if (c->T) {
        HIP_TRY(hipMemsetAsync(cut, 0xFF, (size_t)c->T * 8, s));
        if (nd + na) {
            k_vni_cuts<<<nblocks((uint64_t)nd + na), BLOCK, 0, s>>>(f, cut);
            k_vni_ops<<<nblocks((uint64_t)nd + na), BLOCK, 0, s>>>(f, cut, dp<uint4>(c->vx_ops));
        }
    }
    HIP_TRY(hipGetLastError());
    *nd_out = nd;
    *na_out = na;
    return KDTN_OK;
}

// Every rank's ops in rank order, [all del slots][all add slots], into vx_gops over RCCL:
// the per-rank counts first, then one all-gather of lists padded to the largest rank's.
int vni_ops_gather_rccl(kdtn_ctx* c, uint32_t nd, uint32_t na, uint64_t* gd, uint64_t* ga) {
    hipStream_t s = c->stream;
    const int G = c->nranks;
    TRY(ensure(c->vx_cnt, (size_t)G * 8 + 16));
    uint32_t* cnt = dp<uint32_t>(c->vx_cnt);
    const uint32_t mine[2] = {nd, na};
    HIP_TRY(hipMemcpyAsync(cnt + 2 * c->rank, mine, 8, hipMemcpyHostToDevice, s));
    ncclResult_t r = ncclAllGather(cnt + 2 * c->rank, cnt, 2, ncclUint32, c->comm, s);
    if (r != ncclSuccess) {
        std::snprintf(g_last_error, sizeof(g_last_error), "ncclAllGather (VXLAN op counts): %s", ncclGetErrorString(r));
        return KDTN_EIO;
    }
    std::vector<uint32_t> h(2 * (size_t)G);
    HIP_TRY(hipMemcpyAsync(h.data(), cnt, 8 * (size_t)G, hipMemcpyDeviceToHost, s));
    HIP_TRY(hipStreamSynchronize(s));
    uint32_t md = 0, ma = 0;
    for (int g = 0; g < G; ++g) {
        md = std::max(md, h[2 * g]);
        ma = std::max(ma, h[2 * g + 1]);
    }
    const size_t row = (size_t)md + 2ull * ma;                 // ops per rank, padded
    TRY(ensure(c->vx_send, row * 16 + 16));
    TRY(ensure(c->vx_recv, row * G * 16 + 16));
    TRY(ensure(c->vx_gops, row * G * 16 + 16));
    uint8_t* send = dp<uint8_t>(c->vx_send);
    HIP_TRY(hipMemsetAsync(send, 0, row * 16, s));             // VOP_NONE padding
    if (nd) HIP_TRY(hipMemcpyAsync(send, c->vx_ops.p, (size_t)nd * 16, hipMemcpyDeviceToDevice, s));
    if (na)
        HIP_TRY(hipMemcpyAsync(send + (size_t)md * 16, dp<uint8_t>(c->vx_ops) + (size_t)nd * 16, 2ull * na * 16,
                               hipMemcpyDeviceToDevice, s));
    if (row) {
        r = ncclAllGather(send, c->vx_recv.p, row * 4, ncclUint32, c->comm, s);
        if (r != ncclSuccess) {
            std::snprintf(g_last_error, sizeof(g_last_error), "ncclAllGather (VXLAN ops): %s", ncclGetErrorString(r));
            return KDTN_EIO;
        }
        uint8_t* g = dp<uint8_t>(c->vx_gops);
        const uint8_t* rv = dp<uint8_t>(c->vx_recv);
        if (md) HIP_TRY(hipMemcpy2DAsync(g, (size_t)md * 16, rv, row * 16, (size_t)md * 16, G, hipMemcpyDeviceToDevice, s));
        if (ma)
            HIP_TRY(hipMemcpy2DAsync(g + (size_t)md * G * 16, 2ull * ma * 16, rv + (size_t)md * 16, row * 16,
                                     2ull * ma * 16, G, hipMemcpyDeviceToDevice, s));
    }
    *gd = (uint64_t)md * G;
    *ga = 2ull * ma * G;
    return KDTN_OK;
}

}  // namespace

extern "C" {

int kdtn_vni_ops_export(kdtn_ctx* c, kdtn_vni_op* dels, uint32_t del_cap, kdtn_vni_op* adds, uint32_t add_cap,
                        uint32_t* n_del, uint32_t* n_add) {
    if (!c || !n_del || !n_add) return KDTN_EINVAL;
    HIP_TRY(hipSetDevice(c->device));
    uint32_t nd = 0, na = 0;
    TRY(vni_ops_compute(c, &nd, &na));
    *n_del = nd;
    *n_add = 2 * na;
    if ((dels && nd > del_cap) || (adds && 2 * na > add_cap)) return KDTN_ENOSPC;
    hipStream_t s = c->stream;
    if (dels && nd) HIP_TRY(hipMemcpyAsync(dels, c->vx_ops.p, (size_t)nd * 16, hipMemcpyDeviceToHost, s));
    if (adds && na)
        HIP_TRY(hipMemcpyAsync(adds, dp<uint8_t>(c->vx_ops) + (size_t)nd * 16, 2ull * na * 16, hipMemcpyDeviceToHost, s));
    HIP_TRY(hipStreamSynchronize(s));
    return KDTN_OK;
}

int kdtn_vni_ops_import(kdtn_ctx* c, const kdtn_vni_op* dels, uint32_t n_del, const kdtn_vni_op* adds, uint32_t n_add) {
    if (!c || !c->ran || (n_del && !dels) || (n_add && !adds) || (uint64_t)n_del + n_add + c->V >= 0x7FFFFFFFull)
        return KDTN_EINVAL;
    HIP_TRY(hipSetDevice(c->device));
    hipStream_t s = c->stream;
    TRY(ensure(c->vx_gops, ((size_t)n_del + n_add) * 16 + 16));
    if (n_del) HIP_TRY(hipMemcpyAsync(c->vx_gops.p, dels, (size_t)n_del * 16, hipMemcpyHostToDevice, s));
    if (n_add)
        HIP_TRY(hipMemcpyAsync(dp<uint8_t>(c->vx_gops) + (size_t)n_del * 16, adds, (size_t)n_add * 16,
                               hipMemcpyHostToDevice, s));
    HIP_TRY(hipStreamSynchronize(s));
    c->vx_gd = n_del;
    c->vx_ga = n_add;
    c->vx_imported = true;
    return KDTN_OK;
}

int kdtn_epoch_vni_apply(kdtn_ctx* c, kdtn_vni_state* out) {
    if (!c || !c->ran) return KDTN_EINVAL;
    HIP_TRY(hipSetDevice(c->device));
    hipStream_t s = c->stream;
    const bool host_xchg = c->nranks > 1 && !c->comm;
    if (host_xchg && !c->vx_imported) {
        std::snprintf(g_last_error, sizeof(g_last_error),
                      "host transport: kdtn_vni_ops_import every rank's VXLAN ops before kdtn_epoch_vni_apply");
        return KDTN_EINVAL;
    }
    if (c->nranks > 1 && !c->pods_rank_major && !host_xchg) {
        std::snprintf(g_last_error, sizeof(g_last_error), "kdtn_epoch_vni_apply: sharded ingest contexts use the host transport");
        return KDTN_EINVAL;
    }
    c->n_ev = 0;
    (void)hipEventRecord(c->ev[0], s);
    const uint32_t V = c->V;
    uint64_t nd_all = 0, n_ops = 0;
    const uint4* ops = nullptr;
    if (!host_xchg) {
        uint32_t nd = 0, na = 0;
        TRY(vni_ops_compute(c, &nd, &na));
        if (c->nranks > 1) {
            TRY(vni_ops_gather_rccl(c, nd, na, &nd_all, &n_ops));
            ops = dp<uint4>(c->vx_gops);
        } else {
            nd_all = nd;
            n_ops = 2ull * na;
            ops = dp<uint4>(c->vx_ops);
        }
    } else {
        nd_all = c->vx_gd;
        n_ops = c->vx_ga;
        ops = dp<uint4>(c->vx_gops);
    }
    const uint64_t n_ext = n_ops + V;
    if (n_ext + nd_all >= 0x7FFFFFFFull) return KDTN_EINVAL;
    TRY(ensure(c->vx_dead, (size_t)V + 16));
    const uint4* ents = dp<uint4>(c->v_ents);
    uint8_t* dead = dp<uint8_t>(c->vx_dead);
    if (V) {                                          // the run built the snapshot table
        k_vni_shadow<<<nblocks(V), BLOCK, 0, s>>>(ents, V, dp<uint32_t>(c->v_slots), c->vni_mask, dead);
        if (nd_all) k_vni_del<<<nblocks(nd_all), BLOCK, 0, s>>>(ops, (uint32_t)nd_all, ents, dp<uint32_t>(c->v_slots),
                                                                c->vni_mask, dead);
    }
    timer_mark(c, "vni_ops");
    const uint32_t mask = next_pow2(n_ext * 2) - 1;
    TRY(ensure(c->vx_slots, ((size_t)mask + 1) * 4));
    HIP_TRY(hipMemsetAsync(c->vx_slots.p, 0xFF, ((size_t)mask + 1) * 4, s));
    uint32_t* slots = dp<uint32_t>(c->vx_slots);
    const uint4* aops = ops + nd_all;
    const uint32_t nb = nblocks(n_ext, SCAN_CHUNK);
    TRY(ensure(c->vx_part, (size_t)nb * 8 + 8));
    TRY(ensure(c->vx_node, (size_t)n_ext * 4));
    TRY(ensure(c->vx_vni, (size_t)n_ext * 4));
    TRY(ensure(c->vx_netns, (size_t)n_ext * 4));
    TRY(ensure(c->vx_vis, (size_t)n_ext + 16));
    uint32_t* n_out = dp<uint32_t>(c->misc) + MISC_VNI_N;
    HIP_TRY(hipMemsetAsync(n_out, 0, 4, s));
    if (n_ext) {
        k_vni_insert<<<nblocks(n_ext), BLOCK, 0, s>>>(aops, (uint32_t)n_ops, ents, dead, V, slots, mask);
        uint8_t* vis = dp<uint8_t>(c->vx_vis);
        k_vni_vis_count<<<nb, BLOCK, 0, s>>>(aops, (uint32_t)n_ops, ents, dead, V, slots, mask, vis,
                                            dp<uint64_t>(c->vx_part));
        k_scan_top<<<1, SCAN_TOP_BLOCK, 0, s>>>(dp<uint64_t>(c->vx_part), nb);
        k_vni_vis_write<<<nb, BLOCK, 0, s>>>(aops, (uint32_t)n_ops, ents, dead, V, vis, dp<uint64_t>(c->vx_part),
                                            dp<uint32_t>(c->vx_node), dp<int32_t>(c->vx_vni), dp<uint32_t>(c->vx_netns),
                                            n_out);
    }
    HIP_TRY(hipGetLastError());
    timer_mark(c, "vni_map");
    // keys whose result depends on the reference's goroutine order (kdtn_vni_contested)
    const uint32_t dmask = nd_all ? next_pow2(nd_all * 2) - 1 : 0u;
    const uint32_t nbf = nblocks(n_ops + 1, SCAN_CHUNK);
    TRY(ensure(c->vx_flag, (size_t)n_ops * 4 + 16));
    TRY(ensure(c->vx_dkeys, ((size_t)dmask + 1) * 16));
    TRY(ensure(c->vx_dused, ((size_t)dmask + 1) * 4));
    TRY(ensure(c->vx_cpos, ((size_t)n_ops + 1) * 8));
    TRY(ensure(c->vx_cpart, (size_t)nbf * 8 + 8));
    TRY(ensure(c->vx_cnode, (size_t)n_ops * 4 + 16));
    TRY(ensure(c->vx_cvni, (size_t)n_ops * 4 + 16));
    HIP_TRY(hipMemsetAsync(c->vx_flag.p, 0, (size_t)n_ops * 4 + 16, s));
    HIP_TRY(hipMemsetAsync(c->vx_dused.p, 0, ((size_t)dmask + 1) * 4, s));
    if (nd_all) k_vni_dtab_insert<<<nblocks(nd_all), BLOCK, 0, s>>>(ops, (uint32_t)nd_all, dp<uint4>(c->vx_dkeys),
                                                                     dp<uint32_t>(c->vx_dused), dmask);
    if (n_ops) k_vni_contest<<<nblocks(n_ops), BLOCK, 0, s>>>(aops, (uint32_t)n_ops, ents, dead, slots, mask,
                                                             dp<uint4>(c->vx_dkeys), dp<uint32_t>(c->vx_dused),
                                                             nd_all ? dmask : 0u, dp<uint32_t>(c->vx_flag));
    k_scan_partial<<<nbf, BLOCK, 0, s>>>(dp<uint32_t>(c->vx_flag), (uint32_t)n_ops, dp<uint64_t>(c->vx_cpart));
    k_scan_top<<<1, SCAN_TOP_BLOCK, 0, s>>>(dp<uint64_t>(c->vx_cpart), nbf);
    k_scan_final<<<nbf, BLOCK, 0, s>>>(dp<uint32_t>(c->vx_flag), (uint32_t)n_ops, dp<uint64_t>(c->vx_cpart),
                                       dp<uint64_t>(c->vx_cpos));
    if (n_ops) k_vni_contest_write<<<nblocks(n_ops), BLOCK, 0, s>>>(aops, dp<uint32_t>(c->vx_flag),
                                                                   dp<uint64_t>(c->vx_cpos), (uint32_t)n_ops,
                                                                   dp<uint32_t>(c->vx_cnode), dp<int32_t>(c->vx_cvni));
    HIP_TRY(hipGetLastError());
    timer_mark(c, "vni_contested");
    HIP_TRY(hipMemcpyAsync(c->h_misc + 5, n_out, 4, hipMemcpyDeviceToHost, s));
    HIP_TRY(hipMemcpyAsync(c->h_misc + 6, dp<uint64_t>(c->vx_cpos) + n_ops, 4, hipMemcpyDeviceToHost, s));
    HIP_TRY(hipStreamSynchronize(s));
    const uint32_t n = c->h_misc[5];
    c->vx_ncont = c->h_misc[6];
    c->vx_contest_ok = true;
    // the new map becomes the resident one (the next upload's KDTN_VNI_RESIDENT); this upload's
    // snapshot (v_*, v_ents, V) stays as it is, so a re-run or a second apply of this upload
    // sees the same epoch-start map
    std::swap(c->r_node, c->vx_node);
    std::swap(c->r_vni, c->vx_vni);
    std::swap(c->r_netns, c->vx_netns);
    c->vres_ok = true;
    c->vres_in_r = true;
    c->vres_n = n;
    c->vres_D = c->D;
    return out ? kdtn_vni_download(c, out) : KDTN_OK;
}

int kdtn_vni_contested(kdtn_ctx* c, uint32_t* node, int32_t* vni, uint32_t cap, uint32_t* n) {
    if (!c || !n || !c->vx_contest_ok) return KDTN_EINVAL;
    HIP_TRY(hipSetDevice(c->device));
    *n = c->vx_ncont;
    if (!node && !vni) return KDTN_OK;
    if (c->vx_ncont > cap) return KDTN_ENOSPC;
    hipStream_t s = c->stream;
    if (c->vx_ncont && node)
        HIP_TRY(hipMemcpyAsync(node, c->vx_cnode.p, (size_t)c->vx_ncont * 4, hipMemcpyDeviceToHost, s));
    if (c->vx_ncont && vni) HIP_TRY(hipMemcpyAsync(vni, c->vx_cvni.p, (size_t)c->vx_ncont * 4, hipMemcpyDeviceToHost, s));
    HIP_TRY(hipStreamSynchronize(s));
    return KDTN_OK;
}

int kdtn_vni_download(kdtn_ctx* c, kdtn_vni_state* out) {
    if (!c || !out) return KDTN_EINVAL;
    if (!c->vres_ok) {
        out->n = 0;
        return KDTN_OK;
    }
    HIP_TRY(hipSetDevice(c->device));
    const uint32_t n = c->vres_n;
    out->n = n;
    if (!out->node && !out->vni && !out->net_ns) return KDTN_OK;
    if (n > out->cap) return KDTN_ENOSPC;
    hipStream_t s = c->stream;
    DevBuf& bn = c->vres_in_r ? c->r_node : c->v_node;
    DevBuf& bv = c->vres_in_r ? c->r_vni : c->v_vni;
    DevBuf& bs = c->vres_in_r ? c->r_netns : c->v_netns;
    if (n && out->node) HIP_TRY(hipMemcpyAsync(out->node, bn.p, (size_t)n * 4, hipMemcpyDeviceToHost, s));
    if (n && out->vni) HIP_TRY(hipMemcpyAsync(out->vni, bv.p, (size_t)n * 4, hipMemcpyDeviceToHost, s));
    if (n && out->net_ns) HIP_TRY(hipMemcpyAsync(out->net_ns, bs.p, (size_t)n * 4, hipMemcpyDeviceToHost, s));
    HIP_TRY(hipStreamSynchronize(s));
    return KDTN_OK;
}

int kdtn_set_timing(kdtn_ctx* c, int level) {
    if (!c || level < 0 || level > 2) return KDTN_EINVAL;
    c->timing = level;
    return KDTN_OK;
}

int kdtn_last_kernel_times(kdtn_ctx* c, const char** names, float* ms, int cap) {
    if (!c) return KDTN_EINVAL;
    (void)hipSetDevice(c->device);
    (void)hipStreamSynchronize(c->stream);
    int n = std::min(cap, c->n_ev);
    for (int i = 0; i < n; ++i) {
        if (names) names[i] = c->ev_name[i];
        float t = 0.f;
        (void)hipEventElapsedTime(&t, c->ev[i], c->ev[i + 1]);
        if (ms) ms[i] = t;
    }
    return n;
}

// ---- resident epoch state (kdtn_state.hip) ----------------------------------------------
}  // extern "C"

namespace {

// Device layout of a delta's arrays (and the host layout that lets them travel in one copy,
// kdtn.engine.pin_delta): topo, src_ip, net_ns, des_off, [prev, ns, name], spec_nil, then the
// references 4-B aligned.
struct DeltaPack {
    size_t topo, src, netns, off, prev, ns, name, nil, ref, total;
    DeltaPack(uint32_t n, uint32_t nref, uint32_t remap_T) {
        topo = 0;
        src = topo + (size_t)n * 4;
        netns = src + (size_t)n * 4;
        off = netns + (size_t)n * 4;
        prev = off + (n ? ((size_t)n + 1) * 4 : 0);
        ns = prev + (size_t)remap_T * 4;
        name = ns + (remap_T ? (size_t)n * 4 : 0);
        nil = name + (remap_T ? (size_t)n * 4 : 0);
        ref = align_up(nil + n, 4);
        total = ref + (size_t)nref * 4;
    }
};

// offsets of a store from per-topology lengths: u64 (off64[T] = total) and u32, no readback
int scan_lengths(kdtn_ctx* c, DevBuf& len, uint32_t T, DevBuf& off64, DevBuf& part, DevBuf& off32) {
    hipStream_t s = c->stream;
    const uint32_t nb = nblocks((uint64_t)T + 1, SCAN_CHUNK);
    TRY(ensure(off64, ((size_t)T + 1) * 8));
    TRY(ensure(part, (size_t)nb * 8 + 16));
    TRY(ensure(off32, ((size_t)T + 1) * 4));
    k_scan_partial<<<nb, BLOCK, 0, s>>>(dp<uint32_t>(len), T, dp<uint64_t>(part));
    k_scan_top<<<1, SCAN_TOP_BLOCK, 0, s>>>(dp<uint64_t>(part), nb);
    k_scan_final<<<nb, BLOCK, 0, s>>>(dp<uint32_t>(len), T, dp<uint64_t>(part), dp<uint64_t>(off64));
    k_off_narrow<<<nblocks((uint64_t)T + 1), BLOCK, 0, s>>>(dp<uint64_t>(off64), T, dp<uint32_t>(off32));
    HIP_TRY(hipGetLastError());
    return KDTN_OK;
}

// new u32 offsets of a store from per-topology lengths (st_len) into st_off32; returns the total
int plan_offsets(kdtn_ctx* c, uint32_t T, uint64_t* total) {
    hipStream_t s = c->stream;
    TRY(scan_lengths(c, c->st_len, T, c->st_off64, c->st_part, c->st_off32));
    HIP_TRY(hipMemcpyAsync(total, dp<uint64_t>(c->st_off64) + T, 8, hipMemcpyDeviceToHost, s));
    HIP_TRY(hipStreamSynchronize(s));
    if (*total >= 0x7FFFFFFFull) {
        std::snprintf(g_last_error, sizeof(g_last_error), "link store of %llu records", (unsigned long long)*total);
        return KDTN_EINVAL;
    }
    return KDTN_OK;
}

// The resident pod tables after a delta: the changed Topologies' rows (dl_topo, n of them on
// this rank) patched into the pod table and their lookup slots, instead of the next runs
// refilling, exchanging and rebuilding all of them. Across RCCL ranks the changed rows are
// all-gathered (the per-rank counts first, then the rows padded to the largest count); when
// some rank changed more than a quarter of a slice, or the tables are not resident (host
// transport, no full build yet), the next run does the full build instead.
int patch_pods(kdtn_ctx* c, uint32_t n) {
    c->pods_delta = false;
    if (!c->pods_ready) return KDTN_OK;
    const bool rccl = c->comm != nullptr;
    if (c->nranks > 1 && (!rccl || !c->pods_rank_major)) {
        c->pods_ready = false;
        return KDTN_OK;
    }
    hipStream_t s = c->stream;
    const int G = rccl ? c->nranks : 1;
    uint32_t m = n;
    if (G > 1) {
        TRY(ensure(c->pd_cnt, (size_t)G * 4 + 16));
        uint32_t* cnt = dp<uint32_t>(c->pd_cnt);
        HIP_TRY(hipMemcpyAsync(cnt + c->rank, &n, 4, hipMemcpyHostToDevice, s));
        ncclResult_t r = ncclAllGather(cnt + c->rank, cnt, 1, ncclUint32, c->comm, s);
        if (r != ncclSuccess) {
            std::snprintf(g_last_error, sizeof(g_last_error), "ncclAllGather (changed pod rows): %s", ncclGetErrorString(r));
            return KDTN_EIO;
        }
        std::vector<uint32_t> h((size_t)G);
        HIP_TRY(hipMemcpyAsync(h.data(), cnt, (size_t)G * 4, hipMemcpyDeviceToHost, s));
        HIP_TRY(hipStreamSynchronize(s));
        m = *std::max_element(h.begin(), h.end());
    }
    if ((uint64_t)m * 4 > (uint64_t)c->slice + 4096) {      // a full exchange is cheaper
        c->pods_ready = false;
        return KDTN_OK;
    }
    if (m) {
        TRY(ensure(c->pd_send, (size_t)m * 32));
        TRY(ensure(c->pd_recv, (size_t)m * G * 32));
        k_pods_pack<<<nblocks(m), BLOCK, 0, s>>>(topo_view(c), dp<uint32_t>(c->dl_rows), n, m,
                                                 c->slice * (uint32_t)c->rank, dp<uint4>(c->pd_send));
        const uint4* ent = dp<uint4>(c->pd_send);
        if (G > 1) {
            ncclResult_t r = ncclAllGather(c->pd_send.p, c->pd_recv.p, (size_t)m * 8, ncclUint32, c->comm, s);
            if (r != ncclSuccess) {
                std::snprintf(g_last_error, sizeof(g_last_error), "ncclAllGather (pod rows): %s", ncclGetErrorString(r));
                return KDTN_EIO;
            }
            ent = dp<uint4>(c->pd_recv);
        }
        k_pods_patch<<<nblocks((uint64_t)m * G), BLOCK, 0, s>>>(ent, m * (uint32_t)G, dp<uint4>(c->pods),
                                                               dp<uint4>(c->pod_direct), c->pod_stamp, c->D);
        HIP_TRY(hipGetLastError());
    }
    c->pods_delta = true;
    return KDTN_OK;
}

// per-topology plan arrays for T topologies
int plan_alloc(kdtn_ctx* c, uint32_t T) {
    TRY(ensure(c->st_cnt, 32 * 4));
    TRY(ensure(c->st_len, (size_t)T * 4 + 16));
    TRY(ensure(c->st_base, (size_t)T * 4 + 16));
    TRY(ensure(c->st_mode, (size_t)T + 16));
    TRY(ensure(c->st_flags, (size_t)T + 16));
    return KDTN_OK;
}

void state_changed(kdtn_ctx* c) {
    c->ran = false;
    c->encoded = false;
    c->tc_done = false;
    c->fan_valid = false;
    c->lc_valid = false;
    c->si_run = false;
    c->rp_done = false;
    c->j_done = false;
    c->tables_cur = false;
}

}  // namespace

extern "C" {

int kdtn_epoch_commit(kdtn_ctx* c, const uint8_t* mask, uint32_t* n_committed) {
    if (!c || !c->uploaded) return KDTN_EINVAL;
    if (!mask && (!c->ran || !fanout_stages_ok(c))) {
        std::snprintf(g_last_error, sizeof(g_last_error),
                      "kdtn_epoch_commit without a mask needs a run with the resolve and qdisc stages");
        return KDTN_EINVAL;
    }
    HIP_TRY(hipSetDevice(c->device));
    hipStream_t s = c->stream;
    HIP_TRY(hipStreamSynchronize(s));
    const uint32_t T = c->T;
    if (mask && T && std::memchr(mask, 0, T) == nullptr) {
        // every Topology committed: the realised store IS the desired store (the same records at
        // the same offsets), so no reassembly — real takes the desired store's buffer, des keeps
        // reading that memory (every writer of des resets its view to its own buffer first),
        // real_off := des_off and the status-nil flags follow the spec's
        k_commit_all_flags<<<nblocks(T), BLOCK, 0, s>>>(dp<uint8_t>(c->t_flags), T);
        HIP_TRY(hipMemcpyAsync(c->t_roff.p, c->t_noff.p, ((size_t)T + 1) * 4, hipMemcpyDeviceToDevice, s));
        HIP_TRY(hipGetLastError());
        std::swap(c->real, c->des);
        c->des.view = c->real.view;
        c->des.n = c->real.n;
        TRY(prepare_work(c, c->slice, c->real.n, c->des.n));
        HIP_TRY(hipStreamSynchronize(s));
        state_changed(c);
        c->pods_imported = false;
        if (n_committed) *n_committed = T;
        return KDTN_OK;
    }
    TRY(plan_alloc(c, T));
    const uint8_t* dmask = nullptr;
    const uint32_t* cut = nullptr;
    if (mask) {
        TRY(upload(c, c->st_mask, mask, T));
        dmask = dp<uint8_t>(c->st_mask);
    } else {
        TRY(counts_fresh(c));
        TRY(run_reach(c, nullptr, 0));                      // per-topology first failing entries
        cut = dp<uint32_t>(c->f_cut);
    }
    uint32_t* ncnt = dp<uint32_t>(c->st_cnt);
    HIP_TRY(hipMemsetAsync(ncnt, 0, 32 * 4, s));
    if (T)
        k_commit_plan<<<nblocks(T), BLOCK, 0, s>>>(topo_view(c), dp<uint8_t>(c->action), cut, dmask,
                                                   dp<uint32_t>(c->st_len), dp<uint32_t>(c->st_base),
                                                   dp<uint8_t>(c->st_mode), dp<uint8_t>(c->st_flags), ncnt);
    uint64_t M = 0;
    TRY(plan_offsets(c, T, &M));
    TRY(link_store_alloc(c, c->sh_real, (uint32_t)M));
    if (M)
        k_store_assemble<<<nblocks(M), BLOCK, 0, s>>>(dp<uint32_t>(c->st_off32), T, dp<uint32_t>(c->st_base),
                                                      dp<uint8_t>(c->st_mode), nullptr, c->real.view, c->des.view,
                                                      (uint32_t)M, AsmGuard{}, dp<uint32_t>(c->sh_real.buf));
    HIP_TRY(hipGetLastError());
    uint32_t cnt[32] = {};
    HIP_TRY(hipMemcpyAsync(cnt, ncnt, sizeof cnt, hipMemcpyDeviceToHost, s));
    HIP_TRY(hipStreamSynchronize(s));
    uint32_t nc = 0;
    for (uint32_t v : cnt) nc += v;
    std::swap(c->real, c->sh_real);
    std::swap(c->t_roff, c->st_off32);
    std::swap(c->t_flags, c->st_flags);
    TRY(prepare_work(c, c->slice, c->real.n, c->des.n));
    HIP_TRY(hipStreamSynchronize(s));
    state_changed(c);
    c->pods_imported = false;
    if (n_committed) *n_committed = nc;
    return KDTN_OK;
}

int kdtn_epoch_upload_delta(kdtn_ctx* c, const kdtn_epoch_delta* d) {
    if (!c || !d || !c->uploaded) return KDTN_EINVAL;
    HIP_TRY(hipSetDevice(c->device));
    g_last_error[0] = 0;
    end_shard_ingest(c);
    TRY(check_strtab(d->kdict, "kdict", d->kdict_keep));
    TRY(check_strtab(d->pdict, "pdict", d->pdict_keep));
    const bool remap = d->prev != nullptr;                 // the Topology set changes
    const uint32_t T0 = c->T, Tn = remap ? d->n_topos : T0, n = d->n_changed;
    const uint32_t N0 = c->des.n, M0 = c->real.n, D = d->kdict.n, P = d->pdict.n;
    const uint32_t kk = d->kdict_keep, pk = d->pdict_keep;
    auto bad = [&](const char* what, uint32_t i) {
        std::snprintf(g_last_error, sizeof(g_last_error), "delta: %s (at %u)", what, i);
        return KDTN_EINVAL;
    };
    // O(1) host checks; everything per element is checked on the GPU (k_delta_check, k_delta_plan,
    // the inline records' column maxima) and read back with the call's one synchronisation
    if (kk != c->D || pk != c->P) {
        std::snprintf(g_last_error, sizeof(g_last_error),
                      "delta: kdict_keep %u / pdict_keep %u must equal the resident dictionaries' sizes %u / %u "
                      "(a delta extends them; a shrunk or rewritten dictionary needs kdtn_epoch_upload)",
                      kk, pk, c->D, c->P);
        return KDTN_EINVAL;
    }
    if (kk > c->kd_valid || pk > c->pd_valid) return bad("the resident dictionaries were not parsed (run first)", kk);
    // the kept prefixes end where the resident arenas end (before any copy is enqueued: the
    // suffixes are written at the host's offsets, which must not overlap resident bytes)
    if (d->kdict.offs[kk] != c->kd_arena || d->pdict.offs[pk] != c->pd_arena) {
        std::snprintf(g_last_error, sizeof(g_last_error),
                      "delta: the kept dictionary prefixes end at byte %u / %u, the resident arenas at %llu / %llu",
                      d->kdict.offs[kk], d->pdict.offs[pk], (unsigned long long)c->kd_arena,
                      (unsigned long long)c->pd_arena);
        return KDTN_EINVAL;
    }
    if (n > Tn) return bad("more changed topologies than topologies", n);
    if (n && (!d->topo || !d->src_ip || !d->net_ns || !d->spec_nil || !d->des_off)) return bad("missing column", 0);
    if (remap && n && (!d->ns || !d->name)) return bad("missing ns / name of the changed topologies", 0);
    const uint32_t nref = n ? d->des_off[n] : 0;
    if (n && d->des_off[0] != 0) return bad("des_off[0] != 0", 0);
    if (nref && !d->ref) return bad("missing ref", 0);
    const uint32_t slice = remap ? (d->pod_slice ? d->pod_slice : Tn) : c->slice;
    if (slice < Tn) return bad("pod_slice below n_topos", slice);
    const uint64_t nbound = (uint64_t)N0 + nref;            // kept segments + the changed lists
    if (nbound >= 0x7FFFFFFFull) return bad("desired store over 2^31 records", (uint32_t)(nbound >> 32));
    TRY(check_vnis(c, d->vnis, D, kk));
    const kdtn_link_table& L = d->records;
    const uint32_t nr = L.n;
    if (nr) {
        for (int k = 0; k < KDTN_NKEY; ++k)
            if (!L.key[k]) return bad("records: missing key column", k);
        for (int k = 0; k < KDTN_NPROP; ++k)
            if (!L.prop[k]) return bad("records: missing prop column", k);
        if (!L.uid || !L.gap) return bad("records: missing uid / gap", 0);
    }
    // Two streams: the host-to-device copies on the copy stream, in the order the kernels need
    // them (the delta's arrays, its references, the dictionary suffixes, the inline records),
    // and the kernels on the context stream, each waiting only for its inputs — so the plan and
    // the assembly of the kept and referenced records run while the inline records cross the
    // host link. Buffers are sized first (an allocation may synchronise the device).
    hipStream_t s = c->stream;
    hipStream_t cs = c->copy_stream ? c->copy_stream : s;
    TRY(ensure(c->misc, 256));
    uint32_t* misc = dp<uint32_t>(c->misc);
    // the delta's arrays in one device block (DeltaPack): a caller whose host arrays sit in the
    // same layout (kdtn.engine.pin_delta) has them copied by one or two copies
    const DeltaPack pk_{n, nref, remap ? Tn : 0u};
    TRY(ensure(c->dl_pack, pk_.total + 64));
    uint8_t* pack = dp<uint8_t>(c->dl_pack);
    uint32_t* p_topo = reinterpret_cast<uint32_t*>(pack + pk_.topo);
    uint32_t* p_src = reinterpret_cast<uint32_t*>(pack + pk_.src);
    uint32_t* p_netns = reinterpret_cast<uint32_t*>(pack + pk_.netns);
    uint32_t* p_off = reinterpret_cast<uint32_t*>(pack + pk_.off);
    uint32_t* p_prev = reinterpret_cast<uint32_t*>(pack + pk_.prev);
    uint32_t* p_ns = reinterpret_cast<uint32_t*>(pack + pk_.ns);
    uint32_t* p_name = reinterpret_cast<uint32_t*>(pack + pk_.name);
    uint8_t* p_nil = pack + pk_.nil;
    uint32_t* p_ref = reinterpret_cast<uint32_t*>(pack + pk_.ref);
    TRY(link_store_alloc(c, c->dl_rec, nr));
    const size_t col = (size_t)nr * 4, uid_at = align_up(col * LINK_COLS32, 8);
    TRY(ensure(c->stage, uid_at + (size_t)nr * 8 + 128));
    TRY(ensure(c->dl_dest, (size_t)nr * 4));
    TRY(plan_alloc(c, Tn));
    TRY(ensure(c->st_chg, (size_t)Tn * 4 + 16));
    TRY(ensure(c->dl_rows, (size_t)n * 4 + 16));
    TRY(ensure(c->sh_src, (size_t)Tn * 4));
    TRY(ensure(c->sh_netns, (size_t)Tn * 4));
    TRY(ensure(c->sh_flags, (size_t)Tn));
    if (remap) {
        TRY(ensure(c->sh_ns, (size_t)Tn * 4));
        TRY(ensure(c->sh_name, (size_t)Tn * 4));
        TRY(ensure(c->st_rlen, (size_t)Tn * 4 + 16));
        TRY(ensure(c->st_rbase, (size_t)Tn * 4 + 16));
        TRY(ensure(c->st_mask, (size_t)Tn + 16));
        TRY(ensure(c->st_seen, ((size_t)T0 + 31) / 32 * 4 + 16));
    }
    TRY(link_store_alloc(c, c->sh_des, (uint32_t)nbound));
    if (remap) TRY(link_store_alloc(c, c->sh_real, M0));
    // --- copies (copy stream), after everything already queued on the context stream. From here
    // on an error return first waits for both streams: the copies read the caller's arrays,
    // which it may release once the call has returned
    StreamsDrain drain{s, cs};
    HIP_TRY(hipEventRecord(c->ev_cp[0], s));
    if (cs != s) HIP_TRY(hipStreamWaitEvent(cs, c->ev_cp[0], 0));
    {   // segments in pack order; host-adjacent neighbours merge into one copy. The per-Topology
        // arrays go first and alone (the plan and the kept segments' assembly need only them),
        // then the references
        const void* src[9] = {d->topo, d->src_ip, d->net_ns, d->des_off, d->prev, d->ns, d->name, d->spec_nil, d->ref};
        const size_t at[9] = {pk_.topo, pk_.src, pk_.netns, pk_.off, pk_.prev, pk_.ns, pk_.name, pk_.nil, pk_.ref};
        const size_t len[9] = {(size_t)n * 4, (size_t)n * 4, (size_t)n * 4, pk_.prev - pk_.off, pk_.ns - pk_.prev,
                               pk_.name - pk_.ns, pk_.nil - pk_.name, (size_t)n, (size_t)nref * 4};
        int i = 0;
        while (i < 9) {
            if (!len[i]) { ++i; continue; }
            const uint8_t* h0 = static_cast<const uint8_t*>(src[i]);
            size_t bytes = len[i];
            int j = i + 1;
            // the device block is contiguous (padding included): the host array must sit at the
            // same distance from the run's start
            while (j < (i < 8 ? 8 : 9) && (!len[j] || static_cast<const uint8_t*>(src[j]) == h0 + (at[j] - at[i]))) {
                if (len[j]) bytes = at[j] + len[j] - at[i];
                ++j;
            }
            HIP_TRY(hipMemcpyAsync(pack + at[i], h0, bytes, hipMemcpyHostToDevice, cs));
            if (i <= 7 && j >= 8) HIP_TRY(hipEventRecord(c->ev_cp[1], cs));   // the small arrays are in
            i = j;
        }
        if (!n) HIP_TRY(hipEventRecord(c->ev_cp[1], cs));
    }
    HIP_TRY(hipEventRecord(c->ev_cp[2], cs));                                   // and the references
    c->uploaded = false;                            // (restored below when the delta is rejected)
    const uint32_t saved[6] = {c->D, c->P, c->kd_valid, c->pd_valid, c->kd_from, c->pd_from};
    const uint64_t saved_arena[2] = {c->kd_arena, c->pd_arena};
    // appends past the resident strings (the kept prefix's end offset is not rewritten: the
    // check below compares it with the host's)
    TRY(upload_dicts(c, d->kdict, d->pdict, kk, pk, cs));
    uint8_t* st = static_cast<uint8_t*>(c->stage.p);
    uint32_t segs[LINK_COLS32][2];
    int nseg = 0;
    if (nr) {
        TRY(stage_columns(c, st, L, col, cs, segs, &nseg));
        HIP_TRY(hipMemcpyAsync(st + uid_at, L.uid, (size_t)nr * 8, hipMemcpyHostToDevice, cs));
        HIP_TRY(hipEventRecord(c->ev_col[nseg], cs));
    }
    HIP_TRY(hipEventRecord(c->ev_cp[3], cs));
    // --- kernels (context stream)
    uint32_t* colmax = misc + MISC_COLMAX;
    HIP_TRY(hipMemsetAsync(misc + MISC_DELTA_ERR, 0, 4, s));
    HIP_TRY(hipMemsetAsync(misc + MISC_ROWCHG_N, 0, 4, s));
    HIP_TRY(hipMemsetAsync(colmax, 0, COL_GAP * 4, s));
    HIP_TRY(hipMemsetAsync(misc + MISC_DELTA_MULTI, 0, 4, s));
    if (nr) HIP_TRY(hipMemsetAsync(c->dl_dest.p, 0xFF, (size_t)nr * 4, s));
    HIP_TRY(hipMemsetAsync(c->st_chg.p, 0xFF, (size_t)Tn * 4, s));
    if (remap) {
        HIP_TRY(hipMemsetAsync(c->st_seen.p, 0, ((size_t)T0 + 31) / 32 * 4 + 16, s));
        HIP_TRY(hipMemsetAsync(c->st_mask.p, ASM_SEG_A, (size_t)Tn + 16, s));
    }
    if (cs != s) HIP_TRY(hipStreamWaitEvent(s, c->ev_cp[1], 0));
    if (n) k_delta_map<<<nblocks(n), BLOCK, 0, s>>>(p_topo, n, Tn, dp<uint32_t>(c->st_chg));
    const DeltaCheckIn ci{p_topo, p_off, p_nil,
                          p_src, p_netns, p_ref,
                          dp<uint32_t>(c->kd_offs), dp<uint32_t>(c->pd_offs), n, nref, Tn, D, nr, N0,
                          kk, pk, d->kdict.offs[kk], d->pdict.offs[pk]};
    {   // the per-Topology arrays and the kept dictionaries now; the references once they are in
        DeltaCheckIn c1 = ci;
        c1.nref = 0;
        k_delta_check<<<std::max<uint32_t>(1u, nblocks(n)), BLOCK, 0, s>>>(c1, misc + MISC_DELTA_ERR);
    }
    // plan over the new topology table: new rows into scratch columns, the state is untouched
    DeltaPlanIn pi{topo_view(c), dp<uint32_t>(c->st_chg), remap ? p_prev : nullptr,
                   p_off, p_src, p_netns, p_nil,
                   p_ns, p_name, Tn, D};
    DeltaPlanOut po{dp<uint32_t>(c->sh_ns), dp<uint32_t>(c->sh_name), dp<uint32_t>(c->sh_src),
                    dp<uint32_t>(c->sh_netns), dp<uint8_t>(c->sh_flags), dp<uint32_t>(c->st_len),
                    dp<uint32_t>(c->st_base), dp<uint8_t>(c->st_mode), dp<uint32_t>(c->st_rlen),
                    dp<uint32_t>(c->st_rbase), dp<uint32_t>(c->dl_rows), misc + MISC_ROWCHG_N,
                    dp<uint32_t>(c->st_seen), misc + MISC_DELTA_ERR};
    if (Tn) k_delta_plan<<<nblocks(Tn), BLOCK, 0, s>>>(pi, po);
    // the new desired store: kept segments and previous-record references now (grid over the
    // bound, the exact count stays on the device), the inline records once they have arrived
    TRY(scan_lengths(c, c->st_len, Tn, c->st_off64, c->st_part, c->st_off32));
    const AsmGuard g{misc + MISC_DELTA_ERR, dp<uint64_t>(c->st_off64) + Tn, 1u, 1u};
    if (nbound)
        k_store_assemble<<<nblocks(nbound), BLOCK, 0, s>>>(dp<uint32_t>(c->st_off32), Tn, dp<uint32_t>(c->st_base),
                                                           dp<uint8_t>(c->st_mode), p_ref, c->des.view,
                                                           c->dl_rec.view, (uint32_t)nbound, g,
                                                           dp<uint32_t>(c->sh_des.buf));
    if (remap) {                                    // kept Topologies' status segments move with them
        TRY(scan_lengths(c, c->st_rlen, Tn, c->st_roff64, c->st_rpart, c->st_roff32));
        const AsmGuard gr{misc + MISC_DELTA_ERR, dp<uint64_t>(c->st_roff64) + Tn, 0u, 0u};
        if (M0)
            k_store_assemble<<<nblocks(M0), BLOCK, 0, s>>>(dp<uint32_t>(c->st_roff32), Tn, dp<uint32_t>(c->st_rbase),
                                                           dp<uint8_t>(c->st_mask), nullptr, c->real.view, c->real.view,
                                                           M0, gr, dp<uint32_t>(c->sh_real.buf));
    }
    // the references once they have arrived: checked, previous records copied to their places,
    // the inline records' destinations noted (before the records themselves have arrived)
    if (cs != s) HIP_TRY(hipStreamWaitEvent(s, c->ev_cp[2], 0));
    if (nref) {
        DeltaCheckIn c2 = ci;
        c2.n = 0;
        c2.kd_keep = c2.pd_keep = 0;                   // (checked above)
        k_delta_check<<<std::min<uint32_t>(nblocks(nref), 4 * c->n_cus), BLOCK, 0, s>>>(c2, misc + MISC_DELTA_ERR);
        k_delta_refs<<<nblocks(nref), BLOCK, 0, s>>>(p_off, p_topo, n, p_ref, nref, dp<uint32_t>(c->st_off32),
                                                     c->des.view, misc + MISC_DELTA_ERR, dp<uint32_t>(c->dl_dest),
                                                     misc + MISC_DELTA_MULTI, dp<uint32_t>(c->sh_des.buf));
    }
    // staging columns straight to their places as each copy arrives, with the id-range maxima
    const uint32_t place_grid = std::min<uint32_t>(nblocks(nr), 4 * c->n_cus);
    for (int k = 0; nr && k <= nseg; ++k) {
        if (cs != s) HIP_TRY(hipStreamWaitEvent(s, c->ev_col[k], 0));
        const bool uid_seg = k == nseg;
        k_delta_place<<<place_grid, BLOCK, 0, s>>>(
            reinterpret_cast<const uint32_t*>(st), reinterpret_cast<const int64_t*>(st + uid_at), nr,
            dp<uint32_t>(c->dl_dest), misc + MISC_DELTA_ERR, dp<uint32_t>(c->sh_des.buf), colmax,
            uid_seg ? (uint32_t)LINK_COLS32 : segs[k][0], uid_seg ? (uint32_t)LINK_COLS32 : segs[k][1], uid_seg ? 1u : 0u);
    }
    if (cs != s) HIP_TRY(hipStreamWaitEvent(s, c->ev_cp[3], 0));
    k_delta_totals<<<1, 64, 0, s>>>(dp<uint64_t>(c->st_off64), Tn, remap ? dp<uint64_t>(c->st_roff64) : nullptr, misc);
    HIP_TRY(hipGetLastError());
    uint32_t* hm = c->h_misc + 64;
    HIP_TRY(hipMemcpyAsync(hm, misc, 64 * 4, hipMemcpyDeviceToHost, s));
    HIP_TRY(hipStreamSynchronize(s));              // the call's one synchronisation
    uint32_t err = hm[MISC_DELTA_ERR];
    if (d->records.n)
        for (int k = 0; k < COL_GAP; ++k)
            if (hm[MISC_COLMAX + k] >= (k < KDTN_NKEY ? D : P)) err |= DERR_COLS;
    if (err) {
        static const char* what[] = {"topo not strictly ascending below n_topos", "des_off not monotone",
                                     "spec nil but records", "status / name id out of range", "ref out of range",
                                     "prev: index out of range or named twice", "a created topology has no spec",
                                     "kept dictionary prefix differs from the resident one",
                                     "inline record id out of range"};
        int b = 0;
        while (!(err & (1u << b))) ++b;
        bad(what[b], err);
        state_changed(c);
        // nothing resident was replaced: the dictionaries only wrote past the resident strings
        // (unless their kept prefix itself disagreed), so their sizes go back and a corrected
        // delta can follow; the next run re-parses the previous upload's suffix
        c->D = saved[0], c->P = saved[1], c->kd_valid = saved[2], c->pd_valid = saved[3];
        c->kd_from = saved[4], c->pd_from = saved[5];
        c->kd_arena = saved_arena[0], c->pd_arena = saved_arena[1];
        c->uploaded = !(err & DERR_KEEP);
        if (err & DERR_KEEP) {                     // the resident strings themselves are suspect
            c->kd_valid = c->pd_valid = c->si_k = c->si_p = 0;
            c->ix_k.n = c->ix_k.mask = 0;
            c->ix_p.n = c->ix_p.mask = 0;
        }
        return KDTN_EINVAL;
    }
    if (hm[MISC_DELTA_MULTI]) {
        // an inline record referenced more than once: the staged delta's tiles, then every
        // reference placed from them (rare; one more synchronisation)
        k_soa_to_tiles<<<std::min<uint32_t>(nblocks(nr), 4 * c->n_cus), BLOCK, 0, s>>>(
            reinterpret_cast<const uint32_t*>(st), reinterpret_cast<const int64_t*>(st + uid_at), nr,
            dp<uint32_t>(c->dl_rec.buf), colmax);
        k_delta_inline<<<nblocks(nref), BLOCK, 0, s>>>(p_off, p_topo, n,
                                                       p_ref, nref, dp<uint32_t>(c->st_off32),
                                                       c->dl_rec.view, misc + MISC_DELTA_ERR,
                                                       dp<uint32_t>(c->sh_des.buf));
        HIP_TRY(hipGetLastError());
        HIP_TRY(hipStreamSynchronize(s));
    }
    const uint64_t N = (uint64_t)hm[MISC_DELTA_N] | ((uint64_t)hm[MISC_DELTA_N + 1] << 32);
    std::swap(c->des, c->sh_des);
    c->des.n = c->des.view.n = (uint32_t)N;
    std::swap(c->t_noff, c->st_off32);
    std::swap(c->t_src, c->sh_src);
    std::swap(c->t_netns, c->sh_netns);
    std::swap(c->t_flags, c->sh_flags);
    if (remap) {
        const uint64_t M = (uint64_t)hm[MISC_DELTA_M] | ((uint64_t)hm[MISC_DELTA_M + 1] << 32);
        std::swap(c->real, c->sh_real);
        c->real.n = c->real.view.n = (uint32_t)M;
        std::swap(c->t_roff, c->st_roff32);
        std::swap(c->t_ns, c->sh_ns);
        std::swap(c->t_name, c->sh_name);
        c->T = Tn;
    }
    TRY(prepare_vnis(c, d->vnis));
    TRY(prepare_work(c, slice, c->real.n, c->des.n));
    if (remap) {                                    // rows moved: the next run builds the pod tables
        c->pods_ready = false;
        c->pods_delta = false;
    } else {
        TRY(patch_pods(c, hm[MISC_ROWCHG_N]));
    }
    if (d->vnis.n && d->vnis.n != KDTN_VNI_RESIDENT)
        HIP_TRY(hipStreamSynchronize(s));          // the snapshot's host arrays may be released after return
    state_changed(c);
    c->pods_imported = false;
    c->uploaded = true;
    drain.armed = false;
    return KDTN_OK;
}

int kdtn_epoch_tables_info(kdtn_ctx* c, kdtn_ingest_info* info) {
    if (!c || !c->uploaded) return KDTN_EINVAL;
    kdtn_ingest_info& I = c->j_info;             // host-known sizes: no device access
    I = kdtn_ingest_info{};
    I.n_topos = c->T;
    I.n_desired = c->des.n;
    I.n_realised = c->real.n;
    I.n_kdict = c->D;
    I.n_pdict = c->P;
    I.kdict_bytes = c->kd_arena;
    I.pdict_bytes = c->pd_arena;
    c->tables_cur = true;
    if (info) *info = I;
    return KDTN_OK;
}

}  // extern "C"

// ======================================================================================
// Incremental CR ingest on the resident state (kdtn_informer.hip kernels)
// ======================================================================================
namespace {

// The resident string index of one dictionary (bytes / offs, D strings) brought up to date:
// extended with the strings appended since it was built, rebuilt (twice the capacity) when it
// would pass half full with `extra` more strings, or when the dictionary was rewritten.
int strix_update(kdtn_ctx* c, kdtn_ctx::StrIndex& ix, DevBuf& bytes, DevBuf& offs, uint32_t D, uint32_t extra) {
    hipStream_t s = c->stream;
    const uint64_t want = next_pow2(2ull * ((uint64_t)D + extra) + 64);
    uint32_t from = ix.n;
    if (ix.n > D || !ix.slots.p || !ix.mask || (uint64_t)ix.mask + 1 < want) {
        const uint64_t cap = std::max<uint64_t>(want, (uint64_t)ix.mask + 1);
        if (cap > (1ull << 31)) {
            std::snprintf(g_last_error, sizeof(g_last_error), "string index of %llu slots", (unsigned long long)cap);
            return KDTN_ENOMEM;
        }
        TRY(ensure(ix.slots, (size_t)cap * 8));
        HIP_TRY(hipMemsetAsync(ix.slots.p, 0, (size_t)cap * 8, s));
        ix.mask = (uint32_t)cap - 1;
        from = 0;
    }
    if (D > from)
        k_strix_insert<<<nblocks(D - from), BLOCK, 0, s>>>(dp<uint8_t>(bytes), dp<uint32_t>(offs), from, D,
                                                             dp<unsigned long long>(ix.slots), ix.mask);
    ix.n = D;
    return KDTN_OK;
}

// Local (document) strings → resident ids; misses ranked (new ids) and sized (arena offsets)
int strix_lookup(kdtn_ctx* c, kdtn_ctx::StrIndex& ix, DevBuf& lb, DevBuf& lo, uint32_t nl, DevBuf& rb,
                 DevBuf& ro, DevBuf& map, DevBuf& rank, DevBuf& boff) {
    hipStream_t s = c->stream;
    TRY(ensure(map, (size_t)nl * 4));
    TRY(ensure(c->ji_miss, (size_t)nl * 4));
    TRY(ensure(c->ji_mlen, (size_t)nl * 4));
    TRY(ensure(rank, ((size_t)nl + 1) * 8));
    TRY(ensure(boff, ((size_t)nl + 1) * 8));
    if (nl)
        k_strix_lookup<<<nblocks(nl), BLOCK, 0, s>>>(dp<uint8_t>(lb), dp<uint32_t>(lo), nl, dp<uint8_t>(rb),
                                                     dp<uint32_t>(ro), dp<unsigned long long>(ix.slots), ix.mask,
                                                     dp<uint32_t>(map), dp<uint32_t>(c->ji_miss),
                                                     dp<uint32_t>(c->ji_mlen));
    TRY(scan_u32(c, dp<uint32_t>(c->ji_miss), nl, dp<uint64_t>(rank)));
    TRY(scan_u32(c, dp<uint32_t>(c->ji_mlen), nl, dp<uint64_t>(boff)));
    return KDTN_OK;
}

}  // namespace

extern "C" {

// Incremental CR ingest (include/kdtn.h): the informer's added / updated Topology CRs as a
// TopologyList document decoded into scratch tables, interned into the resident dictionaries,
// matched to the resident rows by (namespace, name), and applied as a delta.
int kdtn_json_ingest_delta(kdtn_ctx* c, const uint32_t* deleted, uint32_t n_deleted, const kdtn_vni_table* vnis,
                           kdtn_ingest_info* info) {
    if (!c || !c->j_loaded || !c->uploaded || (n_deleted && !deleted)) return KDTN_EINVAL;
    HIP_TRY(hipSetDevice(c->device));
    end_shard_ingest(c);
    g_last_error[0] = 0;
    if (c->nranks > 1) {
        std::snprintf(g_last_error, sizeof(g_last_error), "kdtn_json_ingest_delta: single-shard contexts");
        return KDTN_EINVAL;
    }
    if (c->kd_valid < c->D || c->pd_valid < c->P) {
        std::snprintf(g_last_error, sizeof(g_last_error),
                      "kdtn_json_ingest_delta: the resident dictionaries were not parsed (run the epoch first)");
        return KDTN_EINVAL;
    }
    const kdtn_vni_table resident{KDTN_VNI_RESIDENT, nullptr, nullptr, nullptr};
    const kdtn_vni_table& vn = vnis ? *vnis : resident;
    hipStream_t s = c->stream;
    const uint32_t T0 = c->T, N0 = c->des.n, M0 = c->real.n, D0 = c->D, P0 = c->P;
    // 1. decode into scratch (the resident tables are untouched; a rejected document leaves them)
    const JsTargets tg{&c->ji_ns, &c->ji_name, &c->ji_src, &c->ji_netns, &c->ji_flags, &c->ji_roff, &c->ji_noff,
                       &c->ji_des, &c->ji_real, &c->ji_kb, &c->ji_ko, &c->ji_pb, &c->ji_po};
    JsCounts k{};
    {
        const int rc = json_decode(c, tg, &k, info);
        c->uploaded = true;                          // (json_reject clears it: the state stands)
        if (rc != KDTN_OK) return rc;
    }
    const uint32_t Tl = k.T, Nl = k.N;
    const uint64_t n_tokens = c->j_info.n_tokens;
    // 2. intern the document's strings into the resident dictionaries
    TRY(strix_update(c, c->ix_k, c->kd_bytes, c->kd_offs, D0, k.D));
    TRY(strix_update(c, c->ix_p, c->pd_bytes, c->pd_offs, P0, k.P));
    TRY(strix_lookup(c, c->ix_k, c->ji_kb, c->ji_ko, k.D, c->kd_bytes, c->kd_offs, c->ji_kmap, c->ji_rank, c->ji_boff));
    uint64_t cnt[4] = {0, 0, 0, 0};                  // new key strings, their bytes, new prop strings, bytes
    TRY(d2h(c, cnt, dp<uint64_t>(c->ji_rank) + k.D));
    TRY(d2h(c, cnt + 1, dp<uint64_t>(c->ji_boff) + k.D));
    HIP_TRY(hipStreamSynchronize(s));
    const uint64_t D1w = (uint64_t)D0 + cnt[0];
    const uint64_t kar1 = c->kd_arena + cnt[1];
    // offsets are u32 (arena0 + boff): bounded before anything is appended
    if (kar1 > 0xFFFFFF00ull || D1w >= 0x7FFFFFFFull) {
        std::snprintf(g_last_error, sizeof(g_last_error), "kdtn_json_ingest_delta: key dictionary over 4 GiB / 2^31");
        return KDTN_EINVAL;
    }
    const uint32_t D1 = (uint32_t)D1w;
    TRY(ensure_keep(c->kd_bytes, kar1 + 64, c->kd_arena, s));
    TRY(ensure_keep(c->kd_offs, ((size_t)D1 + 1) * 4, ((size_t)D0 + 1) * 4, s));
    if (k.D)
        k_strix_append<<<nblocks(k.D), BLOCK, 0, s>>>(dp<uint8_t>(c->ji_kb), dp<uint32_t>(c->ji_ko), k.D,
                                                      dp<uint64_t>(c->ji_rank), dp<uint64_t>(c->ji_boff), D0,
                                                      (uint32_t)c->kd_arena, dp<uint32_t>(c->ji_kmap),
                                                      dp<uint8_t>(c->kd_bytes), dp<uint32_t>(c->kd_offs));
    // (the rank / offset scratch is reused for the property dictionary after the key append)
    TRY(strix_lookup(c, c->ix_p, c->ji_pb, c->ji_po, k.P, c->pd_bytes, c->pd_offs, c->ji_pmap, c->ji_kpos, c->ji_cpos));
    TRY(d2h(c, cnt + 2, dp<uint64_t>(c->ji_kpos) + k.P));
    TRY(d2h(c, cnt + 3, dp<uint64_t>(c->ji_cpos) + k.P));
    HIP_TRY(hipStreamSynchronize(s));
    const uint64_t P1w = (uint64_t)P0 + cnt[2];
    const uint64_t par1 = c->pd_arena + cnt[3];
    const uint32_t P1 = (uint32_t)P1w;
    if (par1 > 0xFFFFFF00ull || P1w >= 0x7FFFFFFFull) {
        std::snprintf(g_last_error, sizeof(g_last_error), "kdtn_json_ingest_delta: dictionaries over 4 GiB / 2^31");
        return KDTN_EINVAL;
    }
    TRY(ensure_keep(c->pd_bytes, par1 + 64, c->pd_arena, s));
    TRY(ensure_keep(c->pd_offs, ((size_t)P1 + 1) * 4, ((size_t)P0 + 1) * 4, s));
    if (k.P)
        k_strix_append<<<nblocks(k.P), BLOCK, 0, s>>>(dp<uint8_t>(c->ji_pb), dp<uint32_t>(c->ji_po), k.P,
                                                      dp<uint64_t>(c->ji_kpos), dp<uint64_t>(c->ji_cpos), P0,
                                                      (uint32_t)c->pd_arena, dp<uint32_t>(c->ji_pmap),
                                                      dp<uint8_t>(c->pd_bytes), dp<uint32_t>(c->pd_offs));
    // the appended strings join the indexes
    if (D1 > D0)
        k_strix_insert<<<nblocks(D1 - D0), BLOCK, 0, s>>>(dp<uint8_t>(c->kd_bytes), dp<uint32_t>(c->kd_offs), D0, D1,
                                                          dp<unsigned long long>(c->ix_k.slots), c->ix_k.mask);
    if (P1 > P0)
        k_strix_insert<<<nblocks(P1 - P0), BLOCK, 0, s>>>(dp<uint8_t>(c->pd_bytes), dp<uint32_t>(c->pd_offs), P0, P1,
                                                          dp<unsigned long long>(c->ix_p.slots), c->ix_p.mask);
    c->ix_k.n = D1;
    c->ix_p.n = P1;
    // 3. the document's tables in resident ids
    TRY(ensure(c->ji_nil, (size_t)Tl + 16));
    if (Tl)
        k_ix_map_topos<<<nblocks(Tl), BLOCK, 0, s>>>(dp<uint32_t>(c->ji_ns), dp<uint32_t>(c->ji_name),
                                                     dp<uint32_t>(c->ji_src), dp<uint32_t>(c->ji_netns),
                                                     dp<uint8_t>(c->ji_flags), Tl, dp<uint32_t>(c->ji_kmap),
                                                     dp<uint8_t>(c->ji_nil));
    constexpr uint32_t IDW = (KDTN_NKEY + KDTN_NPROP) * TILE_RECS;
    if (Nl)
        k_ix_map_links<<<nblocks((uint64_t)(Nl + TILE_RECS - 1) / TILE_RECS * IDW), BLOCK, 0, s>>>(
            dp<uint32_t>(c->ji_des.buf), Nl, dp<uint32_t>(c->ji_kmap), dp<uint32_t>(c->ji_pmap));
    // 4. the document's Topologies against the resident rows; the deletions; the new table
    const uint64_t kcap = next_pow2(2ull * T0 + 64);
    TRY(ensure(c->ji_keys, (size_t)kcap * 8));
    TRY(ensure(c->ji_vals, (size_t)kcap * 4));
    const uint64_t dcap = next_pow2(2ull * Tl + 64);
    TRY(ensure(c->ji_dkeys, (size_t)dcap * 8));
    TRY(ensure(c->ji_keep, (size_t)T0 * 4 + 16));
    TRY(ensure(c->ji_kpos, ((size_t)T0 + 1) * 8));
    TRY(ensure(c->ji_claim, (size_t)T0 * 4 + 16));
    TRY(ensure(c->ji_res, (size_t)Tl * 4 + 16));
    TRY(ensure(c->ji_created, (size_t)Tl * 4 + 16));
    TRY(ensure(c->ji_cpos, ((size_t)Tl + 1) * 8));
    TRY(ensure(c->misc, 256));
    uint32_t* misc = dp<uint32_t>(c->misc);
    HIP_TRY(hipMemsetAsync(misc + MISC_DELTA_ERR, 0, 4, s));
    HIP_TRY(hipMemsetAsync(c->ji_keys.p, 0, (size_t)kcap * 8, s));
    HIP_TRY(hipMemsetAsync(c->ji_vals.p, 0xFF, (size_t)kcap * 4, s));
    HIP_TRY(hipMemsetAsync(c->ji_dkeys.p, 0, (size_t)dcap * 8, s));
    HIP_TRY(hipMemsetAsync(c->ji_claim.p, 0xFF, (size_t)T0 * 4 + 16, s));
    if (T0) HIP_TRY(hipMemsetD32Async(reinterpret_cast<hipDeviceptr_t>(c->ji_keep.p), 1, T0, s));
    if (T0)
        k_topokey_insert<<<nblocks(T0), BLOCK, 0, s>>>(dp<uint32_t>(c->t_ns), dp<uint32_t>(c->t_name), T0,
                                                       dp<unsigned long long>(c->ji_keys), dp<uint32_t>(c->ji_vals),
                                                       (uint32_t)kcap - 1);
    if (n_deleted) {
        TRY(upload(c, c->ji_del, deleted, (size_t)n_deleted * 4));
        k_topo_delete<<<nblocks(n_deleted), BLOCK, 0, s>>>(dp<uint32_t>(c->ji_del), n_deleted, T0,
                                                           dp<uint32_t>(c->ji_keep), misc + MISC_DELTA_ERR);
    }
    if (Tl)
        k_topokey_match<<<nblocks(Tl), BLOCK, 0, s>>>(dp<uint32_t>(c->ji_ns), dp<uint32_t>(c->ji_name), Tl,
                                                      dp<unsigned long long>(c->ji_keys), dp<uint32_t>(c->ji_vals),
                                                      (uint32_t)kcap - 1, dp<unsigned long long>(c->ji_dkeys),
                                                      (uint32_t)dcap - 1, dp<uint32_t>(c->ji_keep),
                                                      dp<uint32_t>(c->ji_claim), dp<uint32_t>(c->ji_res),
                                                      dp<uint32_t>(c->ji_created), misc + MISC_DELTA_ERR);
    TRY(scan_u32(c, dp<uint32_t>(c->ji_keep), T0, dp<uint64_t>(c->ji_kpos)));
    TRY(scan_u32(c, dp<uint32_t>(c->ji_created), Tl, dp<uint64_t>(c->ji_cpos)));
    uint64_t tot[2] = {0, 0};
    uint32_t err = 0;
    TRY(d2h(c, tot, dp<uint64_t>(c->ji_kpos) + T0));
    TRY(d2h(c, tot + 1, dp<uint64_t>(c->ji_cpos) + Tl));
    TRY(d2h(c, &err, misc + MISC_DELTA_ERR));
    HIP_TRY(hipStreamSynchronize(s));
    HIP_TRY(hipGetLastError());
    auto refuse = [&](const char* what) {
        // the dictionaries only grew past the resident strings: their sizes stay, the arena
        // tails are overwritten later, and the indexes (which hold the appended strings) are
        // rebuilt by the next incremental ingest (mask 0)
        c->ix_k.n = c->ix_k.mask = c->ix_p.n = c->ix_p.mask = 0;
        std::snprintf(g_last_error, sizeof(g_last_error), "kdtn_json_ingest_delta: %s", what);
        state_changed(c);
        return KDTN_EINVAL;
    };
    if (err & 4u) return refuse("a deleted index is out of range");
    if (err & 1u) return refuse("a Topology is both deleted and listed in the document");
    if (err & 2u) return refuse("a Topology is listed twice in the document");
    const uint32_t n_kept = (uint32_t)tot[0], n_created = (uint32_t)tot[1], Tn = n_kept + n_created;
    const bool remap = n_kept != T0 || n_created;
    // 5. the delta: the document's Topologies are the changed list (row l: spec from its
    // records, all inline), laid out over the new table
    TRY(plan_alloc(c, Tn));
    TRY(ensure(c->st_chg, (size_t)Tn * 4 + 16));
    HIP_TRY(hipMemsetAsync(c->st_chg.p, 0xFF, (size_t)Tn * 4 + 16, s));
    if (remap) TRY(ensure(c->dl_prev, (size_t)Tn * 4 + 16));
    const uint32_t nl = std::max(T0, Tl);
    if (nl)
        k_ix_layout<<<nblocks(nl), BLOCK, 0, s>>>(dp<uint32_t>(c->ji_keep), dp<uint64_t>(c->ji_kpos), T0,
                                                  dp<uint32_t>(c->ji_claim), dp<uint32_t>(c->ji_created),
                                                  dp<uint64_t>(c->ji_cpos), Tl, n_kept,
                                                  remap ? dp<uint32_t>(c->dl_prev) : nullptr, dp<uint32_t>(c->st_chg));
    TRY(ensure(c->ji_ref, (size_t)Nl * 4 + 16));
    if (Nl) k_ix_refs<<<nblocks(Nl), BLOCK, 0, s>>>(dp<uint32_t>(c->ji_ref), Nl);
    TRY(ensure(c->dl_rows, (size_t)Tl * 4 + 16));
    TRY(ensure(c->sh_src, (size_t)Tn * 4));
    TRY(ensure(c->sh_netns, (size_t)Tn * 4));
    TRY(ensure(c->sh_flags, (size_t)Tn));
    if (remap) {
        TRY(ensure(c->sh_ns, (size_t)Tn * 4));
        TRY(ensure(c->sh_name, (size_t)Tn * 4));
        TRY(ensure(c->st_rlen, (size_t)Tn * 4 + 16));
        TRY(ensure(c->st_rbase, (size_t)Tn * 4 + 16));
        TRY(ensure(c->st_mask, (size_t)Tn + 16));
        TRY(ensure(c->st_seen, ((size_t)T0 + 31) / 32 * 4 + 16));
        HIP_TRY(hipMemsetAsync(c->st_seen.p, 0, ((size_t)T0 + 31) / 32 * 4 + 16, s));
        HIP_TRY(hipMemsetAsync(c->st_mask.p, ASM_SEG_A, (size_t)Tn + 16, s));
    }
    HIP_TRY(hipMemsetAsync(misc + MISC_ROWCHG_N, 0, 4, s));
    const uint64_t nbound = (uint64_t)N0 + Nl;
    if (nbound >= 0x7FFFFFFFull) return refuse("desired store over 2^31 records");
    TRY(link_store_alloc(c, c->sh_des, (uint32_t)nbound));
    if (remap) TRY(link_store_alloc(c, c->sh_real, M0));
    DeltaPlanIn pi{topo_view(c), dp<uint32_t>(c->st_chg), remap ? dp<uint32_t>(c->dl_prev) : nullptr,
                   dp<uint32_t>(c->ji_noff), dp<uint32_t>(c->ji_src), dp<uint32_t>(c->ji_netns), dp<uint8_t>(c->ji_nil),
                   dp<uint32_t>(c->ji_ns), dp<uint32_t>(c->ji_name), Tn, D1};
    DeltaPlanOut po{dp<uint32_t>(c->sh_ns), dp<uint32_t>(c->sh_name), dp<uint32_t>(c->sh_src),
                    dp<uint32_t>(c->sh_netns), dp<uint8_t>(c->sh_flags), dp<uint32_t>(c->st_len),
                    dp<uint32_t>(c->st_base), dp<uint8_t>(c->st_mode), dp<uint32_t>(c->st_rlen),
                    dp<uint32_t>(c->st_rbase), dp<uint32_t>(c->dl_rows), misc + MISC_ROWCHG_N,
                    dp<uint32_t>(c->st_seen), misc + MISC_DELTA_ERR};
    if (Tn) k_delta_plan<<<nblocks(Tn), BLOCK, 0, s>>>(pi, po);
    TRY(scan_lengths(c, c->st_len, Tn, c->st_off64, c->st_part, c->st_off32));
    const AsmGuard g{misc + MISC_DELTA_ERR, dp<uint64_t>(c->st_off64) + Tn, 0u};
    if (nbound)
        k_store_assemble<<<nblocks(nbound), BLOCK, 0, s>>>(dp<uint32_t>(c->st_off32), Tn, dp<uint32_t>(c->st_base),
                                                           dp<uint8_t>(c->st_mode), dp<uint32_t>(c->ji_ref), c->des.view,
                                                           c->ji_des.view, (uint32_t)nbound, g,
                                                           dp<uint32_t>(c->sh_des.buf));
    if (remap) {
        TRY(scan_lengths(c, c->st_rlen, Tn, c->st_roff64, c->st_rpart, c->st_roff32));
        const AsmGuard gr{misc + MISC_DELTA_ERR, dp<uint64_t>(c->st_roff64) + Tn, 0u};
        if (M0)
            k_store_assemble<<<nblocks(M0), BLOCK, 0, s>>>(dp<uint32_t>(c->st_roff32), Tn, dp<uint32_t>(c->st_rbase),
                                                           dp<uint8_t>(c->st_mask), nullptr, c->real.view, c->real.view,
                                                           M0, gr, dp<uint32_t>(c->sh_real.buf));
    }
    k_delta_totals<<<1, 64, 0, s>>>(dp<uint64_t>(c->st_off64), Tn, remap ? dp<uint64_t>(c->st_roff64) : nullptr, misc);
    HIP_TRY(hipGetLastError());
    uint32_t* hm = c->h_misc + 64;
    HIP_TRY(hipMemcpyAsync(hm, misc, 64 * 4, hipMemcpyDeviceToHost, s));
    HIP_TRY(hipStreamSynchronize(s));
    if (hm[MISC_DELTA_ERR]) return refuse("the document's tables failed the delta checks");
    // 6. the new state
    const uint64_t N = (uint64_t)hm[MISC_DELTA_N] | ((uint64_t)hm[MISC_DELTA_N + 1] << 32);
    std::swap(c->des, c->sh_des);
    c->des.n = c->des.view.n = (uint32_t)N;
    std::swap(c->t_noff, c->st_off32);
    std::swap(c->t_src, c->sh_src);
    std::swap(c->t_netns, c->sh_netns);
    std::swap(c->t_flags, c->sh_flags);
    if (remap) {
        const uint64_t M = (uint64_t)hm[MISC_DELTA_M] | ((uint64_t)hm[MISC_DELTA_M + 1] << 32);
        std::swap(c->real, c->sh_real);
        c->real.n = c->real.view.n = (uint32_t)M;
        std::swap(c->t_roff, c->st_roff32);
        std::swap(c->t_ns, c->sh_ns);
        std::swap(c->t_name, c->sh_name);
        c->T = Tn;
    }
    // dictionaries: the appended strings are parsed by the next run (kd_from / pd_from)
    c->D = D1;
    c->P = P1;
    c->kd_arena = kar1;
    c->pd_arena = par1;
    c->kd_valid = c->kd_from = D0;
    c->pd_valid = c->pd_from = P0;
    c->si_k = std::min(c->si_k, D0);
    c->si_p = std::min(c->si_p, P0);
    TRY(prepare_dicts(c));
    TRY(check_vnis(c, vn, D1, D0));
    TRY(prepare_vnis(c, vn));
    TRY(prepare_work(c, remap ? Tn : c->slice, c->real.n, c->des.n));
    c->pods_ready = false;                         // rows changed: the next run rebuilds the pod tables
    c->pods_delta = false;
    HIP_TRY(hipStreamSynchronize(s));
    state_changed(c);
    c->pods_imported = false;
    c->uploaded = true;
    c->j_info = kdtn_ingest_info{};
    c->j_info.n_topos = c->T;
    c->j_info.n_desired = c->des.n;
    c->j_info.n_realised = c->real.n;
    c->j_info.n_kdict = D1;
    c->j_info.n_pdict = P1;
    c->j_info.n_tokens = n_tokens;
    c->j_info.kdict_bytes = kar1;
    c->j_info.pdict_bytes = par1;
    if (info) *info = c->j_info;
    return KDTN_OK;
}

}  // extern "C"
