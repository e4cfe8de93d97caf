// kdtn_kernels.h — HIP kernels of one reconcile epoch (gfx950 / CDNA4, wave64).
//
// Data layout in HBM (struct-of-arrays, records grouped by Topology):
//   link table   : ONE allocation per side in tiles of 64 records (AoSoA, see DevLinks):
//                  key[0..6] (u32 kdict ids) | prop[0..11] (u32 pdict ids) | gap (u32) | uid (i64)
//                  → 88 B per record, one base pointer per table in the kernel arguments
//   topologies   : u32 ns/name/src_ip/net_ns ids, u8 flags, u32 offsets (T+1) per side
//   dictionaries : u8 arena + u32 offsets, parsed once per epoch (one thread per string,
//                  arena slices staged through LDS) into compact lookup tables:
//                  kbits: 3 bitsets over key strings (CIDR_BAD, MAC_BAD, PHYSICAL; 1.5 MB
//                  per 12M strings, L2-resident); ppct u32 (Percentage2u32 or PCT_ERR);
//                  pdur {us, ticks, err}; prate {lo, hi, err}
//   pod table    : pods[g] = {ns, name, src_ip, net_ns|spec_nil<<31} per global pod index;
//                  lookup table of 16-B self-contained slots indexed by the name's kdict id
//                  and stamped per epoch: a lookup is ONE gather with no probing (the slot
//                  also carries the PHYSICAL bit of the name, so a hit needs no key-string
//                  flag read); names shared by several pods go through an overflow table.
// Kernels (launch order):
//   k_kdict_flags   MakeVeth / addLink predicates per key string          (D threads)
//   k_pdict_parse   ParseDuration / ParseFloatPercentage / ParseRate      (P threads)
//   k_pods_fill     this rank's pod-status slice                          (slice threads)
//   [RCCL all-gather of the pod-status table when nranks > 1]
//   k_pod_direct_scatter + k_pod_direct_verify, k_vni_pack + k_vni_ht_build
//   k_reconcile     ONE pass per workgroup of TPW topologies: Reconcile gate + CalcDiff in
//                   LDS, decoupled look-back for the batch bases, then barrier-free emission
//                   of the batch lists, addLink/delLink/UpdateLinks pure prefix, MakeQdiscs.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/kdtn.h"
#include "kdtn_parse.h"

namespace kdtn {

constexpr int BLOCK = 256;   // 4 waves of 64
constexpr int TPW = 64;      // topologies per workgroup in k_reconcile (one per lane of wave 0)
constexpr int CAP = 2048;    // LDS window capacity, records (old + new) per workgroup
constexpr int STAGE = 8192;  // LDS bytes for staged dictionary slices

constexpr uint32_t PCT_ERR = 0xFFFFFFFEu;   // Percentage2u32 never yields this value

// key-string predicates, one bitset each (bit i of word i/32 = string i)
enum : int {
    KB_CIDR_BAD = 0,    // non-empty and net.ParseCIDR fails
    KB_MAC_BAD = 1,     // non-empty and net.ParseMAC fails
    KB_PHYSICAL = 2,    // has prefix "physical/"
    KB_NSETS = 3,
};
// special key-string ids found by k_kdict_flags (0xFFFFFFFF when absent)
enum : int { SPECIAL_DEFAULT = 0, SPECIAL_LOCALHOST = 4, MISC_FAN_NODES = 12, MISC_VNI_N = 13,
             MISC_COMMIT_N = 14, MISC_ROWCHG_N = 15, MISC_COLMAX = 16 /* [19] */, MISC_DELTA_ERR = 36,
             MISC_DELTA_N = 38 /* u64 */, MISC_DELTA_M = 40 /* u64 */,
             MISC_DELTA_MULTI = 42 };   // misc words (64 = 256 B)
// epoch sync header (u32 words; zeroed by the epoch's only memset, the look-back status
// follows at SYNC_HEADER_BYTES). The ticket counter, which every k_reconcile workgroup
// increments, has a 128-B line to itself; the host reads words [SYNC_TOTALS, SYNC_TOTALS + 4)
// (totals, look-back error) back with one copy.
enum : int { SYNC_TICKET = 0, SYNC_TOTALS = 32 /* [3] del, upd, add */, SYNC_ERR = 35,
             SYNC_FIRST_PARTIAL_INV = 36 /* ~first partial chunk: 0 = none */, SYNC_HEADER_BYTES = 256 };
// pod slot flag bits (in the g word of a wide slot; pod indices < 2^30)
constexpr uint32_t POD_SPEC_NIL = 0x80000000u, POD_PHYSICAL = 0x40000000u, POD_INDEX = 0x3FFFFFFFu;

// record flags
enum : uint8_t { RF_DEL = 1, RF_UPD = 2, RF_ADD = 4, RF_MATCHED = 0x80 };   // MATCHED: CalcDiff scratch

// Link store: tiles of 64 records (AoSoA). A tile holds, for its 64 records, each u32 column
// as 256 contiguous bytes (key[0..6], prop[0..11], gap) followed by the i64 uid column
// (512 B): 5,632 B per tile. A wave's column load is one 256-B run, and every column of a
// record is a fixed immediate offset from one per-record pointer (no per-column base
// registers).
enum { COL_KEY0 = 0, COL_PROP0 = KDTN_NKEY, COL_GAP = KDTN_NKEY + KDTN_NPROP, COL_UID = COL_GAP + 1 };
constexpr int LINK_COLS32 = COL_UID;               // u32 columns before the i64 uid column
constexpr int TILE_RECS = 64;
constexpr int TILE_WORDS = (LINK_COLS32 + 2) * TILE_RECS;   // 1,408 u32 = 5,632 B

struct DevLinks {
    const uint32_t* base;   // tile t at base + t*TILE_WORDS
    uint32_t n;
    // word 0 of record i's tile row: column c of record i at rec(i)[c*64]
    __device__ __forceinline__ const uint32_t* rec(uint32_t i) const {
        return base + (size_t)(i >> 6) * TILE_WORDS + (i & 63u);
    }
    template <bool NT> __device__ __forceinline__ uint32_t col(const uint32_t* r, int c) const {
        if constexpr (NT) return __builtin_nontemporal_load(r + c * TILE_RECS);
        else return r[c * TILE_RECS];
    }
    template <bool NT> __device__ __forceinline__ int64_t uid_at(const uint32_t* r, uint32_t i) const {
        const int64_t* p = reinterpret_cast<const int64_t*>(r - (i & 63u) + COL_UID * TILE_RECS) + (i & 63u);
        if constexpr (NT) return __builtin_nontemporal_load(p);
        else return *p;
    }
    __device__ __forceinline__ uint32_t key(int k, uint32_t i) const { return rec(i)[(COL_KEY0 + k) * TILE_RECS]; }
    __device__ __forceinline__ uint32_t prop(int k, uint32_t i) const { return rec(i)[(COL_PROP0 + k) * TILE_RECS]; }
    __device__ __forceinline__ uint32_t gap(uint32_t i) const { return rec(i)[COL_GAP * TILE_RECS]; }
    __device__ __forceinline__ int64_t uid(uint32_t i) const { return uid_at<false>(rec(i), i); }
    template <bool NT> __device__ __forceinline__ uint32_t key_s(int k, uint32_t i) const {
        return col<NT>(rec(i), COL_KEY0 + k);
    }
    template <bool NT> __device__ __forceinline__ uint32_t prop_s(int k, uint32_t i) const {
        return col<NT>(rec(i), COL_PROP0 + k);
    }
    template <bool NT> __device__ __forceinline__ uint32_t gap_s(uint32_t i) const {
        return col<NT>(rec(i), COL_GAP);
    }
    template <bool NT> __device__ __forceinline__ int64_t uid_s(uint32_t i) const {
        return uid_at<NT>(rec(i), i);
    }
};

// Profiling build (make -C kube-dtn_amd prof → prof/libkdtn_prof.so, -DKDTN_PROFILING=1):
// the A/B variants below are instantiated and selected from KDTN_VARIANT / KDTN_KD_SUB /
// KDTN_JS_VARIANT. The product library (kdtn/libkdtn.so) compiles only DEFAULT_VARIANT and
// the parity-tested paths, and reads no environment variable.
#ifndef KDTN_PROFILING
#define KDTN_PROFILING 0
#endif
// epoch front: the pod lookup build (scatter, verify + full-prefix scan) on a side stream (the
// comm stream after the all-gather when RCCL exchanges the rows) beside the dictionary parses
#ifndef KDTN_LOOKUP_SIDE_DEFAULT
#define KDTN_LOOKUP_SIDE_DEFAULT 0
#endif
// epoch front: k_kdict_flags and k_pdict_parse as one launch (k_dict_parse)
#ifndef KDTN_DICT_FUSE_DEFAULT
#define KDTN_DICT_FUSE_DEFAULT false    // A/B in one process: N = 1 0.797 vs 0.811 ms, N = 8 0.183 vs 0.185 (r05e)
#endif
// k_pdict_parse: one thread per (string, interpretation) instead of one per string
#ifndef KDTN_PD_SPLIT_DEFAULT
#define KDTN_PD_SPLIT_DEFAULT true    // 125k-pod config 2: 0.0374 -> 0.0341 ms; 1M: equal
#endif
// Emission variants (A/B in the profiling build; the product runs DEFAULT_VARIANT):
//   bit 0: non-temporal streaming loads of link columns
//   bit 1: non-temporal output stores
//   bit 2: (profiling) compute MakeQdiscs but do not store it
//   bit 3: non-temporal pod-slot gathers
//   bit 4: (profiling) per-workgroup phase timestamps into RecWork::trace
//   bits 5, 6: (profiling, wrong results) skip the pod-slot / percentage-table gathers
//   bits 7, 8: occupancy target of 5 / 6 waves per SIMD (register budget 96 / 80 VGPRs)
//   bit 9: parsed-table gathers only for non-empty property ids (id 0 = "" parses to 0)
//   bit 10: (A/B) always run the look-back, ignoring k_full_prefix
//   bit 11: comparison-heavy build (product): CalcDiff windows dominate (realised lists are
//           non-empty), so the bulk emission is not software-pipelined and the kernel
//           targets DIFF_WAVES waves per SIMD; kdtn_epoch_run picks it when M > 0 and N > 0
//   bit 12: (A/B) bulk loop: the next record's segment search before this record's gathers
//   bit 15: (A/B) bulk emission stages the wave's 64 qdisc structs at once and stores them with
//           16-B stores (about half the store instructions of two 32-struct halves of 8-B stores)
//   bit 14: first bulk record's columns loaded before the gate / count / base phases (product;
//           A/B vs 515: 0.6164 / 0.6180 ms at 1M pods, 0.0849 / 0.0869 at 125k, 0.1563 / 0.1583 config 4)
//   bit 16: bulk emission by LDS-DMA: each wave copies whole 64-record tiles of the link store
//           (the 20 of 22 column units an entry reads, 1 KiB per global_load_lds_dwordx4) into its
//           LDS slot and reads its record's columns there; the next tile's copy is issued behind
//           this record's gathers
constexpr int VAR_NT_LOAD = 1, VAR_NT_STORE = 2, VAR_NO_QSTORE = 4, VAR_NT_POD = 8, VAR_TRACE = 16,
              VAR_SKIP_POD = 32, VAR_SKIP_PCT = 64, VAR_OCC5 = 128, VAR_OCC6 = 256,
              VAR_MASK_EMPTY = 512, VAR_NO_PREFIX = 1024, VAR_DIFF = 2048, VAR_DECODE_FIRST = 4096, VAR_PREFETCH = 16384,
              VAR_Q16 = 32768, VAR_GLDS = 65536,
              VAR_PMAC_COLS = 131072,    // (internal to VAR_GLDS) the entry's peer_mac id is in RecCols
              VAR_AB = 262144,           // CalcDiff window: old + positional new records in one load phase
              VAR_SKIP_KB1 = 524288,     // (profiling, wrong results) skip the local-MAC bitset gather
              VAR_SKIP_KB3 = 1048576,    // (profiling, wrong results) skip all three bitset gathers
              VAR_HB = 2097152,          // CalcDiff window: both sides' key hashes first, one load round per old record
              VAR_POD8 = 4194304;        // (profiling, wrong results) the pod-slot gather as an 8-B load from
                                         // an 8-MB table: the footprint of a compact slot, timing only
// VAR_GLDS: the tile column units an add entry reads, in LDS order: local_ip, local_mac (key 1, 2),
// peer_ip, peer_mac, peer_pod (key 4..6), the 12 properties, gap, uid (2 units): every column of
// the tile but local_intf and peer_intf. A delete reads units 0, 1 and the uid (at units 2, 3).
constexpr int GL_UNITS = 20;
KD_INLINE int gl_col(int u) { return u < 2 ? u + 1 : u + 2; }     // add tile: LDS unit -> tile column unit
KD_INLINE int gl_col_del(int u) { return u < 2 ? u + 1 : u + 18; }   // delete tile (units 0..3)
constexpr int DIFF_WAVES = 5;
constexpr int var_waves(int v) {
    return (v & VAR_OCC6) ? 6 : (v & VAR_OCC5) ? 5 : (v & VAR_DIFF) ? DIFF_WAVES : (v & (VAR_PREFETCH | VAR_GLDS)) ? 4 : 1;
}
constexpr int TRACE_WORDS = 8;   // entry, topologies loaded, counts done, bases known, end, hw ids,
                                  // CalcDiff window phase A done, phase B done (fast path)
constexpr int DEFAULT_VARIANT = VAR_NT_LOAD | VAR_NT_STORE | VAR_MASK_EMPTY | VAR_PREFETCH;   // 16899
// the comparison-heavy build kdtn_epoch_run launches when both link lists are non-empty; its
// CalcDiff windows hash both sides' keys first (VAR_HB: 0.845 -> 0.671 ms on 5 config-3 churn
// epochs, profiles/r06q_window_hb_cfg3.json; VAR_AB measured and not kept, r06d)
constexpr int DIFF_VARIANT = DEFAULT_VARIANT | VAR_DIFF | VAR_HB;   // 2116099
// instantiations of the profiling build (DEFAULT_VARIANT is always instantiated): e.g. 547 / 579
// / 611 skip the pod-slot / percentage / both gathers, 519 skips the qdisc stores, 531 the
// trace build of the default
#define KDTN_PROFILING_VARIANTS(X) X(0) X(1) X(2) X(3) X(4) X(5) X(9) X(11) X(17) X(33) X(65) X(97) \
    X(101) X(113) X(129) X(257) X(513) X(521) X(523) X(529) X(531) X(545) X(547) X(579) X(611) X(519) \
    X(641) X(643) X(771) X(1025) X(1537) X(2579) X(4611) X(515) X(16915) X(16963) X(16931) X(16995) X(16903) X(49667) \
    X(66051) X(65539) X(281091) X(264723) X(541187) X(1065475) X(18947) X(2099731) X(4211203)

struct DevTopos {
    const uint32_t* ns;
    const uint32_t* name;
    const uint32_t* src_ip;
    const uint32_t* net_ns;
    const uint8_t* flags;
    const uint32_t* real_off;
    const uint32_t* des_off;
    uint32_t n;
};

struct DevTables {             // read-only lookup structures of the epoch
    const uint32_t* kbits;     // [KB_NSETS][kb_words]
    uint32_t kb_words;         // words per bitset (multiple of 2)
    const uint32_t* ppct;      // [P]
    const uint2* pdur;         // [P] {us, ticks}; DUR_ERR = {0, 1} (time2Tick(0) == 0)
    const uint2* prate;        // [P] {lo, hi}; all-ones = error or 2^64-1: see rate_err
    const uint32_t* rate_err;  // [ceil(P/64)*2] bitset: ParseRate failed
    const uint4* pods;         // [pod_total] {ns, name, src_ip, net_ns|spec_nil<<31}
    const uint4* pod_direct;   // [D] by name id: {ns, g<<2|phys<<1|spec_nil, src_ip|netns_empty<<31, stamp<<1|multi}
    uint32_t pod_stamp;        // this epoch's stamp
    const unsigned long long* pod_ovf;   // [ovf_mask+1] {stamp, pod index} of shared names, keyed by (ns, name)
    uint32_t ovf_mask;
    const uint4* vnis;         // [vni_mask+1] open-addressing slots {node, vni, net_ns, 0}, node ~0 = empty
    const uint32_t* vni_slots; // (build scratch: entry index per slot)
    uint32_t vni_mask;         // 0 ⇒ empty table
    const uint32_t* special;   // [SPECIAL_DEFAULT] "default", [SPECIAL_LOCALHOST] "localhost"
    int32_t vxlan_base;
};

struct RecOut {
    uint8_t* action;
    uint32_t* del_off;
    uint32_t* add_off;
    uint32_t* upd_off;
    uint32_t* del_idx;
    uint32_t* add_idx;
    uint32_t* upd_idx;
    uint4* del_res;            // kdtn_resolved as 16 B
    uint4* add_res;
    uint4* upd_res;
    uint2* add_qdisc;          // kdtn_qdisc as 9 × 8 B
    uint2* upd_qdisc;
    uint8_t* add_qerr;         // per add entry its qdisc error byte (kdtn_qdisc byte 70) in a dense array,
                               // with RESOLVE and QDISC: the reach rule reads it instead of the 72-B records
    uint32_t* totals;          // [3] del, upd, add
    uint32_t* htotals;         // the same [3] in page-locked host memory (no readback copy), or null
    uint32_t stages;
};

struct RecWork {
    uint32_t* sync;            // header (SYNC_*), then status at SYNC_HEADER_BYTES
    uint32_t* herr;            // page-locked host word for a look-back error, or null
    unsigned long long* status;   // [nwg*3] look-back granules: state<<32 | count
    uint32_t* hscratch;        // [M+N] window hashes of topologies larger than CAP
    uint8_t* fscratch;         // [M+N] record flags when a workgroup exceeds CAP
    uint32_t* otarget;         // [M]   first matching desired index (slow path)
    unsigned long long* trace; // [nwg][TRACE_WORDS] (VAR_TRACE only)
    const uint32_t* first_partial_inv;   // k_full_prefix: ~(first chunk not known to emit all records)
    uint32_t* wcount;          // [nwg*3] list counts per workgroup (VAR_DIFF: k_place_scan input)
    uint32_t m_cap, n_cap;     // VAR_DIFF: deferred chunks emit at m_cap + o0 / n_cap + n0
    uint32_t nwg;
    uint32_t split;            // workgroups per chunk (grid = nwg * split; 1 with VAR_TRACE)
};

// VAR_DIFF placement (after k_reconcile): exclusive bases per workgroup and list totals, then
// the deferred chunks' entries moved from the upper halves of the output arrays.
__global__ void k_place_scan(const uint32_t* wcount, uint32_t nwg, uint32_t* wbase, RecOut out, uint32_t T);
template <bool WAVE>
__global__ void k_place(DevTopos T, const uint32_t* wcount, const uint32_t* wbase, const uint32_t* first_partial_inv,
                        RecOut out, uint32_t m_cap, uint32_t n_cap, uint32_t nwg, uint32_t parts);
constexpr int PLACE_SCAN_BLOCK = 1024, PLACE_PER = 8;    // k_place_scan: workgroups per thread per tile

__global__ void k_special_clip(uint32_t* special, uint32_t k0);
template <int SUB, bool X4, int NT>
__global__ void k_kdict_flags(const uint8_t* bytes, const uint32_t* offs, uint32_t first, uint32_t n,
                              uint32_t* kbits, uint32_t kb_words, uint32_t* special);
__global__ void k_kdict_flags_ws(const uint8_t* bytes, const uint32_t* offs, uint32_t first, uint32_t n,
                                 uint32_t* kbits, uint32_t kb_words, uint32_t* special);
__global__ void k_kdict_flags_pp(const uint8_t* bytes, const uint32_t* offs, uint32_t first, uint32_t n,
                                 uint32_t* kbits, uint32_t kb_words, uint32_t* special);
__global__ void k_kdict_flags_v1(const uint8_t* bytes, const uint32_t* offs, uint32_t first, uint32_t n,
                                 uint32_t* kbits, uint32_t kb_words, uint32_t* special);
__global__ void k_kdict_null(const uint8_t* bytes, const uint32_t* offs, uint32_t first, uint32_t n,
                             uint32_t* kbits, uint32_t kb_words, uint32_t* special);
__global__ void k_kdict_loadonly(const uint8_t* bytes, const uint32_t* offs, uint32_t first, uint32_t n,
                                 uint32_t* kbits, uint32_t kb_words, uint32_t* special);
template <int WHICH>
__global__ void k_pdict_only(const uint8_t* bytes, const uint32_t* offs, uint32_t first, uint32_t n, double tick,
                             uint32_t* ppct, uint2* pdur, uint2* prate, uint32_t* rate_err);
enum : int { PD_DUR = 1, PD_PCT = 2, PD_RATE = 4, PD_RATE_GENERIC = 8 /* (A/B) no ASCII fast path */ };
template <bool SPLIT>
__global__ void k_pdict_parse(const uint8_t* bytes, const uint32_t* offs, uint32_t first, uint32_t n, double tick,
                              uint32_t* ppct, uint2* pdur, uint2* prate, uint32_t* rate_err);
__global__ void k_pods_fill(DevTopos T, uint32_t slice, uint32_t rank_base, uint4* pods);
__global__ void k_dict_parse(const uint8_t* kd_bytes, const uint32_t* kd_offs, uint32_t k0, uint32_t D, uint32_t* kbits,
                             uint32_t kb_words, uint32_t* special, const uint8_t* pd_bytes, const uint32_t* pd_offs,
                             uint32_t p0, uint32_t P, uint32_t nbp, double tick, uint32_t* ppct, uint2* pdur,
                             uint2* prate, uint32_t* rate_err, uint32_t nbk_first);
__global__ void k_dict_parse_w7(const uint8_t* kd_bytes, const uint32_t* kd_offs, uint32_t k0, uint32_t D,
                                uint32_t* kbits, uint32_t kb_words, uint32_t* special, const uint8_t* pd_bytes,
                                const uint32_t* pd_offs, uint32_t p0, uint32_t P, uint32_t nbp, double tick,
                                uint32_t* ppct, uint2* pdur, uint2* prate, uint32_t* rate_err, uint32_t nbk_first);
__global__ void k_epoch_begin(uint4* sync, uint32_t n16, uint32_t nbz, DevTopos T, uint32_t slice, uint32_t rank_base,
                              uint4* pods);
template <int PER>
__global__ void k_pod_direct_scatter(const uint4* pods, uint32_t total, const uint32_t* phys_bits,
                                     const uint8_t* kd_bytes, const uint32_t* kd_offs, uint4* slots, uint32_t stamp,
                                     uint32_t nd, uint32_t nr, uint32_t gathered);
__global__ void k_epoch_front(uint4* sync, uint32_t n16, uint32_t nbz, uint32_t nbs, DevTopos T, uint32_t slice,
                              uint4* pods, uint4* slots, uint32_t stamp, const uint8_t* kd_bytes,
                              const uint32_t* kd_offs, uint32_t k0, uint32_t D, uint32_t* kbits, uint32_t kb_words,
                              uint32_t* special);
__global__ void k_pdict_verify(const uint4* pods, uint32_t total, uint4* slots, uint32_t stamp,
                               unsigned long long* ovf, uint32_t mask, uint32_t nd, DevTopos T,
                               uint32_t* first_partial_inv, uint32_t nbv, uint32_t nbp, const uint8_t* pbytes,
                               const uint32_t* poffs, uint32_t p0, uint32_t np, uint32_t nbd, double tick,
                               uint32_t* ppct, uint2* pdur, uint2* prate, uint32_t* rate_err);
__global__ void k_pod_direct_verify(const uint4* pods, uint32_t total, uint4* slots, uint32_t stamp,
                                    unsigned long long* ovf, uint32_t mask, uint32_t nd);
__global__ void k_vni_ht_build(const uint4* ents, uint32_t n, uint32_t* slots, uint32_t mask);
__global__ void k_vni_fill(const uint4* ents, const uint32_t* slots, uint32_t nslots, uint4* out);
__global__ void k_vni_pack(const uint32_t* node, const int32_t* vni, const uint32_t* net_ns,
                           uint32_t n, uint4* ents);
template <int V>
__global__ void k_reconcile(DevTopos T, DevLinks O, DevLinks N, DevTables tb, RecOut out,
                            RecWork wk);

// ---- wire encoding of the batches (kdtn_wire.hip) --------------------------------------
constexpr int SCAN_CHUNK = BLOCK * 4;   // values per block of the batch-offset scan
constexpr int SCAN_TOP_BLOCK = 1024, SCAN_TOP_PER = 16;   // k_scan_top: one block, totals per thread
constexpr int WIRE_IMG = 8192;          // LDS bytes per wave for a wave's wire output (32 KB per
                                        // block: 5 blocks per CU; a longer wave range stores directly)
constexpr int REMOTE_IMG = 10240;       // k_remote_write: 64 RemotePod messages (~124 B each) and their
                                        // slot metadata fit one round (40 KB per block: 4 blocks per
                                        // CU, the occupancy its ~100 VGPRs allow anyway)
// Inline string tables of the encoders (per dictionary, k_str_inline): one entry per string,
// SI_KW dwords per key string, SI_PW per property string. Byte 0 of an entry is the string's
// length when the string is valid UTF-8 and fits (bytes 1..len hold it, so bytes 0..len are
// the protobuf length varint and the bytes of a string field); SI_LONG: longer, dword 1 = arena
// offset, dword 2 = length; SI_BAD: not valid UTF-8 (proto.Marshal fails; no bytes). A string
// then costs one gather of one line instead of a table entry and its arena bytes. len1: one
// byte per string, its length when <= 254 and valid, else 255 (read the entry) — the sizing
// passes' table (12 MB for 12M strings instead of the 96 MB of 8-B entries).
constexpr int SI_KW = 6, SI_PW = 4;
constexpr uint32_t SI_LONG = 0x40u, SI_BAD = 0x80u;
struct StrTab {
    const uint32_t* inl;            // [n * W] entries
    const uint8_t* len1;            // [n]
    const uint8_t* bytes;           // the dictionary arena (long strings)
};
struct WireIn {
    StrTab kd, pd;
    const uint32_t* coarse[3];      // k_list_coarse of del_off, add_off, upd_off (or null)
    const uint32_t* t_name;
    const uint32_t* t_src;
    const uint32_t* t_netns;
    const uint32_t* t_ns;
    const uint32_t* list_off[3];    // del_off, add_off, upd_off
    const uint32_t* list_idx[3];    // del_idx, add_idx, upd_idx
    uint32_t list_base[3];          // global entry index of each list's first entry
    uint32_t n_entries, T;
};
struct WireWork {
    uint32_t* size;                 // [entries] encoded bytes of the entry (its Link field, plus the
                                    // LocalPod header for the batch's first entry)
    uint32_t* topo;                 // [entries] topology of the entry
    uint64_t* pos;                  // [entries+1] arena offset of every entry (scan of the sizes of
                                    // entries whose batch marshals), pos[entries] = total
    uint32_t* err;                  // [T+1] bit l of err[t]: list l of topology t failed to marshal;
                                    // err[T] != 0: a batch of more than 4 GiB
    uint64_t* off;                  // [3T+1] batch byte offsets
    uint64_t* pinfo;                // [add entries] where the entry's properties field (tag, length,
                                    // LinkProperties) lies: offset from the entry's start << 32 | its
                                    // length — the RemotePod writer copies those bytes (same field 7)
};
// ---- tc argv synthesis (kdtn_tc.hip) ---------------------------------------------------
struct TcIn {
    DevLinks N;
    const uint8_t* reach_add;       // k_reach flags
    const uint8_t* reach_upd;
    const uint32_t* add_idx;
    const uint32_t* upd_idx;
    const uint4* add_res;
    const uint4* upd_res;
    const uint2* add_qdisc;
    const uint2* upd_qdisc;
    StrTab kd;
    uint32_t n_add, n_upd;
};
__global__ void k_tc_sizes(TcIn w, uint32_t* size);
__global__ void k_tc_write(TcIn w, const uint64_t* off, uint8_t* arena);

// ---- resident epoch state: status commit and delta upload (kdtn_state.hip) -----------------
enum : uint8_t { ASM_SEG_A = 0, ASM_SEG_B = 1, ASM_REF = 2 };   // source of a topology's new segment
__global__ void k_commit_plan(DevTopos T, const uint8_t* action, const uint32_t* cut, const uint8_t* mask,
                              uint32_t* len, uint32_t* base, uint8_t* mode, uint8_t* flags_out, uint32_t* n_commit);
__global__ void k_commit_all_flags(uint8_t* flags, uint32_t T);
__global__ void k_delta_map(const uint32_t* topo, uint32_t n, uint32_t T, uint32_t* chg);
// delta validation error bits (misc word MISC_DELTA_ERR)
enum : uint32_t { DERR_TOPO = 1, DERR_OFF = 2, DERR_NIL = 4, DERR_IDS = 8, DERR_REF = 16, DERR_PREV = 32,
                  DERR_NEW = 64, DERR_KEEP = 128, DERR_COLS = 256 };
struct DeltaPlanIn {
    DevTopos T0;                          // the resident (previous) topology table
    const uint32_t* chg;                  // [n_topos] changed-list index, NONE = unchanged
    const uint32_t* prev;                 // [n_topos] previous index | KDTN_DELTA_NEW; NULL = identity
    const uint32_t* d_off;
    const uint32_t* d_src;
    const uint32_t* d_netns;
    const uint8_t* d_nil;
    const uint32_t* d_ns;
    const uint32_t* d_name;
    uint32_t n_topos, D;
};
struct DeltaPlanOut {
    uint32_t* ns;                         // (prev only)
    uint32_t* name;                       // (prev only)
    uint32_t* src_ip;
    uint32_t* net_ns;
    uint8_t* flags;
    uint32_t* dlen;                       // desired plan
    uint32_t* dbase;
    uint8_t* dmode;
    uint32_t* rlen;                       // realised plan (prev only; mode ASM_SEG_A)
    uint32_t* rbase;
    uint32_t* row_list;                   // changed pod-status rows (identity only)
    uint32_t* row_n;
    uint32_t* seen;                       // [ceil(T0/32)] previous indices named (prev only)
    uint32_t* err;
};
struct DeltaCheckIn {
    const uint32_t* topo;
    const uint32_t* off;
    const uint8_t* nil;
    const uint32_t* src;
    const uint32_t* netns;
    const uint32_t* ref;
    const uint32_t* kd_offs;              // resident dictionary offsets (kept prefix)
    const uint32_t* pd_offs;
    uint32_t n, nref, n_topos, D, n_new, n_old;
    uint32_t kd_keep, pd_keep, kd_expect, pd_expect;
};
__global__ void k_delta_plan(DeltaPlanIn in, DeltaPlanOut o);
__global__ void k_delta_check(DeltaCheckIn in, uint32_t* err);
__global__ void k_delta_totals(const uint64_t* doff, uint32_t Tn, const uint64_t* roff, uint32_t* misc);
__global__ void k_off_narrow(const uint64_t* in, uint32_t n, uint32_t* out);
__global__ void k_pods_pack(DevTopos T, const uint32_t* topo, uint32_t n, uint32_t cap, uint32_t rank_base,
                            uint4* out);
__global__ void k_pods_patch(const uint4* ent, uint32_t n, uint4* pods, uint4* slots, uint32_t stamp, uint32_t nd);
__global__ void k_soa_to_tiles(const uint32_t* stage, const int64_t* uid, uint32_t n, uint32_t* out, uint32_t* colmax);
struct AsmGuard {                         // k_store_assemble in a delta upload (all zero otherwise)
    const uint32_t* err;                  // the delta's error word: nothing is copied once set
    const uint64_t* n_dev;                // exact record count (the grid covers a bound)
    uint32_t skip_new;                    // inline records are placed by k_delta_inline
    uint32_t skip_ref;                    // reference lists are placed by k_delta_refs
};
__global__ void k_store_assemble(const uint32_t* off, uint32_t nt, const uint32_t* base, const uint8_t* mode,
                                 const uint32_t* ref, DevLinks A, DevLinks B, uint32_t n, AsmGuard g, uint32_t* out);
__global__ void k_delta_refs(const uint32_t* d_off, const uint32_t* topo, uint32_t n, const uint32_t* ref,
                             uint32_t nref, const uint32_t* off, DevLinks A, const uint32_t* err, uint32_t* dest,
                             uint32_t* multi, uint32_t* out);
__global__ void k_delta_place(const uint32_t* stage, const int64_t* uid, uint32_t n, const uint32_t* dest,
                              const uint32_t* err, uint32_t* out, uint32_t* colmax, uint32_t c0, uint32_t c1,
                              uint32_t with_uid);
__global__ void k_delta_inline(const uint32_t* d_off, const uint32_t* topo, uint32_t n, const uint32_t* ref,
                               uint32_t nref, const uint32_t* off, DevLinks B, const uint32_t* err, uint32_t* out);

// ---- incremental CR ingest on a resident state (kdtn_informer.hip) ------------------------
__global__ void k_strix_insert(const uint8_t* bytes, const uint32_t* offs, uint32_t from, uint32_t n,
                               unsigned long long* slots, uint32_t mask);
__global__ void k_strix_lookup(const uint8_t* lb, const uint32_t* lo, uint32_t nl, const uint8_t* rb, const uint32_t* ro,
                               const unsigned long long* slots, uint32_t mask, uint32_t* map, uint32_t* miss,
                               uint32_t* mlen);
__global__ void k_strix_append(const uint8_t* lb, const uint32_t* lo, uint32_t nl, const uint64_t* rank,
                               const uint64_t* boff, uint32_t D0, uint32_t arena0, uint32_t* map, uint8_t* rb,
                               uint32_t* ro);
__global__ void k_ix_map_topos(uint32_t* ns, uint32_t* name, uint32_t* src, uint32_t* netns, const uint8_t* flags,
                               uint32_t T, const uint32_t* kmap, uint8_t* nil);
__global__ void k_ix_map_links(uint32_t* base, uint32_t n, const uint32_t* kmap, const uint32_t* pmap);
__global__ void k_topokey_insert(const uint32_t* ns, const uint32_t* name, uint32_t T, unsigned long long* keys,
                                 uint32_t* vals, uint32_t mask);
__global__ void k_topokey_match(const uint32_t* ns, const uint32_t* name, uint32_t Tl, const unsigned long long* keys,
                                const uint32_t* vals, uint32_t mask, unsigned long long* dkeys, uint32_t dmask,
                                const uint32_t* keep, uint32_t* claim,
                                uint32_t* res, uint32_t* created, uint32_t* err);
__global__ void k_topo_delete(const uint32_t* del, uint32_t n, uint32_t T, uint32_t* keep, uint32_t* err);
__global__ void k_ix_layout(const uint32_t* keep, const uint64_t* kpos, uint32_t T0, const uint32_t* claim,
                            const uint32_t* created, const uint64_t* cpos, uint32_t Tl, uint32_t n_kept,
                            uint32_t* prev, uint32_t* chg);
__global__ void k_ix_refs(uint32_t* ref, uint32_t n);

// ---- RemotePod messages (kdtn_wire.hip) and the receiving daemon's tc argv (kdtn_tc.hip) ----
// message m: the UpdateRemote payload of add entry rem_idx[m] (m < n_remote, fan-out order) or
// the physical peer's local Update payload of add entry phys_idx[m - n_remote]
struct RemoteIn {
    StrTab kd, pd;
    const uint32_t* add_coarse;     // k_list_coarse of add_off (or null)
    const uint32_t* kd_offs;        // physical peers: TrimPrefix(PeerPod, "physical/") from the arena
    // the run's wire encoding (kdtn_epoch_encode), or w_pinfo = null: an add entry whose AddLinks
    // batch marshalled has its properties field at w_pos[w_nd + e] + (w_pinfo[e] >> 32)
    const uint64_t* w_pinfo;
    const uint64_t* w_pos;
    const uint8_t* w_arena;
    const uint32_t* w_err;
    uint32_t w_nd;
    const uint32_t* t_ns;
    const uint32_t* t_src;
    const uint32_t* t_netns;
    const uint32_t* add_off;
    const uint32_t* add_idx;
    const uint4* add_res;
    const uint2* add_qdisc;
    const uint4* pods;              // global pod-status rows (the peer's status.net_ns)
    const uint32_t* rem_idx;
    const uint32_t* phys_idx;
    const uint8_t* send;            // k_reach flags per add entry (REACH_SEND: an UpdateRemote)
    const uint32_t* phys_flag;      // per add entry: a physical peer's local Update
    const uint64_t* phys_pos;       // exclusive scan of phys_flag
    const uint32_t* rem_inv;        // per add entry with REACH_SEND: its message index
    DevLinks N;
    uint32_t n_msgs, n_remote, T, n_add;
};
__global__ void k_remote_phys_flags(const uint8_t* reach_add, const uint4* add_res, uint32_t na, uint32_t* flag);
__global__ void k_remote_phys_scatter(const uint32_t* flag, const uint64_t* pos, uint32_t na, uint32_t* phys_idx);
__global__ void k_remote_sizes(RemoteIn r, uint32_t* msz, uint32_t* tsz);
__global__ void k_remote_write(RemoteIn r, const uint64_t* off, uint8_t* arena);
__global__ void k_tc_remote_write(RemoteIn r, const uint64_t* off, uint8_t* arena);

// ---- RemotePod fan-out grouping (kdtn_fanout.hip) ---------------------------------------
constexpr int FAN_CHUNK = 1024;        // add entries per single-wave workgroup
constexpr int FAN_NODE_CAP = 8192;     // destination daemons per epoch (LDS histogram)
struct FanIn {
    const uint32_t* add_off;
    const uint4* add_res;
    const uint2* add_qdisc;
    uint32_t T, n_add, stamp;
    const uint32_t* add_node;       // ReachIn.add_node (null: add_res.z)
};
// murmur3 finalizer (hash tables keyed by packed ids)
KD_INLINE uint64_t hash64(uint64_t x) {
    x ^= x >> 33;
    x *= 0xFF51AFD7ED558CCDull;
    x ^= x >> 33;
    x *= 0xC4CEB9FE1A85EC53ull;
    x ^= x >> 33;
    return x;
}
// home slot of a VxlanManager key (node, vni)
KD_INLINE uint32_t vni_home(uint32_t node, uint32_t vni, uint32_t mask) {
    return (uint32_t)hash64(((uint64_t)node << 32) | vni) & mask;
}

// which entries the daemons reach (kdtn_fanout.hip k_reach; include/kdtn.h)
KD_INLINE bool sends_remote(uint4 r, uint32_t qerr) {
    return (r.w & 0xFFu) == KDTN_KIND_CROSS_NODE && ((r.w >> 8) & 0xFFu) == 0 && qerr == 0;
}
// a link whose step fails before its RPC aborts its batch (addLink's error chain; qdisc only
// where built)
KD_INLINE bool add_fails(uint4 r, uint32_t qerr) {
    const uint32_t kind = r.w & 0xFFu;
    if ((r.w >> 8) & 0xFFu) return true;
    return (kind == KDTN_KIND_SAME_NODE || kind == KDTN_KIND_CROSS_NODE || kind == KDTN_KIND_PHYSICAL) && qerr != 0;
}
KD_INLINE uint32_t qdisc_err(const uint2* q, uint32_t e) { return (q[(size_t)e * 9 + 8].y >> 16) & 0xFFu; }
// topology of entry e: offs[t] <= e < offs[t + 1] (upper bound over the T + 1 offsets)
KD_INLINE uint32_t entry_topo(const uint32_t* offs, uint32_t T, uint32_t e) {
    uint32_t lo = 0, hi = T;                           // offs[lo] <= e < offs[hi]
    while (hi - lo > 1) {
        const uint32_t mid = (lo + hi) >> 1;
        if (offs[mid] <= e) lo = mid;
        else hi = mid;
    }
    return lo;
}

enum : uint8_t { REACH_ON = 1, REACH_SEND = 2 };
// message kind of add entry e: 1 = UpdateRemote, 2 = physical local Update, 0 = none
KD_INLINE uint32_t remote_kind(const RemoteIn& r, uint32_t e) {
    if (r.send[e] & REACH_SEND) return 1u;
    return r.phys_flag[e] ? 2u : 0u;
}
KD_INLINE uint32_t remote_msg_index(const RemoteIn& r, uint32_t e, uint32_t kind) {
    return kind == 1u ? r.rem_inv[e] : r.n_remote + (uint32_t)r.phys_pos[e];
}
struct ReachIn {
    const uint32_t* del_off;
    const uint4* del_res;
    const uint32_t* add_off;
    const uint4* add_res;
    const uint2* add_qdisc;
    const uint32_t* upd_off;
    const uint4* upd_res;
    uint32_t T, stamp;
    const uint8_t* add_qerr;        // RecOut.add_qerr (null: the qdisc records' error bytes)
    uint32_t* add_node;             // k_reach_cuts: add_res.z of every add entry in a dense array
                                    // (k_reach and the fan-out read 4 B instead of the 16-B
                                    // records), or null
    const uint32_t* add_coarse;     // k_list_coarse of add_off / upd_off (or null)
    const uint32_t* upd_coarse;
};
// coarse[w] = the topology of list entry 64 w (one thread per topology, its groups' starts)
__global__ void k_list_coarse(const uint32_t* offs, uint32_t T, uint32_t* coarse);
__global__ void k_reach_cuts(ReachIn f, uint32_t nd, uint32_t na, uint32_t nu, uint32_t* cut, uint8_t* st_add);
__global__ void k_reach(ReachIn f, uint32_t na, uint32_t nu, const uint32_t* cut, const uint8_t* st_add, uint32_t* mark,
                        uint8_t* reach_add, uint8_t* reach_upd);

// VxlanManager state after the epoch (kdtn_vni.hip; include/kdtn.h kdtn_epoch_vni_apply)
struct VniOpsIn {
    ReachIn r;                      // the epoch's batches (r.stamp unused)
    const uint32_t* t_src;          // topology status.src_ip / status.net_ns (kdict ids)
    const uint32_t* t_netns;
    const uint4* pods;              // global pod-status rows (peer netns of a remote Update)
    uint32_t n_del, n_add;
};
// one op per del entry (slot e) and two per add entry (slots n_del + 2e, + 1):
// {node, vni, net_ns, kind} with kind VOP_NONE / VOP_DEL / VOP_ADD / VOP_DEL_MISS (a reached
// delLink whose Get(vni) missed the snapshot: no effect on the map, kept for the order check);
// net_ns of a delete = the local pod's netns its Get compares against
enum : uint32_t { VOP_NONE = 0, VOP_DEL = 1, VOP_ADD = 2, VOP_DEL_MISS = 3 };
__global__ void k_vni_cuts(VniOpsIn f, uint32_t* cut);
__global__ void k_vni_ops(VniOpsIn f, const uint32_t* cut, uint4* ops);
__global__ void k_vni_shadow(const uint4* ents, uint32_t n_ents, const uint32_t* slots, uint32_t mask, uint8_t* dead);
__global__ void k_vni_del(const uint4* ops, uint32_t n_del, const uint4* ents, const uint32_t* slots, uint32_t mask,
                          uint8_t* dead);
__global__ void k_vni_insert(const uint4* add_ops, uint32_t n_ops, const uint4* ents, const uint8_t* dead, uint32_t n_ents,
                             uint32_t* slots, uint32_t mask);
__global__ void k_vni_vis_count(const uint4* add_ops, uint32_t n_ops, const uint4* ents, const uint8_t* dead,
                                uint32_t n_ents, const uint32_t* slots, uint32_t mask, uint8_t* vis, uint64_t* part);
__global__ void k_vni_vis_write(const uint4* add_ops, uint32_t n_ops, const uint4* ents, const uint8_t* dead,
                                uint32_t n_ents, const uint8_t* vis, const uint64_t* part, uint32_t* node,
                                int32_t* vni, uint32_t* net_ns, uint32_t* n_out);
// order-dependent keys (kdtn_vni_contested)
__global__ void k_vni_dtab_insert(const uint4* dels, uint32_t n_del, uint4* dkeys, uint32_t* dused, uint32_t dmask);
__global__ void k_vni_contest(const uint4* add_ops, uint32_t n_ops, const uint4* ents, const uint8_t* dead,
                              const uint32_t* slots, uint32_t mask, const uint4* dkeys, const uint32_t* dused,
                              uint32_t dmask, uint32_t* flag);
__global__ void k_vni_contest_write(const uint4* add_ops, const uint32_t* flag, const uint64_t* pos, uint32_t n_ops,
                                    uint32_t* node, int32_t* vni);
__global__ void k_fan_nodes_count(const uint32_t* mark, uint32_t nw, uint64_t* part);
__global__ void k_fan_nodes_write(const uint32_t* mark, uint32_t nw, const uint64_t* part, uint32_t* node_idx,
                                  uint32_t* nodes, uint32_t* n_nodes);
__global__ void k_fan_count(FanIn f, const uint8_t* send, const uint32_t* node_idx, const uint32_t* n_nodes,
                            uint32_t* counts, uint32_t nchunks);
__global__ void k_fan_scatter(FanIn f, const uint8_t* send, const uint32_t* node_idx, const uint32_t* n_nodes,
                              const uint64_t* base, uint32_t nchunks, uint32_t* out_idx, uint32_t* out_inv);
KD_INLINE uint64_t block_exclusive(uint64_t v, uint64_t* sh, uint64_t* total) {
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    uint64_t x = v;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        const uint64_t o = __shfl_up(x, d, 64);
        if (lane >= d) x += o;
    }
    if (lane == 63) sh[wave] = x;
    __syncthreads();
    uint64_t base = 0, tot = 0;
#pragma unroll
    for (int k = 0; k < BLOCK / 64; ++k) {
        if (k < wave) base += sh[k];
        tot += sh[k];
    }
    __syncthreads();
    *total = tot;
    return base + x - v;
}

template <int W>
__global__ void k_str_inline(const uint8_t* bytes, const uint32_t* offs, uint32_t n, uint32_t* inl, uint8_t* len1);
__global__ void k_wire_entry_sizes(WireIn w, DevLinks O, DevLinks N, WireWork wk);
__global__ void k_wire_scan_partial(WireIn w, WireWork wk, uint64_t* part);
__global__ void k_wire_scan_final(WireIn w, WireWork wk, const uint64_t* part);
__global__ void k_wire_batch_off(WireIn w, WireWork wk);

__global__ void k_scan_partial(const uint32_t* size, uint32_t n, uint64_t* part);
__global__ void k_scan_top(uint64_t* part, uint32_t nb);
__global__ void k_scan_final(const uint32_t* size, uint32_t n, const uint64_t* part, uint64_t* off);
__global__ void k_wire_write(WireIn w, DevLinks O, DevLinks N, WireWork wk, uint8_t* arena);
__global__ void k_qdisc_batch(DevLinks props, DevTables tb, uint2* out);
constexpr int FP_BLOCK = 1024, FP_GRID = 256;       // k_full_prefix launch shape
__global__ void k_full_prefix(DevTopos T, uint32_t* first_partial_inv);
template <int PER>
__global__ void k_pod_verify_prefix(const uint4* pods, uint32_t total, uint4* slots, uint32_t stamp,
                                    unsigned long long* ovf, uint32_t mask, uint32_t nd, DevTopos T,
                                    uint32_t* first_partial_inv, uint32_t nbv, uint32_t nr, uint32_t gathered);

// ---- CR ingest: TopologyList JSON → epoch tables (kdtn_ingest.hip) ------------------------
// The token stream: brackets, strings and scalars (the ',' / ':' bytes are no tokens), as two
// arrays of 4-byte words — the byte offset, and the meta word: pre-depth (bits 0-23) | kind << 24
// (4 bits) | sep << 28, the separator between the previous token and this one (SEP_* of the
// earliest when several stand there, which k_js_tokens reports). Kernels that need only
// depths and kinds (the parent scans) read the meta words alone.
enum : uint32_t { TK_OBJ = 0, TK_OBJ_END = 1, TK_ARR = 2, TK_ARR_END = 3, TK_COLON = 4, TK_COMMA = 5,
                  TK_STR = 6, TK_SCALAR = 7 };
constexpr uint32_t TK_DEPTH_MASK = 0xFFFFFFu;
enum : uint32_t { SEP_NONE = 0, SEP_COLON = 1, SEP_COMMA = 2 };
struct JsToks {
    uint32_t* pos;             // byte offset of the token's first byte
    uint32_t* meta;            // pre-depth | kind << 24 | sep << 28
};
constexpr int JS_PD = 16;                    // depth levels resolved by the parent max-scan
constexpr int JS_PER = 16;                   // tokens per thread in tile kernels
constexpr int JS_TILE = BLOCK * JS_PER;      // tokens per tile
constexpr uint32_t JS_NONE = 0xFFFFFFFFu, JS_DEEP = 0xFFFFFFFEu;
// container roles on the TopologyList schema
enum : uint32_t { R_NONE = 0, R_ROOT, R_ITEMS, R_ITEM, R_META, R_SPEC, R_STATUS, R_SPEC_LINKS, R_STATUS_LINKS,
                  R_LINK_S, R_LINK_R, R_PROPS_S, R_PROPS_R };
constexpr uint32_t JS_ST_OVERFLOW = 1, JS_ST_LONG = 2;   // intern status bits
// ingest variants (KDTN_JS_VARIANT, profiling build only; bits 1-3 give wrong tables)
constexpr uint32_t JSV_COHERENT = 1, JSV_NO_SEEN = 2, JSV_NO_REP = 4, JSV_NO_INTERN = 8, JSV_NO_INLINE = 16,
                   JSV_NO_INLINE_K = 32, JSV_NO_INLINE_P = 64,   // 16: neither dictionary, 32 / 64: keys / props
                   JSV_MASKS = 128,            // string ends from the mask words only (no window SWAR)
                   JSV_NO_STRCHK = 256, JSV_NO_SCALAR = 512;   // k_js_validate without string / scalar checks

struct JsDoc {
    const uint8_t* doc;        // padded with spaces to nb*64 (+64 B)
    uint32_t n;                // document bytes
    uint32_t nb;               // 64-byte blocks
    const uint64_t* qmask;     // unescaped quotes
    const uint64_t* bsmask;    // backslashes
    const uint64_t* hbmask;    // bytes >= 0x80
    const uint64_t* escmask;   // bytes escaped by an odd backslash run right before them
    uint32_t variant;          // (profiling build) KDTN_JS_VARIANT bits, 0 otherwise
};
struct JsMasks {
    uint64_t* tok;             // token starts
    uint64_t* open;            // { [ outside strings
    uint64_t* close;           // } ] outside strings
    uint32_t* gcnt;            // per workgroup of BLOCK blocks, 5 arrays of ng: tokens, 64 + opens -
                               // closes, opens, colons, scalar tokens (group_sums)
};
struct JsTopoOut {
    uint32_t* ns;
    uint32_t* name;
    uint32_t* src_ip;
    uint32_t* net_ns;
    uint32_t* flags;           // u32 KDTN_TOPO_* bits during the decode
    uint32_t* real_off;
    uint32_t* des_off;
};
// A decoded link record in the row-major staging: JS_ROW words in the tile's column order
// (keys, properties, gap, then the i64 uid as two words); k_js_finalize_links transposes whole
// tiles into the AoSoA store and maps the id columns' slot + 1 to the dictionary ids.
constexpr int JS_ROW = LINK_COLS32 + 2;
static_assert(JS_ROW * TILE_RECS == TILE_WORDS, "a staged tile is a store tile");
struct JsStore {
    uint32_t* base;            // row-major staging, JS_ROW words per record, whole tiles
};
// An intern table slot (32 B, one per aligned quarter line): the key word (0 = empty) and, for
// a document string of at most JS_INL bytes with no zero byte, its bytes, stored by the
// inserting thread after its CAS. A repeated string compares against those bytes instead of
// re-reading its first occurrence's window in the document (a random position). A slot whose
// bytes are not stored yet reads as zeros (the table is cleared per decode), and no inline
// string has a zero byte, so a zero byte within the length means "not available".
constexpr uint32_t JS_INL = 24;
constexpr uint32_t JS_MAX_PROBE = 256;         // longest probe run before the table is grown
struct JsSlot {
    unsigned long long kw;
    uint32_t b[6];
};
static_assert(sizeof(JsSlot) == 32, "32-byte slots");
struct JsDict {
    JsSlot* slots;             // key words + inline bytes (the probes)
    unsigned long long* keys;  // the key words again, dense (the per-slot passes after the decode)
    uint32_t* rep;             // first occurrence (token index) per slot
    uint32_t mask;
};
struct JsIntern {
    const uint8_t* doc;
    uint8_t* heap;             // decoded strings that differ from their raw bytes
    unsigned long long* heap_used;
    uint64_t heap_cap;
    uint32_t* status;          // JS_ST_* bits
    uint32_t* owner;           // token index per (object, schema field): root 1, topology 9, record 22
    uint32_t* vown;            // per member value: its owner slot, JS_NONE = not a schema field
    uint32_t own_des, own_real;   // first record slot of each side
    JsDict kd, pd;
    uint32_t variant;
};
__global__ void k_js_quotes(JsDoc j, uint64_t* qmask, uint64_t* bsmask, uint64_t* hbmask, uint64_t* escmask,
                            uint32_t* gq);
__global__ void k_js_classify(JsDoc j, const uint64_t* gqoff, JsMasks m, uint32_t ng, unsigned long long* err);
__global__ void k_js_tokens(JsDoc j, JsMasks m, const uint64_t* goff, uint32_t ng, JsToks tk, uint32_t* olist,
                            uint8_t* odep, uint32_t* vlist, uint32_t* slist, unsigned long long* err);
__global__ void k_js_scalars(JsDoc j, const uint32_t* tpos, const uint32_t* slist, uint32_t nscal, unsigned long long* err);
__global__ void k_js_par_agg(const uint32_t* tmeta, uint32_t ntok, uint32_t* tagg);
__global__ void k_js_par_group(const uint32_t* tagg, uint32_t ntiles, uint32_t* gagg);
__global__ void k_js_par_top(uint32_t* gagg, uint32_t ng);
__global__ void k_js_par_tiles(uint32_t* tagg, uint32_t ntiles, const uint32_t* gagg);
__global__ void k_js_par_apply(const uint32_t* tmeta, uint32_t ntok, const uint32_t* texcl, uint32_t* par, uint32_t* deep);
__global__ void k_js_deep(const uint32_t* tmeta, uint32_t ntok, uint32_t* par, const uint32_t* deep);
__global__ void k_js_tail(JsDoc j, JsToks tk, uint32_t ntok, const uint32_t* par, unsigned long long* err);
__global__ void k_js_validate(JsDoc j, JsToks tk, uint32_t ntok, const uint32_t* par, uint8_t* ecand,
                              unsigned long long* err);
__global__ void k_js_roles(JsDoc j, JsToks tk, const uint32_t* olist, uint32_t nopen, const uint32_t* par,
                           uint8_t* role, const uint8_t* odep, uint32_t level);
__global__ void k_js_elems_count(JsDoc j, JsToks tk, uint32_t ntok, const uint32_t* par, uint8_t* role,
                                 uint32_t* cnt3, uint8_t* ecls, unsigned long long* derr);
__global__ void k_js_elems_write(const uint8_t* ecls, uint32_t ntok, const uint64_t* coff3, uint32_t ntiles,
                                 uint32_t* ord, JsTopoOut to);
__global__ void k_js_values(JsDoc j, JsToks tk, const uint32_t* vlist, uint32_t nval, const uint32_t* par,
                            const uint8_t* role, const uint32_t* ord, JsTopoOut to, JsStore des, JsStore real,
                            JsIntern in, unsigned long long* derr);
__global__ void k_js_dups(const uint32_t* vlist, uint32_t nval, const uint32_t* vown,
                          uint32_t* owner, uint32_t* any);
__global__ void k_js_dups_report(const uint32_t* tpos, const uint32_t* vlist, uint32_t nval, const uint32_t* vown,
                                 const uint32_t* owner, const uint32_t* any, unsigned long long* derr);
__global__ void k_js_rep_mark(JsDict dt, uint32_t* bits);
__global__ void k_js_popc(const uint32_t* bits, uint32_t nw, uint32_t* cnt);
__global__ void k_js_ids(JsDict dt, const uint32_t* bits, const uint64_t* wrank, uint32_t* slot_id, uint32_t* len_by_id,
                         uint32_t* slot_of_id);
__global__ void k_js_dict_copy(JsDict dt, JsIntern in, const uint32_t* slot_of_id, uint32_t n, const uint64_t* off64,
                               uint32_t* offs, uint8_t* arena);
__global__ void k_js_finalize_links(const uint32_t* rows, uint32_t* tiles, const uint32_t* kslot_id,
                                    const uint32_t* pslot_id);
__global__ void k_js_finalize_topos(JsTopoOut to, uint32_t T, const uint32_t* kslot_id, uint8_t* flags8);

// sharded ingest (kdtn_json_ingest_shard): keep[t] = this shard owns topology t; then the
// kept topologies' columns and records compacted into fresh tables (document order kept)
__global__ void k_shard_mark(DevTopos T, const uint8_t* kd_bytes, const uint32_t* kd_offs, uint32_t nshards,
                             uint32_t shard, uint32_t* keep, uint32_t* kreal, uint32_t* kdes);
__global__ void k_shard_topos(DevTopos T, const uint32_t* keep, const uint64_t* tidx, const uint64_t* roff,
                              const uint64_t* noff, DevTopos out, uint32_t* doc_index);
__global__ void k_shard_links(DevLinks in, const uint32_t* off, uint32_t nt, const uint32_t* keep,
                              const uint64_t* noff, uint32_t* out_base);

}  // namespace kdtn
