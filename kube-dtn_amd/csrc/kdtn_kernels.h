// kdtn_kernels.h — HIP kernels of one reconcile epoch (gfx950 / CDNA4, wave64).
//
// Data layout in HBM (all SoA, one column per field, records grouped by Topology):
//   link tables  : 7 × u32 key-string ids, i64 uid, 12 × u32 property ids, u32 gap
//                  (88 B per record per side)
//   topologies   : u32 ns/name/src_ip/net_ns ids, u8 flags, u32 offsets (T+1) per side
//   dictionaries : u8 arena + u32 offsets; parsed once per epoch into compact tables
//                  kflags (u8 per key string) and pparsed (16 B per property string)
// Kernels (launch order):
//   k_kdict_flags   MakeVeth/addLink predicates per key string         (D threads)
//   k_pdict_parse   ParseDuration/ParseFloatPercentage/ParseRate       (P threads)
//   k_pods_fill     pod-status slice of this rank (16 B per pod)       (slice threads)
//   [RCCL all-gather of the pod-status table when nranks > 1]
//   k_pod_ht_build  (ns,name) → pod index open-addressing table        (pods threads)
//   k_vni_ht_build  (node,vni) → VxlanManager entry                    (V threads)
//   k_diff          gate + CalcDiff per workgroup of TPW topologies, LDS-staged hashes
//   k_scan          exclusive scan of the per-workgroup batch counts   (1 workgroup)
//   k_emit          order-preserving compaction into batch lists + resolve + MakeQdiscs
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/kdtn.h"
#include "kdtn_parse.h"

namespace kdtn {

constexpr int BLOCK = 256;   // 4 waves of 64
constexpr int TPW = 64;      // topologies per workgroup in k_diff / k_emit (= one wave of lanes)
constexpr int CAP = 4096;    // LDS window capacity, records (old + new)

// key-string flags
enum : uint8_t {
    KF_CIDR_BAD = 1,    // non-empty and net.ParseCIDR fails
    KF_MAC_BAD = 2,     // non-empty and net.ParseMAC fails
    KF_LOCALHOST = 4,   // == "localhost"
    KF_PHYSICAL = 8,    // has prefix "physical/"
};
// property-string flags (pparsed.w)
enum : uint32_t { PF_DUR_ERR = 1, PF_PCT_ERR = 2, PF_RATE_ERR = 4 };

// record flags written by k_diff
enum : uint8_t { RF_DEL = 1, RF_UPD = 2, RF_ADD = 1 };

struct DevLinks {
    const uint32_t* key[KDTN_NKEY];
    const int64_t* uid;
    const uint32_t* prop[KDTN_NPROP];
    const uint32_t* gap;
    uint32_t n;
};

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

struct DevTables {            // read-only lookup structures of the epoch
    const uint8_t* kflags;    // [D]
    const uint4* pparsed;     // [P] {p2u, dur_us, dur_ticks, flags}
    const uint64_t* prate;    // [P]
    const uint4* pods;        // [pod_total] {ns, name, src_ip, net_ns | spec_nil<<31}
    const uint64_t* pod_keys; // [pod_mask+1]
    const uint32_t* pod_vals;
    uint32_t pod_mask;
    const uint64_t* vni_keys; // [vni_mask+1]
    const uint32_t* vni_vals;
    const uint32_t* vni_netns;
    uint32_t vni_mask;
    const uint32_t* default_id;  // kdict id of "default" (0xFFFFFFFF if absent)
    uint32_t pod_base;        // global pod index of local topology 0
    int32_t vxlan_base;
};

struct DiffOut {
    uint8_t* oflag;           // [M]
    uint32_t* otarget;        // [M] first matching desired index (valid when RF_UPD)
    uint8_t* nflag;           // [N]
    uint8_t* action;          // [T]
    uint32_t* wg_cnt;         // [nwg*3] del, upd, add
    uint32_t* hscratch;       // [M+N] window hashes for topologies larger than CAP
    uint8_t* fscratch;        // [M+N] window flags for topologies larger than CAP
};

struct EmitOut {
    uint32_t* del_off;
    uint32_t* add_off;
    uint32_t* upd_off;
    uint32_t* del_idx;
    uint32_t* add_idx;
    uint32_t* upd_idx;
    uint4* del_res;           // kdtn_resolved as 16 B
    uint4* add_res;
    uint4* upd_res;
    uint2* add_qdisc;         // kdtn_qdisc as 9 × 8 B
    uint2* upd_qdisc;
    const uint32_t* wg_base;  // [nwg*3]
    uint32_t stages;
};

__global__ void k_kdict_flags(const uint8_t* bytes, const uint32_t* offs, uint32_t n,
                              uint8_t* flags, uint32_t* default_id);
__global__ void k_pdict_parse(const uint8_t* bytes, const uint32_t* offs, uint32_t n, double tick,
                              uint4* parsed, uint64_t* rate);
__global__ void k_pods_fill(DevTopos T, uint32_t slice, uint32_t rank_base, uint4* pods);
__global__ void k_pod_ht_build(const uint4* pods, uint32_t total, uint64_t* keys, uint32_t* vals,
                               uint32_t mask);
__global__ void k_vni_ht_build(const uint32_t* node, const int32_t* vni, uint32_t n, uint64_t* keys,
                               uint32_t* vals, uint32_t mask);
__global__ void k_diff(DevTopos T, DevLinks O, DevLinks N, DiffOut out);
__global__ void k_scan(const uint32_t* wg_cnt, uint32_t nwg, uint32_t* wg_base, uint32_t* totals,
                       uint32_t T, uint32_t* del_off, uint32_t* add_off, uint32_t* upd_off);
__global__ void k_emit(DevTopos T, DevLinks O, DevLinks N, const uint8_t* oflag,
                       const uint32_t* otarget, const uint8_t* nflag, const uint8_t* action,
                       DevTables tb, EmitOut out);
__global__ void k_qdisc_batch(DevLinks props, const uint4* pparsed, const uint64_t* prate,
                              uint2* out);

}  // namespace kdtn
