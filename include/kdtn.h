/*
 * kdtn.h — C-ABI of the MI355X batch topology-reconcile engine (libkdtn.so).
 *
 * This is the drop-in boundary for kube-dtn's reconcile hot path. The reference
 * (dtn-dslab/kube-dtn, Go) calls these pure functions directly; a Go build binds
 * this header through cgo (stub in INTEGRATION.md). Every entry point below cites
 * the reference function it replaces (paths relative to the reference root).
 *
 *   kdtn_reconcile_epoch  replaces, for every dirty Topology at once:
 *     - the Reconcile gate   controllers/topology_controller.go:77-88
 *     - CalcDiff             controllers/topology_controller.go:288-318
 *     - EqualWithoutProperties controllers/topology_controller.go:342-351
 *     - the pure prefix of the daemon batch handlers
 *         AddLinks/addLink   daemon/kubedtn/handler.go:592-611, 316-459
 *         DelLinks/delLink   daemon/kubedtn/handler.go:613-632, 461-492
 *         UpdateLinks        daemon/kubedtn/handler.go:634-671
 *     - MakeVeth parse       common/veth.go:13-41
 *     - MakeQdiscs           common/qdisc.go:20-199, 361-370 (+ netlink.NewNetem)
 *     - GetVniFromUid        common/utils.go:29-31
 *     - VxlanManager.Get     daemon/vxlan/manager.go:65-71
 *   kdtn_make_qdiscs      replaces common.MakeQdiscs (common/qdisc.go:20) for a batch
 *   kdtn_diff             replaces CalcDiff + the Reconcile gate alone
 *   kdtn_resolve          replaces the pure prefix of the daemon's AddLinks / DelLinks for
 *                         one LinksBatchQuery (handler.go:592-632)
 *   kdtn_epoch_encode     replaces Link.ToProto + proto.Marshal of the batches
 *   kdtn_epoch_fanout     groups the daemons' UpdateRemote RPCs (common/utils.go:39-67)
 *                         per destination daemon
 *   kdtn_epoch_tc         synthesises SetVethQdiscs' `tc ... tbf` argv (common/qdisc.go:252-266)
 *   kdtn_epoch_remote_encode  marshals the RemotePod bodies of Remote.Update
 *                         (common/utils.go:39-67, daemon/kubedtn/handler.go:348-371)
 *   kdtn_epoch_late_pods  getPod's API-server fallback on an informer miss
 *                         (daemon/kubedtn/handler.go:35-39): late pod rows for the lookup
 *
 * Conventions
 *   - No C++ or HIP types cross this ABI: plain pointers, sizes and PODs.
 *   - Inputs are caller-owned HOST memory; the engine copies them to HBM and keeps
 *     no caller pointer after a call returns (cgo rule).
 *   - Return codes: 0 = OK, negative errno-style engine errors (kdtn_strerror).
 *     Per-link semantic failures are DATA (kdtn_err in the output records), never
 *     return codes — mirroring the reference where each link's error aborts only its
 *     own batch (handler.go:604-605).
 *   - A kdtn_ctx is not thread-safe; callers serialise (one per process/GPU).
 *   - Strings are interned: a kdtn_strtab is a DEDUPLICATED dictionary (id equality
 *     <=> byte equality) and id 0 MUST be the empty string "". kdtn_interner_*
 *     builds such tables.
 */
#ifndef KDTN_H
#define KDTN_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define KDTN_ABI_VERSION 1

/* ---- engine errors (return codes) ------------------------------------------------ */
#define KDTN_OK          0
#define KDTN_EINVAL    (-22)   /* malformed tables (offsets, ids out of range, ...)   */
#define KDTN_ENOMEM    (-12)   /* device or host allocation failed                    */
#define KDTN_EIO        (-5)   /* HIP / RCCL runtime failure                          */
#define KDTN_ENOSPC    (-28)   /* an output capacity is smaller than the batch        */
#define KDTN_ENODEV    (-19)   /* no usable gfx950 device                             */

/* ---- per-link semantic errors: first failing step, reference order --------------- */
typedef enum kdtn_err {
    KDTN_E_NONE = 0,
    KDTN_E_VETH_CIDR = 1,      /* MakeVeth local  net.ParseCIDR   common/veth.go:22          */
    KDTN_E_VETH_MAC = 2,       /* MakeVeth local  net.ParseMAC    common/veth.go:33          */
    KDTN_E_LATENCY = 3,        /* ParseDuration(latency)          common/qdisc.go:28         */
    KDTN_E_LATENCY_CORR = 4,   /* ParseFloatPercentage            common/qdisc.go:34         */
    KDTN_E_JITTER = 5,         /* common/qdisc.go:40 */
    KDTN_E_LOSS = 6,           /* common/qdisc.go:46 */
    KDTN_E_LOSS_CORR = 7,      /* common/qdisc.go:52 */
    KDTN_E_DUPLICATE = 8,      /* common/qdisc.go:58 */
    KDTN_E_DUPLICATE_CORR = 9, /* common/qdisc.go:64 */
    KDTN_E_REORDER_PROB = 10,  /* common/qdisc.go:70 */
    KDTN_E_REORDER_CORR = 11,  /* common/qdisc.go:76 */
    KDTN_E_CORRUPT_PROB = 12,  /* common/qdisc.go:82 */
    KDTN_E_CORRUPT_CORR = 13,  /* common/qdisc.go:88 */
    KDTN_E_RATE = 14,          /* ParseRate                       common/qdisc.go:110        */
    KDTN_E_PEER_LOOKUP = 15,   /* getPod miss                     daemon/kubedtn/handler.go:375-379 */
    KDTN_E_PEER_NO_LINKS = 16, /* ToProtoPod: peer spec.links nil handler.go:65-69,380-384   */
    KDTN_E_PEER_VETH_CIDR = 17,/* MakeVeth peer (same node)       handler.go:402             */
    KDTN_E_PEER_VETH_MAC = 18,
    KDTN_E_REMOTE_CIDR = 19    /* peer daemon's Update: net.ParseCIDR(IntfIp = link.PeerIp) in
                                  vxlan.CreateOrUpdate (daemon/vxlan/vxlan.go:80-83) fails, so
                                  UpdateRemote (common/utils.go:62-65) and addLink (handler.go:448-451)
                                  return it after the local VXLAN + qdiscs were set up */
} kdtn_err;

/* Reconcile decision per Topology (controllers/topology_controller.go:77-88). */
typedef enum kdtn_action {
    KDTN_ACT_SKIP = 0,     /* reflect.DeepEqual(status.links, spec.links)          :77   */
    KDTN_ACT_CREATED = 1,  /* status.links == nil: no batches, status := spec      :81   */
    KDTN_ACT_DIFF = 2      /* CalcDiff → DelLinks, AddLinks, UpdateLinks           :88   */
} kdtn_action;

/* addLink classification (daemon/kubedtn/handler.go:316-459). */
typedef enum kdtn_kind {
    KDTN_KIND_NONE = 0,        /* not classified (error before classification, or not an add) */
    KDTN_KIND_MACVLAN = 1,     /* peer_pod == "localhost"                 handler.go:333   */
    KDTN_KIND_PHYSICAL = 2,    /* peer_pod has prefix "physical/"         handler.go:348   */
    KDTN_KIND_PEER_DEAD = 3,   /* peer SrcIp or NetNs empty → skip, OK    handler.go:386-395 */
    KDTN_KIND_SAME_NODE = 4,   /* peer.SrcIp == local.SrcIp → veth pair   handler.go:399   */
    KDTN_KIND_CROSS_NODE = 5   /* VXLAN + RemotePod to peer daemon        handler.go:419   */
} kdtn_kind;

/* Link string columns (api/v1/topology_types.go:59-95), key of EqualWithoutProperties. */
enum {
    KDTN_K_LOCAL_INTF = 0, KDTN_K_LOCAL_IP, KDTN_K_LOCAL_MAC,
    KDTN_K_PEER_INTF, KDTN_K_PEER_IP, KDTN_K_PEER_MAC, KDTN_K_PEER_POD,
    KDTN_NKEY
};
/* LinkProperties string fields (api/v1/topology_types.go:119-176); Gap is separate. */
enum {
    KDTN_P_LATENCY = 0, KDTN_P_LATENCY_CORR, KDTN_P_JITTER, KDTN_P_LOSS, KDTN_P_LOSS_CORR,
    KDTN_P_RATE, KDTN_P_DUPLICATE, KDTN_P_DUPLICATE_CORR, KDTN_P_REORDER_PROB,
    KDTN_P_REORDER_CORR, KDTN_P_CORRUPT_PROB, KDTN_P_CORRUPT_CORR,
    KDTN_NPROP
};

/* Topology flags */
#define KDTN_TOPO_STATUS_NIL 0x1u   /* status.links == nil (JSON null/absent) */
#define KDTN_TOPO_SPEC_NIL   0x2u   /* spec.links   == nil                    */

/* ---- input tables ----------------------------------------------------------------- */
typedef struct kdtn_strtab {
    const uint8_t*  bytes;   /* arena                                          */
    const uint32_t* offs;    /* n+1 byte offsets; string i = bytes[offs[i], offs[i+1]) */
    uint32_t        n;       /* number of strings; id 0 must be ""             */
} kdtn_strtab;

/* A set of Link records, grouped by owning Topology (segments given by kdtn_topo_table). */
typedef struct kdtn_link_table {
    uint32_t        n;
    const uint32_t* key[KDTN_NKEY];   /* kdict ids                                   */
    const int64_t*  uid;              /* Link.UID (int on amd64 = int64)             */
    const uint32_t* prop[KDTN_NPROP]; /* pdict ids                                   */
    const uint32_t* gap;              /* LinkProperties.Gap                          */
} kdtn_link_table;

typedef struct kdtn_topo_table {
    uint32_t        n;          /* T topologies in this shard                          */
    const uint32_t* ns;         /* kdict id of metadata.namespace                      */
    const uint32_t* name;       /* kdict id of metadata.name                           */
    const uint32_t* src_ip;     /* kdict id of status.src_ip                           */
    const uint32_t* net_ns;     /* kdict id of status.net_ns                           */
    const uint8_t*  flags;      /* KDTN_TOPO_* bits                                    */
    const uint32_t* real_off;   /* T+1 offsets into the realised table (status.links)  */
    const uint32_t* des_off;    /* T+1 offsets into the desired table  (spec.links)    */
} kdtn_topo_table;

/* Snapshot of the daemons' VxlanManager maps (daemon/vxlan/manager.go:14-17):
 * entry i says: on the node whose HOST_IP is kdict id node[i], VNI vni[i] is held
 * by netns kdict id net_ns[i]. Keys (node, vni) must be unique (first wins). */
typedef struct kdtn_vni_table {
    uint32_t        n;
    const uint32_t* node;
    const int32_t*  vni;
    const uint32_t* net_ns;
} kdtn_vni_table;

/* kdtn_epoch_in.vnis.n = KDTN_VNI_RESIDENT: use the context's resident map (the last uploaded
 * snapshot, or the state kdtn_epoch_vni_apply left) instead of uploading one. Its ids must still
 * name the same strings, so the upload must keep (kdict_keep) at least the dictionary the map
 * was made for; KDTN_EINVAL otherwise, and always for kdtn_json_ingest (the engine interns
 * that dictionary itself). The snapshot an upload starts from stays its epoch-start map: a
 * re-run of the same upload after kdtn_epoch_vni_apply decides vni_hit as the first run did. */
#define KDTN_VNI_RESIDENT 0xFFFFFFFFu

typedef struct kdtn_epoch_in {
    kdtn_strtab     kdict;      /* key strings: names, namespaces, intfs, IPs, MACs, src_ip, net_ns */
    kdtn_strtab     pdict;      /* LinkProperties strings                               */
    kdtn_topo_table topos;
    kdtn_link_table realised;   /* status.links of every topology, grouped             */
    kdtn_link_table desired;    /* spec.links of every topology, grouped               */
    kdtn_vni_table  vnis;
    uint32_t        pod_slice;  /* multi-GPU: pod-table entries per rank (>= topos.n); 0 = topos.n */
    /* Append-only interning across epochs: the first kdict_keep (pdict_keep) strings are
     * byte-identical to the previous upload's on this context, whose parsed tables (MakeVeth /
     * addLink predicates, ParseDuration / ParseFloatPercentage / ParseRate results) are kept:
     * only the new suffix is uploaded and each kdtn_epoch_run parses only the strings this
     * upload added. 0 = upload and parse the whole dictionary. KDTN_EINVAL when the prefix was
     * not parsed on this context (no run since an upload that kept fewer strings, or the
     * arena offsets disagree). */
    uint32_t        kdict_keep, pdict_keep;
} kdtn_epoch_in;

/* Property sets for the standalone kdtn_make_qdiscs (daemon UpdateLinks path). */
typedef struct kdtn_props_table {
    uint32_t        n;
    const uint32_t* prop[KDTN_NPROP];
    const uint32_t* gap;
} kdtn_props_table;

/* ---- outputs ---------------------------------------------------------------------- */
/* MakeQdiscs result (common/qdisc.go:20-126 + netlink.NewNetem). 72 bytes.
 * err != 0  ⇔ MakeQdiscs returned (nil, err): every other field is 0.
 * has_netem == 0 && err == 0  ⇔ empty properties (proto.Size == 0): empty list. */
typedef struct kdtn_qdisc {
    uint32_t latency;        /* time2Tick(latency µs)                                  */
    uint32_t delay_corr;     /* P2U(latency_corr) if latency µs > 0 && jitter µs > 0   */
    uint32_t limit;          /* 1000                                                   */
    uint32_t loss;           /* P2U(loss)                                              */
    uint32_t loss_corr;      /* P2U(loss_corr) if loss > 0                             */
    uint32_t gap;            /* Gap, or 1 if reorder_prob > 0 && Gap == 0              */
    uint32_t duplicate;      /* P2U(duplicate)                                         */
    uint32_t duplicate_corr; /* P2U(duplicate_corr) if duplicate > 0                   */
    uint32_t jitter;         /* time2Tick(jitter µs) if latency ticks > 0 else µs      */
    uint32_t reorder_prob;
    uint32_t reorder_corr;
    uint32_t corrupt_prob;
    uint32_t corrupt_corr;
    uint32_t tbf_buffer;     /* getTbfBurst(rate) common/qdisc.go:361-370              */
    uint64_t tbf_rate;       /* ParseRate, bit/s                                       */
    uint32_t tbf_minburst;   /* 1500                                                   */
    uint8_t  has_netem;
    uint8_t  has_tbf;        /* rate != 0                                              */
    uint8_t  err;            /* kdtn_err (qdisc steps only)                            */
    uint8_t  reserved;
} kdtn_qdisc;

/* Pure-prefix outcome of addLink / delLink / UpdateLinks for one batch entry. 16 bytes. */
typedef struct kdtn_resolved {
    uint32_t peer_topo;  /* global pod index of the peer Topology (lookup succeeded), else 0xFFFFFFFF */
    int32_t  vni;        /* GetVniFromUid(uid) = int32(vxlan_base + uid)                   */
    uint32_t vtep;       /* CROSS_NODE: kdict id of peer status.src_ip; PHYSICAL: kdict id of
                            peer_pod (vtep = bytes[9:]); else 0                             */
    uint8_t  kind;       /* kdtn_kind (add entries)                                        */
    uint8_t  err;        /* kdtn_err: first failing step before the first syscall. For add
                            SAME/CROSS/PHYSICAL the qdisc error is in kdtn_qdisc.err.  For
                            update entries: MakeVeth error, else the MakeQdiscs error.        */
    uint8_t  vni_hit;    /* del: VxlanManager.Get(vni) == local net_ns (handler.go:482-486);
                            add PHYSICAL: local VNI map holds vni for another netns
                            (handler.go:177-179); add CROSS_NODE: same check on the peer's node */
    uint8_t  remote_err; /* add CROSS_NODE: KDTN_E_REMOTE_CIDR when the RemotePod this link sends
                            is rejected by the peer daemon (link.PeerIp set and not a CIDR). The
                            link's local steps run (VXLAN, qdiscs, RPC sent), then addLink returns
                            the error and the batch aborts after this link.                    */
} kdtn_resolved;

/* Epoch outputs, caller-owned host memory. Any pointer may be NULL (not returned).
 * Batches are per Topology: entries of topology t are [off[t], off[t+1]) of each list,
 * in the reference's order (del/upd: status order; add: spec order). */
typedef struct kdtn_batches {
    uint8_t*        action;          /* [T] kdtn_action                                  */
    uint32_t*       del_off;         /* [T+1]                                            */
    uint32_t*       add_off;         /* [T+1]                                            */
    uint32_t*       upd_off;         /* [T+1]                                            */
    uint32_t*       del_idx;         /* realised record index of each DelLinks entry     */
    uint32_t*       add_idx;         /* desired record index of each AddLinks entry      */
    uint32_t*       upd_idx;         /* desired record index of each UpdateLinks entry   */
    kdtn_resolved*  del_res;
    kdtn_resolved*  add_res;
    kdtn_resolved*  upd_res;
    kdtn_qdisc*     add_qdisc;
    kdtn_qdisc*     upd_qdisc;
    uint32_t        del_cap, add_cap, upd_cap;   /* in: entry capacities                */
    uint32_t        n_del, n_add, n_upd;         /* out: entry counts                   */
} kdtn_batches;

typedef struct kdtn_counts { uint32_t n_del, n_add, n_upd, n_topos; } kdtn_counts;

/* Epoch stages (bitmask for kdtn_epoch_run). */
#define KDTN_STAGE_DIFF    0x1u   /* gate + CalcDiff + batch lists                     */
#define KDTN_STAGE_RESOLVE 0x2u   /* MakeVeth + addLink classification + VNI           */
#define KDTN_STAGE_QDISC   0x4u   /* MakeQdiscs for add ∪ update entries                */
#define KDTN_STAGE_ALL     0x7u

/* One context drives one GPU, and one process (rank) drives one context: SURVEY §8(b)'s
 * num_gpus / device-id list / capacities are deliberately not fields here. A controller
 * over G GPUs runs G ranks (kdtn_comm_init / kdtn_comm_set_ranks) and routes each Topology
 * with kdtn_topology_shard; buffers are sized from each upload (and grow with headroom), so
 * there is no capacity to declare up front. */
typedef struct kdtn_config {
    int32_t  device;         /* HIP device ordinal; -1 = current device                */
    int32_t  vxlan_base;     /* common/constants.go:8 VxlanBase (5000)                  */
    double   tick_in_usec;   /* netlink initClock from /proc/net/psched (15.625 typical);
                                0 reproduces an unreadable psched (time2Tick == 0)      */
} kdtn_config;

typedef struct kdtn_ctx kdtn_ctx;
typedef struct kdtn_interner kdtn_interner;

/* ---- lifecycle -------------------------------------------------------------------- */
const char* kdtn_version(void);
const char* kdtn_strerror(int code);
const char* kdtn_err_name(int kdtn_err_code);
int  kdtn_init(kdtn_ctx** out, const kdtn_config* cfg);
void kdtn_destroy(kdtn_ctx* ctx);
/* Run on a caller-provided hipStream_t (passed as void*); NULL restores the ctx stream. */
int  kdtn_set_stream(kdtn_ctx* ctx, void* hip_stream);
/* Reads /proc/net/psched like netlink initClock(); returns 0.0 if unreadable. */
double kdtn_psched_tick_in_usec(void);

/* ---- host string interning (deduplicated dictionaries, id 0 = "") ----------------- */
int      kdtn_interner_new(kdtn_interner** out);
void     kdtn_interner_free(kdtn_interner* it);
uint32_t kdtn_intern(kdtn_interner* it, const char* s, uint32_t len);
int      kdtn_intern_batch(kdtn_interner* it, const uint8_t* bytes, const uint64_t* offs,
                           uint32_t n, uint32_t* ids_out);
/* View of the dictionary; valid until the next kdtn_intern* call on it. */
int      kdtn_interner_table(const kdtn_interner* it, kdtn_strtab* out);

/* ---- reconcile epoch (CalcDiff + resolve + MakeQdiscs over all topologies) --------- */
/* One synchronous call: upload, run KDTN_STAGE_ALL, download into `out`.               */
int kdtn_reconcile_epoch(kdtn_ctx* ctx, const kdtn_epoch_in* in, kdtn_batches* out);
/* Split form (device-resident inputs reused across epochs):                             */
int kdtn_epoch_upload(kdtn_ctx* ctx, const kdtn_epoch_in* in);
int kdtn_epoch_run(kdtn_ctx* ctx, uint32_t stages);          /* async on the ctx stream   */
int kdtn_epoch_sync(kdtn_ctx* ctx, kdtn_counts* counts);     /* waits; counts may be NULL */
int kdtn_epoch_download(kdtn_ctx* ctx, kdtn_batches* out);   /* after run (+ sync)         */
/* The download and every output stage below size their work from the run's list totals: after
 * kdtn_epoch_sync they are at hand; without it the call waits for the run and reads them (an
 * output stage never uses an earlier epoch's counts). Destinations that are page-locked —
 * kdtn_host_alloc, or host memory registered with hipHostRegister / hsa_amd_memory_lock — are
 * written by an SDMA engine (a registered range at its agent address), others by hipMemcpy.
 * Asynchronous download (after sync): the copies into `out` (page-locked, kdtn_host_alloc) run
 * on a stream of their own while the caller goes on (commit, the next kdtn_epoch_upload_delta,
 * whose host-to-device copies share the full-duplex link); the next kdtn_epoch_run waits for
 * them on the GPU before overwriting the outputs. Counts in `out` are set at return; the
 * arrays are valid after kdtn_epoch_download_wait. */
int kdtn_epoch_download_async(kdtn_ctx* ctx, kdtn_batches* out);
int kdtn_epoch_download_wait(kdtn_ctx* ctx);

/* Gate + CalcDiff only (KDTN_STAGE_DIFF): the Del/Add/Update index lists per Topology,
 * without resolve or qdisc records (out->*_res / *_qdisc are not written). Replaces
 * CalcDiff (controllers/topology_controller.go:288-318) and the gate (:77-88). */
int kdtn_diff(kdtn_ctx* ctx, const kdtn_epoch_in* in, kdtn_batches* out);

/* ---- daemon side: one LinksBatchQuery (daemon/kubedtn/handler.go:592-632) --------- */
/* The informer's pods as the daemon sees them (getPod, handler.go:27-41; ToProtoPod
 * :62-88): namespace, name, status src_ip / net_ns, KDTN_TOPO_SPEC_NIL when the pod's
 * spec.links is nil (ToProtoPod's error). */
typedef struct kdtn_pod_table {
    uint32_t        n;
    const uint32_t* ns;
    const uint32_t* name;
    const uint32_t* src_ip;
    const uint32_t* net_ns;
    const uint8_t*  flags;
} kdtn_pod_table;
#define KDTN_BATCH_ADD 0   /* AddLinks: addLink per link (handler.go:592-611, 316-459)   */
#define KDTN_BATCH_DEL 1   /* DelLinks: delLink per link (handler.go:613-632, 461-492)   */
/* Pure prefix of the daemon batch handler for the links of LocalPod = pods[local]:
 * out[i] is link i's plan (kind, peer, VNI, VXLAN map check, first failing step) and,
 * for AddLinks, qout[i] its MakeQdiscs result (qout may be NULL; ignored for DelLinks).
 * The handler aborts at the first link whose err != 0 (kdtn_resolved.err or qout.err).
 * A link whose peer is the local pod itself sees the local pod's spec as non-nil. */
int kdtn_resolve(kdtn_ctx* ctx, const kdtn_strtab* kdict, const kdtn_strtab* pdict,
                 const kdtn_pod_table* pods, uint32_t local, const kdtn_link_table* links,
                 int batch_kind, const kdtn_vni_table* vnis, kdtn_resolved* out, kdtn_qdisc* qout);

/* Pinned host memory for inputs/outputs (optional: faster H2D/D2H than pageable). */
void* kdtn_host_alloc(uint64_t bytes);
void  kdtn_host_free(void* p);

/* ---- standalone MakeQdiscs over a batch of property sets (UpdateLinks path) -------- */
int kdtn_make_qdiscs(kdtn_ctx* ctx, const kdtn_strtab* pdict, const kdtn_props_table* props,
                     kdtn_qdisc* out);

/* ---- resident epoch state: status commit and delta upload ----------------------------
 * Reconcile ends with Status.Links = Spec.Links for a Topology it saw for the first time
 * (CREATED) or whose DelLinks / AddLinks / UpdateLinks RPCs all succeeded; a failed RPC
 * returns before the status write (controllers/topology_controller.go:81-85, 93-116, 125-138).
 * kdtn_epoch_commit applies that to the context's resident link stores on the GPU: the
 * realised store (status.links) becomes, per Topology, its desired segment when committed,
 * else its old realised segment (KDTN_TOPO_STATUS_NIL follows: a nil spec commits a nil
 * status). mask = NULL commits what the engine predicts (CREATED, and DIFF Topologies none
 * of whose batch entries fails — the kdtn_epoch_fanout reach rule; needs a run with RESOLVE
 * and QDISC); else mask[t] != 0 commits Topology t (the caller saw its RPCs and status
 * update succeed). Call the output stages (encode, fanout, tc, remote, vni_apply) first:
 * after a commit the context needs a run. n_committed (may be NULL) = committed Topologies. */
int kdtn_epoch_commit(kdtn_ctx* ctx, const uint8_t* mask, uint32_t* n_committed);

/* The next epoch's inputs as a delta against the context's resident state (the status
 * after kdtn_epoch_commit, the previous desired store, the topology rows): only the
 * Topologies whose spec (or status.src_ip / status.net_ns) changed, and for each of them its
 * new spec.links as references — a record of the previous desired store by index, or
 * KDTN_DELTA_NEW | k for inline record k of `records`.
 * Dictionaries: a delta EXTENDS the resident dictionaries (append-only interning): kdict_keep
 * and pdict_keep must equal the context's dictionary sizes (the resident records' ids stay
 * valid), only the suffix is uploaded; KDTN_EINVAL otherwise (a shrunk or rewritten
 * dictionary needs kdtn_epoch_upload).
 * Topology set (informer add / delete events: a Topology CR created — the Reconcile CREATED
 * path, controllers/topology_controller.go:81-85 — or deleted): prev == NULL keeps the set.
 * Otherwise the new table has n_topos Topologies and prev[t] names the previous index of new
 * Topology t (each at most once, any order), or is KDTN_DELTA_NEW for a Topology this delta
 * creates: a created Topology must be listed in topo[] (its spec), takes metadata ns / name
 * from ns[] / name[] at its changed-list position, and its status.links are nil (a new CR has
 * no status). Previous Topologies no prev[t] names are deleted with their spec and status.
 * topo[] indices are new-table indices. pod_slice as kdtn_epoch_in (0 = n_topos); the pod
 * tables are rebuilt by the next run.
 * Validation runs on the GPU with one host synchronisation per call; a rejected delta
 * (KDTN_EINVAL) leaves the resident state as it was (a new run is needed). */
#define KDTN_DELTA_NEW 0x80000000u
typedef struct kdtn_epoch_delta {
    kdtn_strtab     kdict, pdict;
    uint32_t        kdict_keep, pdict_keep;
    uint32_t        n_changed;
    const uint32_t* topo;       /* [n_changed] strictly ascending topology indices            */
    const uint32_t* src_ip;     /* [n_changed] status.src_ip (kdict id)                        */
    const uint32_t* net_ns;     /* [n_changed] status.net_ns                                   */
    const uint8_t*  spec_nil;   /* [n_changed] 1: spec.links nil (no records)                  */
    const uint32_t* des_off;    /* [n_changed + 1] offsets into ref                            */
    const uint32_t* ref;        /* [des_off[n_changed]] previous desired record | NEW-tagged   */
    kdtn_link_table records;    /* inline records                                              */
    kdtn_vni_table  vnis;       /* VxlanManager snapshot or KDTN_VNI_RESIDENT                  */
    /* Topology set changes (prev == NULL: unchanged; the fields below are then ignored)      */
    uint32_t        n_topos;    /* new T                                                       */
    const uint32_t* prev;       /* [n_topos] previous index, or KDTN_DELTA_NEW (created)       */
    const uint32_t* ns;         /* [n_changed] metadata.namespace (read for created ones)      */
    const uint32_t* name;       /* [n_changed] metadata.name      (read for created ones)      */
    uint32_t        pod_slice;  /* multi-GPU pod-table entries per rank; 0 = n_topos           */
} kdtn_epoch_delta;
int kdtn_epoch_upload_delta(kdtn_ctx* ctx, const kdtn_epoch_delta* delta);

/* ---- wire encoding of the batches (proto/v1 LinksBatchQuery) ------------------------ */
/* The request bodies Reconcile sends after CalcDiff: for topology t and list l (0 DelLinks,
 * 1 AddLinks, 2 UpdateLinks) the bytes of proto.Marshal(&pb.LinksBatchQuery{LocalPod:
 * &pb.Pod{Name, SrcIp, NetNs, KubeNs}, Links: common.Map(links, Link.ToProto)})
 * (controllers/topology_controller.go:180-188, 223-231, 266-274;
 * api/v1/topology_types.go:97-109,178-194). Arena regions del | add | upd, topology order:
 * batch (l, t) = bytes[off[l*T + t], off[l*T + t + 1]); empty when the list is empty (no
 * RPC) or when Marshal fails on a string that is not valid UTF-8 (err[t] bit l).      */
typedef struct kdtn_wire {
    uint8_t*  bytes;        /* [cap] arena                                               */
    uint64_t  cap;          /* in: arena capacity                                        */
    uint64_t* off;          /* [3T+1] batch byte offsets                                 */
    uint32_t* err;          /* [T] bit l: list l of the topology failed to marshal        */
    uint64_t  n_bytes;      /* out: arena bytes used                                     */
} kdtn_wire;
/* After kdtn_epoch_run (any stages) + kdtn_epoch_sync: encode every batch on the GPU;
 * returns the arena size through n_bytes. Synchronous. */
int kdtn_epoch_encode(kdtn_ctx* ctx, uint64_t* n_bytes);
int kdtn_epoch_download_wire(kdtn_ctx* ctx, kdtn_wire* out);

/* ---- which batch entries the daemons reach ------------------------------------------- */
/* Reconcile sends a topology's batches in the order DelLinks, AddLinks, UpdateLinks and
 * stops at the first RPC that fails (controllers/topology_controller.go:93-116); each daemon
 * handler stops at its first failing link (daemon/kubedtn/handler.go:601-607, 622-628,
 * 644-662). An entry is REACHED when no earlier entry of its list and no entry of an
 * earlier list of its topology failed. A link fails when: del — kdtn_resolved.err; add —
 * kdtn_resolved.err, or its qdisc err for the kinds that build qdiscs (SAME_NODE,
 * CROSS_NODE, PHYSICAL), or kdtn_resolved.remote_err (after its own local steps); update —
 * kdtn_resolved.err. kdtn_epoch_fanout and kdtn_epoch_tc apply this rule.             */

/* ---- RemotePod fan-out grouped per destination daemon ------------------------------ */
/* The UpdateRemote RPCs the daemons would send for this epoch's AddLinks batches
 * (daemon/kubedtn/handler.go:419-453, common/utils.go:39-67): an entry sends one when it is
 * REACHED, CROSS_NODE and its qdisc was built (SetupVxLan → MakeQdiscs fails first). The
 * reference sends one RPC per link;
 * here they are grouped per destination daemon (peer status.src_ip = kdtn_resolved.vtep):
 * node[k] = kdict id of daemon k (ascending), its entries idx[off[k] .. off[k+1]) are
 * add-list entry indices in add-list order. Requires a run with RESOLVE and QDISC. */
typedef struct kdtn_fanout {
    uint32_t* node;          /* [node_cap]                                            */
    uint32_t* off;           /* [node_cap + 1]                                        */
    uint32_t* idx;           /* [idx_cap]                                             */
    uint32_t  node_cap, idx_cap;
    uint32_t  n_nodes, n_send;   /* out                                               */
} kdtn_fanout;
int kdtn_epoch_fanout(kdtn_ctx* ctx, kdtn_fanout* out);

/* ---- RemotePod messages (proto/v1 RemotePod, kube_dtn.proto:65-79) ------------------- */
/* The request bodies of the Remote.Update calls the epoch's AddLinks make, marshalled on the
 * GPU so a daemon hands pre-encoded bytes to its gRPC stream (a raw codec) instead of
 * building and marshalling one RemotePod per link:
 *   - messages [0, n_remote): UpdateRemote (common/utils.go:39-67) of every add entry that
 *     sends one — exactly kdtn_epoch_fanout's senders, in its order (destination daemons
 *     ascending, add-list order within), so daemon k's stream is messages
 *     [fanout.off[k], fanout.off[k+1]). Payload {NetNs: peer status.net_ns, IntfName:
 *     link.PeerIntf, IntfIp: link.PeerIp, PeerVtep: local status.src_ip, Vni, KubeNs: local
 *     namespace, Properties: link.Properties, Name: link.PeerPod} (utils.go:42-51);
 *   - messages [n_remote, n_msgs): the local Update a PHYSICAL peer makes the daemon run on
 *     itself (daemon/kubedtn/handler.go:348-371) for every reached PHYSICAL add entry whose
 *     MakeVeth passed, add-list order: {NetNs: local status.net_ns, IntfName: link.LocalIntf,
 *     IntfIp: link.LocalIp, PeerVtep: PeerPod without "physical/", Vni, KubeNs, Properties,
 *     Name: link.PeerPod}.
 * Message m = bytes[off[m], off[m+1]): varint length + RemotePod (a delimited stream); empty
 * when a string is not valid UTF-8 (proto.Marshal fails). entry[m] = its add-list entry.
 * Beside each remote message, the receiving daemon's SetVethQdiscs argv for IntfName
 * (Update → SetupVxLan → MakeQdiscs → SetVethQdiscs, daemon/vxlan/vxlan.go:31-51; same
 * format as kdtn_epoch_tc) = tc_bytes[tc_off[m], tc_off[m+1]): present when the link has a
 * TBF and the peer's CreateOrUpdate accepts IntfIp (remote_err == 0); physical messages
 * have none here (their tc is kdtn_epoch_tc's slot 2e). Needs a run with RESOLVE and QDISC.
 * Called after kdtn_epoch_encode of the same run, it copies each message's Properties field
 * from its AddLinks entry's Link bytes (the same pb.LinkProperties field 7) instead of
 * re-encoding the property strings; the bytes are the same either way. */
typedef struct kdtn_remote_info {
    uint32_t n_msgs, n_remote;
    uint64_t n_bytes, n_tc_bytes;
} kdtn_remote_info;
typedef struct kdtn_remote_pods {
    uint8_t*  bytes;    uint64_t cap;          /* [n_bytes] messages                          */
    uint64_t* off;                             /* [n_msgs + 1]                                */
    uint32_t* entry;                           /* [n_msgs] add-list entry of each message     */
    uint8_t*  tc_bytes; uint64_t tc_cap;       /* [n_tc_bytes] receiving daemon's tc argv     */
    uint64_t* tc_off;                          /* [n_msgs + 1]                                */
    uint32_t  msg_cap;                         /* capacity of off / entry / tc_off (messages) */
} kdtn_remote_pods;
int kdtn_epoch_remote_encode(kdtn_ctx* ctx, kdtn_remote_info* info);      /* after run + sync */
int kdtn_epoch_download_remote(kdtn_ctx* ctx, kdtn_remote_pods* out);

/* ---- tc argv of the TBF qdiscs -------------------------------------------------------- */
/* SetVethQdiscs (common/qdisc.go:252-266) applies the TBF by exec'ing
 *   tc qdisc add dev <LinkName> parent 1:1 handle 10:0 tbf rate <Rate> burst <Buffer>
 *      latency 50ms minburst <Minburst>
 * inside the interface's netns. For every REACHED AddLinks / UpdateLinks entry whose plan
 * has no error and whose MakeQdiscs produced a TBF this writes that argv (arguments
 * NUL-terminated, without the leading "tc"). Command slots: add entry e has two, 2e for
 * link.LocalIntf (UpdateLinks' veth, the local VXLAN, or the local end of a veth pair) and
 * 2e+1 for link.PeerIntf in the peer pod's netns (SAME_NODE only: CreateVeth sets the
 * qdiscs on both ends, common/veth.go:53-60); update entry u has one, slot 2*n_add + u, for
 * link.LocalIntf. Slot g = bytes[off[g], off[g+1]), empty = no tc command. */
typedef struct kdtn_tc_argv {
    uint8_t*  bytes;
    uint64_t  cap;
    uint64_t* off;           /* [2*n_add + n_upd + 1] command slots                   */
    uint64_t  n_bytes;       /* out                                                    */
} kdtn_tc_argv;
int kdtn_epoch_tc(kdtn_ctx* ctx, uint64_t* n_bytes);   /* after run(QDISC|RESOLVE) + sync */
int kdtn_epoch_download_tc(kdtn_ctx* ctx, kdtn_tc_argv* out);

/* ---- CR ingest: TopologyList JSON → device-resident epoch tables ---------------------- */
/* The step before the diff: the controller's informer lists the
 * Topology CRs as a Kubernetes `TopologyList` JSON document and decodes it with
 * sigs.k8s.io/json (apimachinery v0.24, case-sensitive keys) into the typed structs of
 * api/v1/topology_types.go:28-56,59-95,119-176. kdtn_json_ingest performs that decode on
 * the GPU and leaves the result where kdtn_epoch_upload would: interned dictionaries
 * (ids in first-occurrence document order, id 0 = ""), the topology table (items order;
 * metadata.namespace/name, status.src_ip/net_ns, KDTN_TOPO_*_NIL when a links list is
 * absent or null) and both link stores (spec.links = desired, status.links = realised),
 * so kdtn_epoch_run follows with no host SoA build or table upload.
 * Decoding follows Go's encoding/json: full syntax validation first (checkValid,
 * nesting ≤ 10000), string escapes and \u surrogate pairs, invalid UTF-8 coerced to
 * U+FFFD, null leaves a field unchanged (a links list nil), null array elements decode
 * to zero values, uid via ParseInt(·,10,64), gap via ParseUint into uint32, unknown
 * fields skipped. Documented deviations: a schema field repeated inside one object
 * (Go: last wins) is reported as KDTN_JSON_DUPKEY (decode such a document on the host),
 * and fields outside the path (metadata other than name/namespace, status.skipped,
 * apiVersion, kind) are skipped without type checks. */
typedef enum kdtn_json_err {
    KDTN_JSON_OK = 0,
    KDTN_JSON_SYNTAX = 1,   /* not valid JSON (json.SyntaxError)                                */
    KDTN_JSON_DEPTH = 2,    /* nesting deeper than 10000 (scanner maxNestingDepth)              */
    KDTN_JSON_TYPE = 3,     /* json.UnmarshalTypeError on a schema field (wrong JSON type,
                               uid not an int64 literal, gap not a uint32 literal)              */
    KDTN_JSON_DUPKEY = 4    /* a schema field repeated in one object (host fallback)            */
} kdtn_json_err;

typedef struct kdtn_ingest_info {
    uint32_t n_topos, n_desired, n_realised;   /* T, N (spec.links), M (status.links)     */
    uint32_t n_kdict, n_pdict;                 /* dictionary sizes (including id 0 = "")  */
    int32_t  json_err;                         /* kdtn_json_err                           */
    uint64_t err_offset;                       /* byte offset of an error (best effort)   */
    uint64_t n_tokens;                         /* JSON tokens in the document             */
    uint64_t kdict_bytes, pdict_bytes;         /* dictionary arena sizes                  */
} kdtn_ingest_info;

/* Host copies of the decoded tables (caller-owned, sized from kdtn_ingest_info; any NULL
 * pointer is skipped). Link columns are SoA: key column k of record i at key[k*n + i]. */
typedef struct kdtn_ingest_tables {
    uint8_t*  kd_bytes;  uint32_t* kd_offs;    /* [kdict_bytes], [n_kdict + 1]            */
    uint8_t*  pd_bytes;  uint32_t* pd_offs;
    uint32_t* ns; uint32_t* name; uint32_t* src_ip; uint32_t* net_ns;   /* [T]            */
    uint8_t*  flags;                            /* [T]                                      */
    uint32_t* real_off; uint32_t* des_off;      /* [T + 1]                                  */
    uint32_t* des_key; uint32_t* des_prop; uint32_t* des_gap; int64_t* des_uid;
    uint32_t* real_key; uint32_t* real_prop; uint32_t* real_gap; int64_t* real_uid;
} kdtn_ingest_tables;

#define KDTN_EBADMSG (-74)   /* the JSON document was rejected: kdtn_ingest_info.json_err */

/* H2D of the document (< 4 GiB) into the context's HBM. */
int kdtn_json_upload(kdtn_ctx* ctx, const uint8_t* doc, uint64_t n);
/* Decode the uploaded document on the GPU into the epoch inputs (synchronous). vnis:
 * VxlanManager snapshot (NULL = empty), with ids in the document's kdict: strings not in
 * the document cannot be referenced, so a snapshot is given as kdict ids of the result of
 * a previous ingest of the same document shape. Single-shard contexts only (nranks == 1;
 * a rank of several uses kdtn_json_ingest_shard).
 * Returns KDTN_OK, KDTN_EBADMSG (info->json_err says why) or an engine error. */
int kdtn_json_ingest(kdtn_ctx* ctx, const kdtn_vni_table* vnis, kdtn_ingest_info* info);
/* D2H of the decoded tables of the last successful ingest. */
int kdtn_ingest_download(kdtn_ctx* ctx, kdtn_ingest_tables* out);
/* Incremental CR ingest on the resident state (the informer's event stream,
 * daemon/kubedtn/kubedtn.go:128-142; a controller that keeps the engine resident no longer
 * re-decodes its whole store): the uploaded document (kdtn_json_upload) is a TopologyList of
 * the Topology CRs added or updated since the resident state, deleted[] the resident table
 * indices of the deleted ones. The document is decoded as by kdtn_json_ingest into scratch
 * tables, its strings are interned into the RESIDENT dictionaries on the GPU (a string already
 * there keeps its id, so the resident link stores and the resident VXLAN map stay valid; new
 * strings are appended in first-occurrence order), and the result is applied as
 * kdtn_epoch_upload_delta would: an item whose (namespace, name) is resident replaces that
 * Topology's spec.links and status.src_ip / net_ns (status.links stay the engine's committed
 * status); any other item is a created Topology (status nil: the CREATED path,
 * controllers/topology_controller.go:81-85); deleted Topologies leave the table. The new table
 * keeps the remaining resident rows in order and appends the created ones in document order.
 * vnis: a VXLAN snapshot in resident ids, NULL = KDTN_VNI_RESIDENT. info: the new table's sizes
 * and the document's token count. KDTN_EBADMSG (info->json_err) for a rejected document and
 * KDTN_EINVAL (an item listed twice, deleted and listed, a deleted index out of range) leave
 * the resident state as it was. Single-shard contexts; needs a run since the last upload (the
 * resident dictionaries parsed). */
int kdtn_json_ingest_delta(kdtn_ctx* ctx, const uint32_t* deleted, uint32_t n_deleted, const kdtn_vni_table* vnis,
                           kdtn_ingest_info* info);
/* Sizes of the context's current epoch tables — after an upload, a delta upload, a commit
 * or an ingest — into info (n_topos, n_desired, n_realised, dictionary sizes); after it,
 * kdtn_ingest_download returns those tables (the resident state after a commit). */
int kdtn_epoch_tables_info(kdtn_ctx* ctx, kdtn_ingest_info* info);

/* Sharded ingest for one rank of nshards (SURVEY §8(e) with §8(f) rank 2). Every controller
 * replica's informer holds the whole Topology store (the controller watches all Topologies,
 * controllers/topology_controller.go:332-339), so every rank decodes the WHOLE TopologyList:
 * dictionary ids are then identical on every rank (first occurrence in one document) and
 * each rank fills the pod-status row of every Topology itself — no exchange. The epoch is
 * cut down on the GPU to the Topologies this rank owns (kdtn_topology_shard(namespace,
 * name, nshards) == shard, document order kept; topology table and both link stores
 * compacted), and peers are reported as document indices (kdtn_resolved.peer_topo = the
 * unsharded topology index). Leaves the context as rank `shard` of `nshards` with its pod
 * table in place, so kdtn_epoch_run follows directly (the next kdtn_epoch_upload or ingest
 * restores the rank setup the context had before). info: the shard's n_topos /
 * n_desired / n_realised and the document's dictionaries; kdtn_ingest_download returns the
 * shard's tables. A context with an RCCL communicator is refused. */
int kdtn_json_ingest_shard(kdtn_ctx* ctx, const kdtn_vni_table* vnis, uint32_t nshards, uint32_t shard,
                           kdtn_ingest_info* info);
/* Document index of each of the last ingest's topologies ([info.n_topos]; the identity
 * after an unsharded ingest). */
int kdtn_ingest_shard_topos(kdtn_ctx* ctx, uint32_t* doc_index);

/* ---- multi-GPU (one process per GPU) ---------------------------------------------------- */
/* Owner shard of a Topology: hash64(namespace ‖ "/" ‖ name) mod nshards (SURVEY.md §8(e);
 * the key is the informer's object key, cache.MetaNamespaceKeyFunc). A controller routes
 * each Topology (both its spec and status links) to the context of rank
 * kdtn_topology_shard(...), keeping informer order within a shard, so CalcDiff, resolve and
 * MakeQdiscs are shard-local; the batches of the shards are disjoint sets of Topologies.
 * Host-only: no GPU call. */
uint32_t kdtn_topology_shard(const uint8_t* ns, uint32_t ns_len, const uint8_t* name, uint32_t name_len,
                             uint32_t nshards);

/* The one exchange: peer resolution (getPod + ToProtoPod, daemon/kubedtn/handler.go:375-399)
 * needs the pod-status row of every Topology of every shard. Rank r's topologies occupy the
 * global pod indices [r*pod_slice, r*pod_slice + T_r) — kdtn_resolved.peer_topo is such an
 * index — so every rank uploads the same kdtn_epoch_in.pod_slice (>= its T) and uses the
 * same kdict ids for pod names, namespaces, src_ip and net_ns strings (one shared
 * interner prefix). Transports:
 *   RCCL (production): kdtn_comm_init; kdtn_epoch_run all-gathers the rows over xGMI on a
 *     comm stream, overlapped with the dictionary parses (nranks == 1 also builds a
 *     one-rank communicator, so the RCCL path runs on a single GPU).
 *   host (any collective library, e.g. gloo): kdtn_comm_set_ranks; per epoch, after
 *     kdtn_epoch_upload: kdtn_pods_export → all-gather of pod_slice rows per rank in rank
 *     order → kdtn_pods_import → kdtn_epoch_run (KDTN_EINVAL if the import is missing). */
typedef struct kdtn_pod_row {
    uint32_t ns, name, src_ip;  /* kdict ids; padding rows (T_r <= i < pod_slice) have ns = name = ~0 */
    uint32_t net_ns_nil;        /* kdict id of status.net_ns | KDTN_TOPO_SPEC_NIL-derived bit 31   */
} kdtn_pod_row;
int kdtn_comm_unique_id(uint8_t out[128]);
int kdtn_comm_init(kdtn_ctx* ctx, const uint8_t unique_id[128], int nranks, int rank);
int kdtn_comm_set_ranks(kdtn_ctx* ctx, int nranks, int rank);          /* host transport */
int kdtn_pods_export(kdtn_ctx* ctx, kdtn_pod_row* rows);                /* [pod_slice] rows */
int kdtn_pods_import(kdtn_ctx* ctx, const kdtn_pod_row* rows, uint64_t n);   /* n = pod_slice*nranks */

/* ---- getPod's API-server fallback (daemon/kubedtn/handler.go:27-41) -------------------
 * getPod reads the informer store and, on a miss, GETs the Topology from the API server
 * (m.tClient.Topology(ns).Get). The engine resolves peers against the uploaded table only: a
 * peer absent from it is KDTN_E_PEER_LOOKUP in kdtn_resolved.err. The driver contract:
 *   1. after kdtn_epoch_sync / download, list the AddLinks entries with err ==
 *      KDTN_E_PEER_LOOKUP; each names the key (topology namespace, or "default" when empty;
 *      link.PeerPod) — handler.go:375 getPod(ctx, link.PeerPod, localPod.KubeNs);
 *   2. GET each distinct key; a key the API server does not have stays a miss (the
 *      reference returns that GET's error, which is the same failing step);
 *   3. intern the fetched Topologies' status.src_ip / net_ns strings (a dictionary that
 *      grows goes up first as a kdtn_epoch_upload_delta with n_changed = 0 and
 *      kdict_keep = the resident size), then pass their pod rows here;
 *   4. kdtn_epoch_run + sync + download again, and only then take each batch's first error.
 * The late rows join the peer lookup of every following run as global pod indices
 * nranks*pod_slice + i (kdtn_resolved.peer_topo; the downstream stages read their rows like
 * any other pod's), after the gathered table, so a key the table already holds keeps its
 * table row (the informer store wins, as in getPod). They belong to no batch. Every rank of
 * a sharded run passes the same rows. Cleared by the next kdtn_epoch_upload, upload_delta,
 * JSON ingest or kdtn_epoch_commit. Ids must be below the resident kdict size (KDTN_EINVAL). */
int kdtn_epoch_late_pods(kdtn_ctx* ctx, const kdtn_pod_row* rows, uint32_t n);

/* ---- VxlanManager state after the epoch ---------------------------------------------
 * Replaces the daemons' map mutations (daemon/vxlan/manager.go:57-63 Add / Delete, called at
 * daemon/kubedtn/handler.go:192 remote/physical Update, :440 cross-node addLink, :484-487
 * delLink) for the entries the daemons reach (as kdtn_epoch_fanout defines them): a delete
 * for each reached DelLinks entry whose vni_hit is set (before its first MakeVeth error);
 * for each reached AddLinks entry without error, Store(vni, local netns) on the local node
 * (cross-node and physical peers) and, for cross-node ones whose remote Update succeeds
 * (remote_err == 0), Store(vni, peer netns) on the peer's node. The reference applies them
 * in goroutine order; here every delete comes first, then the adds, and the first add of a
 * key (node, vni) in (topology, add-list, local-before-remote) order wins. The result
 * becomes the context's resident map (KDTN_VNI_RESIDENT) and, with out->node / vni / net_ns
 * (capacity out->cap entries; NULL = count only), is downloaded: entries of the epoch's adds
 * first, then the surviving snapshot entries, keys unique. Needs a run with
 * the resolve and qdisc stages; KDTN_ENOSPC when cap < n (the map is applied anyway).
 * Sharded (nranks > 1): the daemons' maps are node-global, so every rank applies the ops of
 * EVERY rank — in rank order (rank r's ops before rank r+1's; within a rank the order above) —
 * against the replicated snapshot, and all ranks leave the same map. RCCL contexts gather the
 * ops themselves (two all-gathers: counts, then the lists padded to the largest); host
 * transport: kdtn_vni_ops_export on every rank, all-gather by the caller, kdtn_vni_ops_import
 * of the concatenations (dels of ranks 0..G-1, adds of ranks 0..G-1), then this call. */
typedef struct kdtn_vni_state {
    uint64_t  cap;
    uint32_t  n;                /* out: entries of the map after the epoch */
    uint32_t* node;
    int32_t*  vni;
    uint32_t* net_ns;
} kdtn_vni_state;
int kdtn_epoch_vni_apply(kdtn_ctx* ctx, kdtn_vni_state* out);
/* Keys (node, vni) of the last kdtn_epoch_vni_apply whose result depends on the order the
 * reference's goroutines run the epoch's map ops (one Reconcile worker and one gRPC handler
 * goroutine per batch: no order is defined, daemon/vxlan/manager.go:57-71): a key Stored by
 * two entries with different netns (first vs last store wins), or Stored with the very netns a
 * reached delLink of the key compares Get(vni) against (handler.go:484-487: delete-then-store
 * keeps it, store-then-delete removes it). The apply fixes one order (above); these keys are
 * where a caller that needs the daemons' exact state must serialise the batches involved.
 * n = their count; node / vni (capacity cap, NULL = count only) in the order of the key's
 * winning store. KDTN_EINVAL before an apply of the last run. */
int kdtn_vni_contested(kdtn_ctx* ctx, uint32_t* node, int32_t* vni, uint32_t cap, uint32_t* n);
/* One VxlanManager op (16 B): kind 0 none, 1 Delete(vni) on node, 2 Store(vni, net_ns) on node,
 * 3 a reached delLink whose Get(vni) missed (no effect; net_ns of a delete = the local netns
 * its Get compares against). */
typedef struct kdtn_vni_op { uint32_t node; int32_t vni; uint32_t net_ns; uint32_t kind; } kdtn_vni_op;
/* This rank's ops of the last run: n_del delete slots, n_add add slots (two per AddLinks
 * entry: local node, then peer node); NULL arrays = counts only. */
int kdtn_vni_ops_export(kdtn_ctx* ctx, kdtn_vni_op* dels, uint32_t del_cap, kdtn_vni_op* adds, uint32_t add_cap,
                        uint32_t* n_del, uint32_t* n_add);
/* Host transport: every rank's exported lists concatenated in rank order. */
int kdtn_vni_ops_import(kdtn_ctx* ctx, const kdtn_vni_op* dels, uint32_t n_del, const kdtn_vni_op* adds,
                        uint32_t n_add);
/* The resident map (the last uploaded snapshot or applied state): out->n, and the arrays
 * when given (KDTN_ENOSPC when out->cap < n). */
int kdtn_vni_download(kdtn_ctx* ctx, kdtn_vni_state* out);

/* ---- profiling hooks: per-kernel HIP-event times of the last epoch_run (ms) -------- */
/* Timing level of kdtn_epoch_run's HIP events (each costs ≈5 µs of stream time): 0 none,
 * 1 k_reconcile and the placement kernels only, 2 every stage (default). */
int kdtn_set_timing(kdtn_ctx* ctx, int level);
int kdtn_last_kernel_times(kdtn_ctx* ctx, const char** names, float* ms, int cap);
/* The same marks summed over every epoch synced (kdtn_epoch_sync) since the last reset:
 * names[i], ms[i] (sum over epochs), epochs[i] (epochs that marked it); returns the count.
 * reset != 0 clears the totals after reading (call once with reset = 1 before a timed loop).
 * Instrumentation only (no reference counterpart): lets a timed loop read the HIP-event
 * times once instead of once per epoch. */
int kdtn_timer_totals(kdtn_ctx* ctx, const char** names, double* ms, uint32_t* epochs, int cap, int reset);
/* Per-workgroup phase timestamps of k_reconcile (100 MHz clock; 8 words per workgroup:
 * entry, topologies loaded, counts done, batch bases known, end, XCC_ID<<32|HW_ID, CalcDiff
 * window phase A done, phase B done) of the
 * last epoch run with KDTN_VARIANT bit 16 set. Returns the number of words copied. */
int kdtn_debug_wg_trace(kdtn_ctx* ctx, uint64_t* out, uint32_t cap);

#ifdef __cplusplus
}
#endif
#endif /* KDTN_H */
