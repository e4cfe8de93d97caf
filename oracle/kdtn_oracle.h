/*
 * kdtn_oracle.h — TEST INFRASTRUCTURE ONLY (the checker, never the product).
 *
 * CPU restatement, in plain C, of the reference kube-dtn reconcile path
 * (Go; dtn-dslab/kube-dtn) and of the third-party arithmetic it calls:
 *   - Go 1.18 stdlib: time.ParseDuration, strconv.ParseFloat(s,32),
 *     strconv.ParseUint, strings.ToLower/TrimSpace, net.ParseCIDR, net.ParseMAC
 *   - github.com/vishvananda/netlink v1.1.1-0.20201029203352-d40f9887b852
 *     (go.mod:20): NewNetem, Percentage2u32, time2Tick
 * Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may load
 * this library. Parity status: the reference cannot be built here (no Go
 * toolchain); the oracle is pinned by the hand-derived known-answer vectors of
 * tests/golden/ (from config/samples and SURVEY Appendix B) — see DESIGN.md.
 */
#ifndef KDTN_ORACLE_H
#define KDTN_ORACLE_H
#include <stdint.h>
#include "../include/kdtn.h"

#ifdef __cplusplus
extern "C" {
#endif

/* Individual reference functions (0 = ok, nonzero = the reference returned err). */
int      or_parse_duration(const char* s, uint32_t n, uint32_t* us);   /* common/qdisc.go:146-158 */
int      or_parse_float32(const char* s, uint32_t n, float* out);      /* strconv.ParseFloat(s,32) */
int      or_parse_pct(const char* s, uint32_t n, float* out);          /* common/qdisc.go:128-143 */
int      or_parse_rate(const char* s, uint32_t n, uint64_t* out);      /* common/qdisc.go:162-199 */
int      or_parse_cidr(const char* s, uint32_t n);                     /* 1 if net.ParseCIDR ok    */
int      or_parse_mac(const char* s, uint32_t n);                      /* 1 if net.ParseMAC ok     */
uint32_t or_p2u(float p);                                              /* netlink Percentage2u32   */
uint32_t or_time2tick(uint32_t t, double tick_in_usec);                /* netlink time2Tick        */
uint32_t or_tbf_burst(uint64_t rate);                                  /* common/qdisc.go:361-370  */
int32_t  or_vni_from_uid(int64_t uid, int32_t base);                   /* common/utils.go:29-31    */

/* MakeQdiscs on 12 property strings (KDTN_P_* order) + gap. */
void or_make_qdisc(const char* const* strs, const uint32_t* lens, uint32_t gap,
                   double tick_in_usec, kdtn_qdisc* out);

/* Global pod table for peer lookups (multi-shard parity); NULL = the topology table. */
typedef struct or_pods {
    uint32_t        n;
    const uint32_t* ns;
    const uint32_t* name;
    const uint32_t* src_ip;
    const uint32_t* net_ns;
    const uint8_t*  flags;
    uint32_t        base;   /* global index of this shard's topology 0 */
} or_pods;

/* Full epoch over topologies [t_begin, t_end): Reconcile gate, literal O(k^2) CalcDiff,
 * addLink/delLink/UpdateLinks pure prefix, MakeQdiscs. Offsets/lists are relative to
 * t_begin. Returns 0, or KDTN_ENOSPC if a capacity is too small. */
int or_reconcile_epoch(const kdtn_epoch_in* in, const or_pods* pods, double tick_in_usec,
                       int32_t vxlan_base, uint32_t t_begin, uint32_t t_end,
                       kdtn_batches* out);
/* Same, also returning the wall time of the per-topology loop alone (the maps — the
 * daemon's informer store and VxlanManager — already exist when Reconcile runs). */
int or_reconcile_epoch_timed(const kdtn_epoch_in* in, const or_pods* pods, double tick_in_usec,
                             int32_t vxlan_base, uint32_t t_begin, uint32_t t_end,
                             kdtn_batches* out, double* loop_seconds);

/* ---- wire encoding of the batches (kdtn_oracle_wire.c) ---------------------------- */
/* unicode/utf8.ValidString */
int      or_utf8_valid(const uint8_t* s, uint32_t n);
/* proto.Marshal(&pb.LinksBatchQuery{...}) of one batch of topology t: list 0 = DelLinks
 * (realised records), 1 = AddLinks, 2 = UpdateLinks (desired records); idx = record
 * indices. Returns the byte count (0 for an empty list: no RPC), or -1 when a string is
 * not valid UTF-8 (Marshal error). out == NULL: size only. */
int64_t  or_encode_batch(const kdtn_epoch_in* in, uint32_t t, int list, const uint32_t* idx,
                         uint32_t n, uint8_t* out);
/* Every batch of an epoch's outputs, regions del | add | upd in topology order:
 * off[list*T + t] .. off[list*T + t + 1] (off has 3T+1 entries), err[t] bit list set when
 * that batch failed to marshal (its range is empty). bytes == NULL: sizes only. */
uint64_t or_encode_epoch(const kdtn_epoch_in* in, const kdtn_batches* b, uint32_t T,
                         uint8_t* bytes, uint64_t* off, uint8_t* err);

/* RemotePod fan-out of an epoch's AddLinks outputs (needs add_res / add_qdisc): daemons
 * node[0..n_nodes) ascending, entries idx[off[k]..off[k+1]) in add-list order. Capacities:
 * node/off/idx >= n_add (+1 for off). Returns the number of senders. */
uint32_t or_fanout(const kdtn_batches* b, uint32_t T, uint32_t* node, uint32_t* off, uint32_t* idx,
                   uint32_t* n_nodes);

/* SetVethQdiscs' tc argv per add (veth/VXLAN kinds) then update entry with a TBF and no
 * error (common/qdisc.go:252-266); off has n_add + n_upd + 1 entries. */
uint64_t or_tc_epoch(const kdtn_epoch_in* in, const kdtn_batches* b, uint8_t* bytes, uint64_t* off);
/* RemotePod messages of the epoch: the UpdateRemote payloads of or_fanout (first n_remote,
 * fan-out order) then the PHYSICAL peers' local Update payloads (add-list order). entry[m]
 * = add entry of message m; message m = bytes[off[m], off[m+1]) (varint length + RemotePod;
 * empty = Marshal error); the receiving daemon's tc argv = tc[tc_off[m], tc_off[m+1]).
 * peer_netns: net_ns id per peer_topo index. Capacities: entry >= n_add, off/tc_off >=
 * n_add + 1; bytes / tc NULL = sizes only. Returns the message count. */
uint32_t or_remote_epoch(const kdtn_epoch_in* in, const kdtn_batches* b, const uint32_t* peer_netns,
                         uint32_t* entry, uint32_t* n_remote, uint8_t* bytes, uint64_t* off,
                         uint8_t* tc, uint64_t* tc_off, uint64_t* n_bytes, uint64_t* n_tc);
/* VxlanManager maps after the epoch's reached entries (deletes, then first-wins adds);
 * returns the entry count (out_* may be NULL to count). pod_netns: net_ns id per global pod. */
uint32_t or_vni_apply(const kdtn_batches* b, uint32_t T, const uint32_t* t_src, const uint32_t* t_netns,
                      const uint32_t* pod_netns, const kdtn_vni_table* snap, uint32_t* out_node,
                      int32_t* out_vni, uint32_t* out_netns);

/* ---- CR ingest (kdtn_oracle_json.c): TopologyList JSON → epoch tables ------------- */
typedef struct or_json_tables {
    int32_t   json_err;       /* kdtn_json_err                                   */
    uint64_t  err_offset;
    uint32_t  T, N, M, n_kdict, n_pdict;
    uint64_t  kdict_bytes, pdict_bytes;
    uint8_t*  kd_bytes; uint32_t* kd_offs; uint8_t* pd_bytes; uint32_t* pd_offs;
    uint32_t *ns, *name, *src_ip, *net_ns; uint8_t* flags; uint32_t *real_off, *des_off;
    uint32_t *des_key, *des_prop, *des_gap; int64_t* des_uid;     /* key[k*N + i]  */
    uint32_t *real_key, *real_prop, *real_gap; int64_t* real_uid;
} or_json_tables;
/* Decode (Go json.Unmarshal into a TopologyList); 0 = done (json_err says whether the
 * document was accepted), -1 = out of memory. Free with or_json_free. */
int  or_json_ingest(const uint8_t* doc, uint64_t n, or_json_tables* out);
void or_json_free(or_json_tables* t);

#ifdef __cplusplus
}
#endif
#endif
