/*
 * kdtn_oracle_wire.c — TEST INFRASTRUCTURE ONLY: CPU restatement of the gRPC request
 * bodies the reference controller sends after CalcDiff, i.e. proto.Marshal of
 *
 *   &pb.LinksBatchQuery{LocalPod: &pb.Pod{Name, SrcIp, NetNs, KubeNs},
 *                       Links: common.Map(links, v1.Link.ToProto)}
 *
 * for DelLinks / AddLinks / UpdateLinks (controllers/topology_controller.go:180-188,
 * 223-231, 266-274; Link.ToProto / LinkProperties.ToProto api/v1/topology_types.go:97-109,
 * 178-194; message schema proto/v1/kube_dtn.proto:8-53,65-68).
 *
 * Encoding rules restated from google.golang.org/protobuf (go.mod; proto3, no maps):
 * fields in field-number order; scalars and strings omitted when zero / empty (implicit
 * presence); a non-nil message field is always written, even when empty (ToProto always
 * sets Properties, Reconcile always sets LocalPod); int64 as the varint of its two's
 * complement (10 bytes when negative); a string field that is not valid UTF-8 makes
 * Marshal fail ("string field contains invalid UTF-8"), so the RPC is never sent.
 * tests/golden/make_wire_golden.py pins this file against the Python protobuf runtime.
 */
#include "kdtn_oracle.h"

#include <stdio.h>
#include <stdlib.h>
#include <string.h>

typedef struct { const uint8_t* p; uint32_t n; } wstr;

static wstr wget(const kdtn_strtab* t, uint32_t id) {
    wstr s = {t->bytes + t->offs[id], t->offs[id + 1] - t->offs[id]};
    return s;
}

/* unicode/utf8.ValidString (Go): no overlongs, no surrogates, max U+10FFFF */
int or_utf8_valid(const uint8_t* s, uint32_t n) {
    uint32_t i = 0;
    while (i < n) {
        uint8_t c = s[i];
        if (c < 0x80) { i++; continue; }
        uint32_t need, lo = 0x80, hi = 0xBF;
        if (c >= 0xC2 && c <= 0xDF) need = 1;
        else if (c == 0xE0) { need = 2; lo = 0xA0; }
        else if (c >= 0xE1 && c <= 0xEC) need = 2;
        else if (c == 0xED) { need = 2; hi = 0x9F; }
        else if (c >= 0xEE && c <= 0xEF) need = 2;
        else if (c == 0xF0) { need = 3; lo = 0x90; }
        else if (c >= 0xF1 && c <= 0xF3) need = 3;
        else if (c == 0xF4) { need = 3; hi = 0x8F; }
        else return 0;
        if (i + need >= n) return 0;                     /* truncated sequence */
        uint8_t c1 = s[i + 1];
        if (c1 < lo || c1 > hi) return 0;
        for (uint32_t k = 2; k <= need; k++)
            if (s[i + k] < 0x80 || s[i + k] > 0xBF) return 0;
        i += need + 1;
    }
    return 1;
}

static uint32_t vlen(uint64_t v) {
    uint32_t n = 1;
    while (v >= 0x80) { v >>= 7; n++; }
    return n;
}
static uint8_t* put_varint(uint8_t* p, uint64_t v) {
    while (v >= 0x80) { *p++ = (uint8_t)(v | 0x80); v >>= 7; }
    *p++ = (uint8_t)v;
    return p;
}
/* string field: tag, length, bytes (omitted when empty) */
static uint32_t str_size(wstr s) { return s.n ? 1 + vlen(s.n) + s.n : 0; }
static uint8_t* put_str(uint8_t* p, uint32_t field, wstr s) {
    if (!s.n) return p;
    *p++ = (uint8_t)(field << 3 | 2);
    p = put_varint(p, s.n);
    memcpy(p, s.p, s.n);
    return p + s.n;
}

/* pb.Link field numbers (kube_dtn.proto:17-27) for the key columns KDTN_K_* */
static const uint32_t LINK_FIELD[KDTN_NKEY] = {2, 4, 8, 3, 5, 9, 1};   /* local_intf, local_ip, local_mac,
                                                                           peer_intf, peer_ip, peer_mac, peer_pod */
/* pb.LinkProperties field numbers (kube_dtn.proto:29-43) for KDTN_P_*; gap is field 7 */
static const uint32_t PROP_FIELD[KDTN_NPROP] = {1, 2, 3, 4, 5, 6, 8, 9, 10, 11, 12, 13};

typedef struct { const kdtn_epoch_in* in; const kdtn_link_table* L; uint32_t j; } wrec;

static uint32_t props_size(wrec r) {
    uint32_t n = 0;
    for (int k = 0; k < KDTN_NPROP; k++) n += str_size(wget(&r.in->pdict, r.L->prop[k][r.j]));
    if (r.L->gap[r.j]) n += 1 + vlen(r.L->gap[r.j]);
    return n;
}
static uint32_t link_size(wrec r) {
    uint32_t n = 0;
    for (int k = 0; k < KDTN_NKEY; k++) n += str_size(wget(&r.in->kdict, r.L->key[k][r.j]));
    if (r.L->uid[r.j]) n += 1 + vlen((uint64_t)r.L->uid[r.j]);
    uint32_t ps = props_size(r);
    n += 1 + vlen(ps) + ps;
    return n;
}
static int link_utf8_ok(wrec r) {
    for (int k = 0; k < KDTN_NKEY; k++) {
        wstr s = wget(&r.in->kdict, r.L->key[k][r.j]);
        if (!or_utf8_valid(s.p, s.n)) return 0;
    }
    for (int k = 0; k < KDTN_NPROP; k++) {
        wstr s = wget(&r.in->pdict, r.L->prop[k][r.j]);
        if (!or_utf8_valid(s.p, s.n)) return 0;
    }
    return 1;
}
static uint8_t* put_link(uint8_t* p, wrec r) {
    /* fields in number order: peer_pod 1, local_intf 2, peer_intf 3, local_ip 4, peer_ip 5,
       uid 6, properties 7, local_mac 8, peer_mac 9 */
    static const int ORDER[KDTN_NKEY] = {KDTN_K_PEER_POD, KDTN_K_LOCAL_INTF, KDTN_K_PEER_INTF,
                                         KDTN_K_LOCAL_IP, KDTN_K_PEER_IP, KDTN_K_LOCAL_MAC,
                                         KDTN_K_PEER_MAC};
    for (int q = 0; q < 5; q++)
        p = put_str(p, LINK_FIELD[ORDER[q]], wget(&r.in->kdict, r.L->key[ORDER[q]][r.j]));
    if (r.L->uid[r.j]) {
        *p++ = 6 << 3 | 0;
        p = put_varint(p, (uint64_t)r.L->uid[r.j]);
    }
    *p++ = 7 << 3 | 2;
    p = put_varint(p, props_size(r));
    for (int k = 0; k < KDTN_NPROP; k++) {
        if (PROP_FIELD[k] == 8 && r.L->gap[r.j]) {           /* gap (7) precedes duplicate (8) */
            *p++ = 7 << 3 | 0;
            p = put_varint(p, r.L->gap[r.j]);
        }
        p = put_str(p, PROP_FIELD[k], wget(&r.in->pdict, r.L->prop[k][r.j]));
    }
    for (int q = 5; q < 7; q++)
        p = put_str(p, LINK_FIELD[ORDER[q]], wget(&r.in->kdict, r.L->key[ORDER[q]][r.j]));
    return p;
}

/* pb.Pod{Name 1, SrcIp 2, NetNs 3, KubeNs 4} of topology t */
static void pod_strs(const kdtn_epoch_in* in, uint32_t t, wstr s[4]) {
    s[0] = wget(&in->kdict, in->topos.name[t]);
    s[1] = wget(&in->kdict, in->topos.src_ip[t]);
    s[2] = wget(&in->kdict, in->topos.net_ns[t]);
    s[3] = wget(&in->kdict, in->topos.ns[t]);
}

int64_t or_encode_batch(const kdtn_epoch_in* in, uint32_t t, int list, const uint32_t* idx,
                        uint32_t n, uint8_t* out) {
    const kdtn_link_table* L = list == 0 ? &in->realised : &in->desired;
    wstr pod[4];
    pod_strs(in, t, pod);
    if (n == 0) return 0;                                     /* no RPC for an empty list */
    for (int k = 0; k < 4; k++)
        if (!or_utf8_valid(pod[k].p, pod[k].n)) return -1;
    uint32_t psz = 0;
    for (int k = 0; k < 4; k++) psz += str_size(pod[k]);
    uint64_t total = 1 + vlen(psz) + psz;
    for (uint32_t e = 0; e < n; e++) {
        wrec r = {in, L, idx[e]};
        if (!link_utf8_ok(r)) return -1;
        uint32_t ls = link_size(r);
        total += 1 + vlen(ls) + ls;
    }
    if (!out) return (int64_t)total;
    uint8_t* p = out;
    *p++ = 1 << 3 | 2;
    p = put_varint(p, psz);
    for (int k = 0; k < 4; k++) p = put_str(p, (uint32_t)k + 1, pod[k]);
    for (uint32_t e = 0; e < n; e++) {
        wrec r = {in, L, idx[e]};
        *p++ = 2 << 3 | 2;
        p = put_varint(p, link_size(r));
        p = put_link(p, r);
    }
    return (int64_t)(p - out);
}

uint64_t or_encode_epoch(const kdtn_epoch_in* in, const kdtn_batches* b, uint32_t T, uint8_t* bytes,
                         uint64_t* off, uint8_t* err) {
    const uint32_t* lo[3] = {b->del_off, b->add_off, b->upd_off};
    const uint32_t* li[3] = {b->del_idx, b->add_idx, b->upd_idx};
    uint64_t pos = 0;
    for (uint32_t t = 0; t < T; t++) err[t] = 0;
    for (int list = 0; list < 3; list++) {
        for (uint32_t t = 0; t < T; t++) {
            off[(uint64_t)list * T + t] = pos;
            const uint32_t e0 = lo[list][t], n = lo[list][t + 1] - e0;
            int64_t sz = or_encode_batch(in, t, list, li[list] + e0, n, NULL);
            if (sz < 0) {
                err[t] |= (uint8_t)(1u << list);
                continue;
            }
            if (bytes) or_encode_batch(in, t, list, li[list] + e0, n, bytes + pos);
            pos += (uint64_t)sz;
        }
    }
    off[3ull * T] = pos;
    return pos;
}

/* ======================================================================================
 * Which entries the daemons reach: Reconcile sends DelLinks, AddLinks, UpdateLinks in that
 * order and returns at the first failed RPC (controllers/topology_controller.go:93-116);
 * each handler returns at its first failing link (daemon/kubedtn/handler.go:601-607,
 * 622-628, 644-662). ra[e] / ru[e]: bit 0 reached, bit 1 (add) sends a RemotePod.
 * ==================================================================================== */
static int fan_fails(const kdtn_resolved* r, const kdtn_qdisc* q) {
    if (r->err) return 1;
    return (r->kind == KDTN_KIND_SAME_NODE || r->kind == KDTN_KIND_CROSS_NODE ||
            r->kind == KDTN_KIND_PHYSICAL) && q->err;
}

static void or_reach(const kdtn_batches* b, uint32_t T, uint8_t* ra, uint8_t* ru) {
    for (uint32_t t = 0; t < T; t++) {
        int ok = 1;
        for (uint32_t e = b->del_off[t]; e < b->del_off[t + 1] && ok; e++)
            if (b->del_res[e].err) ok = 0;                                  /* delLink :470-474 */
        for (uint32_t e = b->add_off[t]; e < b->add_off[t + 1]; e++) {
            uint8_t a = 0;
            if (ok) {
                const kdtn_resolved* r = &b->add_res[e];
                a = 1;
                if (fan_fails(r, &b->add_qdisc[e])) ok = 0;
                else {
                    if (r->kind == KDTN_KIND_CROSS_NODE) a |= 2;               /* UpdateRemote :448 */
                    if (r->remote_err) ok = 0;                                  /* :449-451 */
                }
            }
            ra[e] = a;
        }
        for (uint32_t e = b->upd_off[t]; e < b->upd_off[t + 1]; e++) {
            uint8_t a = 0;
            if (ok) {
                a = 1;
                if (b->upd_res[e].err) ok = 0;                                  /* :649-657 */
            }
            ru[e] = a;
        }
    }
}

/* ======================================================================================
 * RemotePod fan-out (daemon/kubedtn/handler.go:419-453, 601-607; common/utils.go:39-67):
 * the AddLinks entries that reach UpdateRemote, grouped by destination daemon
 * (vtep = kdict id of the peer's status.src_ip), daemons in ascending id order, entries
 * in add-list order.
 * ==================================================================================== */
static int cmp_u64(const void* a, const void* b) {
    uint64_t x = *(const uint64_t*)a, y = *(const uint64_t*)b;
    return x < y ? -1 : x > y;
}

uint32_t or_fanout(const kdtn_batches* b, uint32_t T, uint32_t* node, uint32_t* off, uint32_t* idx,
                   uint32_t* n_nodes) {
    /* senders as (vtep << 32 | entry), sorted: stable by entry within a vtep */
    uint32_t na = b->add_off[T], nu = b->upd_off[T];
    uint64_t* keys = (uint64_t*)malloc(sizeof(uint64_t) * (na ? na : 1));
    uint8_t* ra = (uint8_t*)malloc(na + 1);
    uint8_t* ru = (uint8_t*)malloc(nu + 1);
    or_reach(b, T, ra, ru);
    uint32_t ns = 0;
    for (uint32_t e = 0; e < na; e++)
        if (ra[e] & 2) keys[ns++] = ((uint64_t)b->add_res[e].vtep << 32) | e;
    free(ra);
    free(ru);
    qsort(keys, ns, sizeof(uint64_t), cmp_u64);
    uint32_t nn = 0;
    for (uint32_t k = 0; k < ns; k++) {
        uint32_t v = (uint32_t)(keys[k] >> 32);
        if (k == 0 || v != (uint32_t)(keys[k - 1] >> 32)) {
            node[nn] = v;
            off[nn] = k;
            nn++;
        }
        idx[k] = (uint32_t)keys[k];
    }
    off[nn] = ns;
    *n_nodes = nn;
    free(keys);
    return ns;
}

/* ======================================================================================
 * tc argv of SetVethQdiscs' TBF (common/qdisc.go:252-266): "qdisc add dev <intf> parent
 * 1:1 handle 10:0 tbf rate <Rate> burst <Buffer> latency 50ms minburst <Minburst>", each
 * argument NUL-terminated, for every REACHED add entry that calls SetVethQdiscs (veth /
 * VXLAN kinds; both ends of a same-node veth pair) and every REACHED update entry, with a
 * TBF and no error.
 * ==================================================================================== */
static uint64_t tc_one(const kdtn_epoch_in* in, uint32_t j, int col, const kdtn_qdisc* q, uint8_t* out) {
    char tmp[256];
    wstr intf = wget(&in->kdict, in->desired.key[col][j]);
    int n1 = snprintf(tmp, sizeof tmp, "qdisc%cadd%cdev%c", 0, 0, 0);
    uint64_t pos = 0;
    if (out) memcpy(out, tmp, (size_t)n1);
    pos += (uint64_t)n1;
    if (out) memcpy(out + pos, intf.p, intf.n);
    pos += intf.n;
    int n2 = snprintf(tmp, sizeof tmp, "%cparent%c1:1%chandle%c10:0%ctbf%crate%c%llu%cburst%c%u%clatency%c50ms%cminburst%c%u%c",
                      0, 0, 0, 0, 0, 0, 0, (unsigned long long)q->tbf_rate, 0, 0, q->tbf_buffer, 0, 0, 0, 0,
                      q->tbf_minburst, 0);
    if (out) memcpy(out + pos, tmp, (size_t)n2);
    return pos + (uint64_t)n2;
}

uint64_t or_tc_epoch(const kdtn_epoch_in* in, const kdtn_batches* b, uint8_t* bytes, uint64_t* off) {
    /* command slots: add entry e → 2e (LocalIntf), 2e+1 (PeerIntf of a same-node veth pair,
     * common/veth.go:53-60); update entry u → 2*n_add + u (LocalIntf) */
    const uint32_t T = in->topos.n;
    uint8_t* ra = (uint8_t*)malloc(b->n_add + 1);
    uint8_t* ru = (uint8_t*)malloc(b->n_upd + 1);
    or_reach(b, T, ra, ru);
    uint64_t pos = 0;
    uint32_t g = 0;
    for (uint32_t e = 0; e < b->n_add; e++) {
        const kdtn_resolved* r = &b->add_res[e];
        const kdtn_qdisc* q = &b->add_qdisc[e];
        const int on = (ra[e] & 1) && q->has_tbf && !q->err && !r->err &&
                       (r->kind == KDTN_KIND_SAME_NODE || r->kind == KDTN_KIND_CROSS_NODE ||
                        r->kind == KDTN_KIND_PHYSICAL);
        off[g++] = pos;
        if (on) pos += tc_one(in, b->add_idx[e], KDTN_K_LOCAL_INTF, q, bytes ? bytes + pos : NULL);
        off[g++] = pos;
        if (on && r->kind == KDTN_KIND_SAME_NODE)
            pos += tc_one(in, b->add_idx[e], KDTN_K_PEER_INTF, q, bytes ? bytes + pos : NULL);
    }
    for (uint32_t e = 0; e < b->n_upd; e++) {
        const kdtn_resolved* r = &b->upd_res[e];
        const kdtn_qdisc* q = &b->upd_qdisc[e];
        off[g++] = pos;
        if ((ru[e] & 1) && q->has_tbf && !q->err && !r->err)
            pos += tc_one(in, b->upd_idx[e], KDTN_K_LOCAL_INTF, q, bytes ? bytes + pos : NULL);
    }
    off[g] = pos;
    free(ra);
    free(ru);
    return pos;
}

/* ======================================================================================
 * RemotePod messages (proto/v1/kube_dtn.proto:65-79: net_ns 1, intf_name 2, intf_ip 3,
 * peer_vtep 4, kube_ns 5, int32 vni 6, properties 7, name 8). Two sources:
 *  - UpdateRemote (common/utils.go:39-51), sent by a reached cross-node addLink after its
 *    own SetupVxLan (handler.go:419-453): {NetNs: peerPod.NetNs, IntfName: link.PeerIntf,
 *    IntfIp: link.PeerIp, PeerVtep: localPod.SrcIp, Vni, KubeNs: localPod.KubeNs,
 *    Properties: link.Properties, Name: link.PeerPod}; messages in or_fanout order (per
 *    destination daemon, add-list order within);
 *  - the physical peer's local Update (handler.go:348-371), built by every reached PHYSICAL
 *    addLink whose MakeVeth passed: {NetNs: localPod.NetNs, IntfName: link.LocalIntf,
 *    IntfIp: link.LocalIp, PeerVtep: PeerPod[len("physical/"):], Vni, KubeNs, Properties,
 *    Name: link.PeerPod}; after the remote ones, in add-list order.
 * localPod is the LinksBatchQuery's LocalPod (controllers/topology_controller.go:180-188:
 * topology name / status src_ip / status net_ns / namespace); peerPod.NetNs is the peer
 * topology's status.net_ns (ToProtoPod, handler.go:62-88). Properties is always a non-nil
 * message (Link.ToProto), so field 7 is always written. Each message is preceded by its
 * varint length (a delimited stream); a message with a string that is not valid UTF-8
 * fails to marshal and is empty (no prefix). Next to each remote message: the receiving
 * daemon's SetVethQdiscs tc argv on IntfName (Update → SetupVxLan → MakeQdiscs →
 * SetVethQdiscs, daemon/vxlan/vxlan.go:31-51), present when the link has a TBF and the
 * daemon's CreateOrUpdate accepts IntfIp (remote_err == 0); physical messages carry none
 * (their tc runs on LocalIntf and is or_tc_epoch's slot 2e).
 * ==================================================================================== */
typedef struct { wstr s[6]; int32_t vni; wrec r; } rpod;   /* s: net_ns intf_name intf_ip peer_vtep kube_ns name */

static uint32_t rpod_size(const rpod* m) {
    uint32_t n = 0;
    for (int k = 0; k < 5; k++) n += str_size(m->s[k]);
    if (m->vni) n += 1 + vlen((uint64_t)(int64_t)m->vni);
    uint32_t ps = props_size(m->r);
    n += 1 + vlen(ps) + ps;
    n += str_size(m->s[5]);
    return n;
}
static int rpod_utf8_ok(const rpod* m) {
    for (int k = 0; k < 6; k++)
        if (!or_utf8_valid(m->s[k].p, m->s[k].n)) return 0;
    for (int k = 0; k < KDTN_NPROP; k++) {
        wstr q = wget(&m->r.in->pdict, m->r.L->prop[k][m->r.j]);
        if (!or_utf8_valid(q.p, q.n)) return 0;
    }
    return 1;
}
static uint8_t* put_rpod(uint8_t* p, const rpod* m) {
    for (int k = 0; k < 5; k++) p = put_str(p, (uint32_t)k + 1, m->s[k]);
    if (m->vni) {
        *p++ = 6 << 3 | 0;
        p = put_varint(p, (uint64_t)(int64_t)m->vni);
    }
    *p++ = 7 << 3 | 2;
    p = put_varint(p, props_size(m->r));
    for (int k = 0; k < KDTN_NPROP; k++) {
        if (PROP_FIELD[k] == 8 && m->r.L->gap[m->r.j]) {
            *p++ = 7 << 3 | 0;
            p = put_varint(p, m->r.L->gap[m->r.j]);
        }
        p = put_str(p, PROP_FIELD[k], wget(&m->r.in->pdict, m->r.L->prop[k][m->r.j]));
    }
    return put_str(p, 8, m->s[5]);
}

uint32_t or_remote_epoch(const kdtn_epoch_in* in, const kdtn_batches* b, const uint32_t* peer_netns,
                         uint32_t* entry, uint32_t* n_remote, uint8_t* bytes, uint64_t* off,
                         uint8_t* tc, uint64_t* tc_off, uint64_t* n_bytes, uint64_t* n_tc) {
    const uint32_t T = in->topos.n, na = b->add_off[T], nu = b->upd_off[T];
    uint32_t* node = (uint32_t*)malloc(sizeof(uint32_t) * (na + 1));
    uint32_t* noff = (uint32_t*)malloc(sizeof(uint32_t) * (na + 2));
    uint32_t* topo = (uint32_t*)malloc(sizeof(uint32_t) * (na + 1));
    uint8_t* ra = (uint8_t*)malloc(na + 1);
    uint8_t* ru = (uint8_t*)malloc(nu + 1);
    uint32_t nn = 0;
    const uint32_t nr = or_fanout(b, T, node, noff, entry, &nn);
    or_reach(b, T, ra, ru);
    for (uint32_t t = 0; t < T; t++)
        for (uint32_t e = b->add_off[t]; e < b->add_off[t + 1]; e++) topo[e] = t;
    uint32_t n = nr;
    for (uint32_t e = 0; e < na; e++)
        if ((ra[e] & 1) && b->add_res[e].kind == KDTN_KIND_PHYSICAL && !b->add_res[e].err) entry[n++] = e;
    uint64_t pos = 0, tpos = 0;
    for (uint32_t m = 0; m < n; m++) {
        const uint32_t e = entry[m], t = topo[e], j = b->add_idx[e];
        const kdtn_link_table* L = &in->desired;
        rpod q;
        q.r.in = in;
        q.r.L = L;
        q.r.j = j;
        q.vni = b->add_res[e].vni;
        q.s[4] = wget(&in->kdict, in->topos.ns[t]);
        q.s[5] = wget(&in->kdict, L->key[KDTN_K_PEER_POD][j]);
        if (m < nr) {
            q.s[0] = wget(&in->kdict, peer_netns[b->add_res[e].peer_topo]);
            q.s[1] = wget(&in->kdict, L->key[KDTN_K_PEER_INTF][j]);
            q.s[2] = wget(&in->kdict, L->key[KDTN_K_PEER_IP][j]);
            q.s[3] = wget(&in->kdict, in->topos.src_ip[t]);
        } else {
            q.s[0] = wget(&in->kdict, in->topos.net_ns[t]);
            q.s[1] = wget(&in->kdict, L->key[KDTN_K_LOCAL_INTF][j]);
            q.s[2] = wget(&in->kdict, L->key[KDTN_K_LOCAL_IP][j]);
            q.s[3] = q.s[5];
            q.s[3].p += 9;                                   /* strings.TrimPrefix "physical/" */
            q.s[3].n -= 9;
        }
        off[m] = pos;
        if (rpod_utf8_ok(&q)) {
            const uint32_t sz = rpod_size(&q);
            if (bytes) {
                uint8_t* w = put_varint(bytes + pos, sz);
                put_rpod(w, &q);
            }
            pos += vlen(sz) + sz;
        }
        tc_off[m] = tpos;
        const kdtn_qdisc* qd = &b->add_qdisc[e];
        if (m < nr && qd->has_tbf && !b->add_res[e].remote_err)
            tpos += tc_one(in, j, KDTN_K_PEER_INTF, qd, tc ? tc + tpos : NULL);
    }
    off[n] = pos;
    tc_off[n] = tpos;
    *n_remote = nr;
    *n_bytes = pos;
    *n_tc = tpos;
    free(node);
    free(noff);
    free(topo);
    free(ra);
    free(ru);
    return n;
}

/* ======================================================================================
 * VxlanManager state after the epoch (daemon/vxlan/manager.go:57-63 Add / Delete as
 * sync.Map Store / Delete): delLink deletes VNI 5000+uid on the local node when Get(vni) is
 * the local pod's netns (daemon/kubedtn/handler.go:480-487); a cross-node addLink stores
 * (vni, local netns) after SetupVxLan (:426-440) and the peer daemon's Update stores
 * (vni, peer netns) (common/utils.go:39-48 payload NetNs = peerPod.NetNs; handler.go:192);
 * a physical peer's local Update stores (vni, local netns) (:348-371). Entries reached as in
 * or_reach. The reference runs them in goroutine order; this restatement fixes one:
 * every delete first, then every add, the first add of a (node, vni) key in (topology,
 * add-list, local-before-remote) order winning. Output: the winning adds in that order,
 * then the snapshot's surviving entries (first occurrence of each key) in snapshot order.
 * ==================================================================================== */
typedef struct { uint64_t* key; uint32_t* val; uint32_t mask; } vmap;
static uint64_t vkey(uint32_t node, int32_t vni) { return ((uint64_t)node << 32) | (uint32_t)vni; }
static uint32_t* vslot(vmap* m, uint64_t k) {      /* value slot of k (UINT32_MAX = absent) */
    uint64_t h = k * 0x9E3779B97F4A7C15ull;
    for (uint32_t i = (uint32_t)(h >> 32) & m->mask;; i = (i + 1) & m->mask) {
        if (m->val[i] == UINT32_MAX || m->key[i] == k) {
            m->key[i] = k;
            return &m->val[i];
        }
    }
}

uint32_t or_vni_apply(const kdtn_batches* b, uint32_t T, const uint32_t* t_src, const uint32_t* t_netns,
                      const uint32_t* pod_netns, const kdtn_vni_table* snap, uint32_t* out_node,
                      int32_t* out_vni, uint32_t* out_netns) {
    const uint32_t nd = b->del_off[T], na = b->add_off[T], V = snap->n;
    uint64_t cap = 64;
    while (cap < 2ull * (V + 2ull * na + 1)) cap <<= 1;
    vmap snapm = {calloc(cap, 8), malloc(cap * 4), (uint32_t)cap - 1};   /* key → first snapshot entry */
    vmap addm = {calloc(cap, 8), malloc(cap * 4), (uint32_t)cap - 1};    /* key → winning add (order) */
    memset(snapm.val, 0xFF, cap * 4);
    memset(addm.val, 0xFF, cap * 4);
    uint8_t* gone = calloc(V + 1, 1);
    for (uint32_t i = 0; i < V; i++) {
        uint32_t* v = vslot(&snapm, vkey(snap->node[i], snap->vni[i]));
        if (*v == UINT32_MAX) *v = i;
        else gone[i] = 1;                                            /* shadowed duplicate */
    }
    uint32_t* an = malloc(sizeof(uint32_t) * (2 * na + 1));
    int32_t* av = malloc(sizeof(int32_t) * (2 * na + 1));
    uint32_t* as = malloc(sizeof(uint32_t) * (2 * na + 1));
    uint32_t nadd = 0;
    (void)nd;
    for (int pass = 0; pass < 2; pass++) {                           /* 0: deletes, 1: adds */
        for (uint32_t t = 0; t < T; t++) {
            int ok = 1;
            for (uint32_t e = b->del_off[t]; e < b->del_off[t + 1] && ok; e++) {
                const kdtn_resolved* r = &b->del_res[e];
                if (r->err) { ok = 0; break; }
                if (pass == 0 && r->vni_hit) {
                    uint32_t* v = vslot(&snapm, vkey(t_src[t], r->vni));
                    if (*v != UINT32_MAX) gone[*v] = 1;
                }
            }
            for (uint32_t e = b->add_off[t]; e < b->add_off[t + 1] && ok; e++) {
                const kdtn_resolved* r = &b->add_res[e];
                if (fan_fails(r, &b->add_qdisc[e])) { ok = 0; break; }
                if (pass == 0) { if (r->kind == KDTN_KIND_CROSS_NODE && r->remote_err) ok = 0; continue; }
                uint32_t node[2], netns[2], k = 0;
                if (r->kind == KDTN_KIND_CROSS_NODE || r->kind == KDTN_KIND_PHYSICAL) {
                    node[k] = t_src[t];
                    netns[k++] = t_netns[t];
                }
                if (r->kind == KDTN_KIND_CROSS_NODE) {
                    if (r->remote_err) ok = 0;
                    else {
                        node[k] = r->vtep;
                        netns[k++] = pod_netns[r->peer_topo];
                    }
                }
                for (uint32_t q = 0; q < k; q++) {
                    uint32_t* v = vslot(&addm, vkey(node[q], r->vni));
                    if (*v != UINT32_MAX) continue;                      /* an earlier add won */
                    *v = nadd;
                    an[nadd] = node[q];
                    av[nadd] = r->vni;
                    as[nadd++] = netns[q];
                }
            }
        }
    }
    uint32_t n = 0;
    for (uint32_t q = 0; q < nadd; q++, n++) {
        if (out_node) { out_node[n] = an[q]; out_vni[n] = av[q]; out_netns[n] = as[q]; }
    }
    for (uint32_t i = 0; i < V; i++) {
        if (gone[i]) continue;
        if (*vslot(&addm, vkey(snap->node[i], snap->vni[i])) != UINT32_MAX) continue;   /* overridden */
        if (out_node) { out_node[n] = snap->node[i]; out_vni[n] = snap->vni[i]; out_netns[n] = snap->net_ns[i]; }
        n++;
    }
    free(snapm.key); free(snapm.val); free(addm.key); free(addm.val); free(gone); free(an); free(av); free(as);
    return n;
}

/* ======================================================================================
 * Keys whose VxlanManager result depends on the goroutine order (kdtn_vni_contested): over
 * the same reached entries and add order as or_vni_apply, a key is contested when two of its
 * Stores carry different netns (first vs last store wins), or when a Store carries the netns a
 * reached delLink of the key compares Get(vni) against (daemon/kubedtn/handler.go:484-487:
 * delete-then-store keeps the entry, store-then-delete removes it). Output: the contested keys
 * in the order of their first (winning) store.
 * ==================================================================================== */
typedef struct { uint32_t node, vni, netns, used; } dkey;
static uint64_t dhash(uint32_t node, uint32_t vni, uint32_t netns) {
    return (((uint64_t)node << 32) ^ ((uint64_t)vni << 16) ^ netns) * 0x9E3779B97F4A7C15ull;
}

uint32_t or_vni_contested(const kdtn_batches* b, uint32_t T, const uint32_t* t_src, const uint32_t* t_netns,
                          const uint32_t* pod_netns, uint32_t* out_node, int32_t* out_vni) {
    const uint32_t nd = b->del_off[T], na = b->add_off[T];
    uint64_t dcap = 64;
    while (dcap < 2ull * nd + 2) dcap <<= 1;
    dkey* dels = calloc(dcap, sizeof(dkey));                          /* reached deletes {node, vni, netns} */
    uint64_t acap = 64;
    while (acap < 4ull * na + 2) acap <<= 1;
    vmap addm = {calloc(acap, 8), malloc(acap * 4), (uint32_t)acap - 1};   /* key → winning store */
    memset(addm.val, 0xFF, acap * 4);
    uint32_t* an = malloc(sizeof(uint32_t) * (2 * na + 1));
    int32_t* av = malloc(sizeof(int32_t) * (2 * na + 1));
    uint32_t* as = malloc(sizeof(uint32_t) * (2 * na + 1));
    uint32_t* aw = malloc(sizeof(uint32_t) * (2 * na + 1));          /* each store's winner */
    uint32_t nst = 0;
    for (uint32_t t = 0; t < T; t++) {
        int ok = 1;
        for (uint32_t e = b->del_off[t]; e < b->del_off[t + 1]; e++) {
            const kdtn_resolved* r = &b->del_res[e];
            if (r->err) { ok = 0; break; }
            const uint32_t node = t_src[t], vni = (uint32_t)r->vni, ns = t_netns[t];
            for (uint64_t i = dhash(node, vni, ns) & (dcap - 1);; i = (i + 1) & (dcap - 1)) {
                if (!dels[i].used) { dels[i] = (dkey){node, vni, ns, 1}; break; }
                if (dels[i].node == node && dels[i].vni == vni && dels[i].netns == ns) break;
            }
        }
        if (!ok) continue;
        for (uint32_t e = b->add_off[t]; e < b->add_off[t + 1]; e++) {
            const kdtn_resolved* r = &b->add_res[e];
            if (fan_fails(r, &b->add_qdisc[e])) break;
            uint32_t node[2], netns[2], k = 0;
            if (r->kind == KDTN_KIND_CROSS_NODE || r->kind == KDTN_KIND_PHYSICAL) {
                node[k] = t_src[t];
                netns[k++] = t_netns[t];
            }
            int stop = 0;
            if (r->kind == KDTN_KIND_CROSS_NODE) {
                if (r->remote_err) stop = 1;
                else {
                    node[k] = r->vtep;
                    netns[k++] = pod_netns[r->peer_topo];
                }
            }
            for (uint32_t q = 0; q < k; q++) {
                uint32_t* v = vslot(&addm, vkey(node[q], r->vni));
                if (*v == UINT32_MAX) *v = nst;
                an[nst] = node[q];
                av[nst] = r->vni;
                as[nst] = netns[q];
                aw[nst++] = *v;
            }
            if (stop) break;
        }
    }
    uint8_t* flag = calloc(nst + 1, 1);
    for (uint32_t q = 0; q < nst; q++) {
        const uint32_t w = aw[q];
        if (as[w] != as[q]) flag[w] = 1;
        for (uint64_t i = dhash(an[q], (uint32_t)av[q], as[q]) & (dcap - 1); dels[i].used; i = (i + 1) & (dcap - 1))
            if (dels[i].node == an[q] && dels[i].vni == (uint32_t)av[q] && dels[i].netns == as[q]) { flag[w] = 1; break; }
    }
    uint32_t n = 0;
    for (uint32_t q = 0; q < nst; q++)
        if (flag[q]) {
            if (out_node) { out_node[n] = an[q]; out_vni[n] = av[q]; }
            n++;
        }
    free(dels); free(addm.key); free(addm.val); free(an); free(av); free(as); free(aw); free(flag);
    return n;
}
