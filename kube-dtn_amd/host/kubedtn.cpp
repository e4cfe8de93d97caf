// kubedtn.cpp — see kubedtn.hpp. Packs reference-shaped records into the C-ABI tables,
// runs one epoch on the GPU and maps the index lists back to records.
#include "kubedtn.hpp"

#include <cstring>
#include <string>

namespace kubedtn {

namespace {

[[noreturn]] void fail(const char* what, int rc) {
    throw std::runtime_error(std::string(what) + ": " + kdtn_strerror(rc));
}

// Field order of the key / property columns (include/kdtn.h KDTN_K_* / KDTN_P_*).
const std::string* key_field(const Link& l, int k) {
    switch (k) {
    case KDTN_K_LOCAL_INTF: return &l.LocalIntf;
    case KDTN_K_LOCAL_IP: return &l.LocalIP;
    case KDTN_K_LOCAL_MAC: return &l.LocalMAC;
    case KDTN_K_PEER_INTF: return &l.PeerIntf;
    case KDTN_K_PEER_IP: return &l.PeerIP;
    case KDTN_K_PEER_MAC: return &l.PeerMAC;
    default: return &l.PeerPod;
    }
}
const std::string* prop_field(const LinkProperties& p, int k) {
    switch (k) {
    case KDTN_P_LATENCY: return &p.Latency;
    case KDTN_P_LATENCY_CORR: return &p.LatencyCorr;
    case KDTN_P_JITTER: return &p.Jitter;
    case KDTN_P_LOSS: return &p.Loss;
    case KDTN_P_LOSS_CORR: return &p.LossCorr;
    case KDTN_P_RATE: return &p.Rate;
    case KDTN_P_DUPLICATE: return &p.Duplicate;
    case KDTN_P_DUPLICATE_CORR: return &p.DuplicateCorr;
    case KDTN_P_REORDER_PROB: return &p.ReorderProb;
    case KDTN_P_REORDER_CORR: return &p.ReorderCorr;
    case KDTN_P_CORRUPT_PROB: return &p.CorruptProb;
    default: return &p.CorruptCorr;
    }
}

class Interner {
  public:
    Interner() {
        if (int rc = kdtn_interner_new(&it_)) fail("kdtn_interner_new", rc);
    }
    ~Interner() { kdtn_interner_free(it_); }
    uint32_t operator()(const std::string& s) { return kdtn_intern(it_, s.data(), (uint32_t)s.size()); }
    kdtn_strtab table() const {
        kdtn_strtab t{};
        kdtn_interner_table(it_, &t);
        return t;
    }
    std::string str(uint32_t id) const {
        const kdtn_strtab t = table();
        return std::string(reinterpret_cast<const char*>(t.bytes) + t.offs[id], t.offs[id + 1] - t.offs[id]);
    }

  private:
    kdtn_interner* it_ = nullptr;
};

struct LinkColumns {           // kdtn_link_table storage
    std::vector<uint32_t> key[KDTN_NKEY], prop[KDTN_NPROP];
    std::vector<int64_t> uid;
    std::vector<uint32_t> gap;
    void add(const Link& l, Interner& kd, Interner& pd) {
        for (int k = 0; k < KDTN_NKEY; ++k) key[k].push_back(kd(*key_field(l, k)));
        for (int k = 0; k < KDTN_NPROP; ++k) prop[k].push_back(pd(*prop_field(l.Properties, k)));
        uid.push_back(l.UID);
        gap.push_back(l.Properties.Gap);
    }
    kdtn_link_table view() const {
        kdtn_link_table t{};
        t.n = (uint32_t)uid.size();
        for (int k = 0; k < KDTN_NKEY; ++k) t.key[k] = key[k].data();
        for (int k = 0; k < KDTN_NPROP; ++k) t.prop[k] = prop[k].data();
        t.uid = uid.data();
        t.gap = gap.data();
        return t;
    }
};

Qdiscs to_qdiscs(const kdtn_qdisc& q) {
    Qdiscs r;
    r.err = q.err;
    if (q.err) return r;                      // MakeQdiscs returned (nil, err)
    if (q.has_netem) {
        Netem n;
        n.Latency = q.latency;
        n.DelayCorr = q.delay_corr;
        n.Limit = q.limit;
        n.Loss = q.loss;
        n.LossCorr = q.loss_corr;
        n.Gap = q.gap;
        n.Duplicate = q.duplicate;
        n.DuplicateCorr = q.duplicate_corr;
        n.Jitter = q.jitter;
        n.ReorderProb = q.reorder_prob;
        n.ReorderCorr = q.reorder_corr;
        n.CorruptProb = q.corrupt_prob;
        n.CorruptCorr = q.corrupt_corr;
        r.netem = n;
    }
    if (q.has_tbf) r.tbf = Tbf{q.tbf_rate, q.tbf_buffer, q.tbf_minburst};
    return r;
}

LinkPlan to_plan(const kdtn_resolved& res, const kdtn_qdisc* q, bool is_add, const Interner& kd) {
    LinkPlan p;
    p.kind = res.kind;
    p.peer = res.peer_topo == 0xFFFFFFFFu ? -1 : (int64_t)res.peer_topo;
    p.vni = res.vni;
    p.vni_hit = res.vni_hit != 0;
    if (res.kind == KDTN_KIND_CROSS_NODE) p.vtep = kd.str(res.vtep);
    if (res.kind == KDTN_KIND_PHYSICAL) p.vtep = kd.str(res.vtep).substr(9);   // PeerPod[9:]
    p.err = res.err;
    if (q) {
        p.qdiscs = to_qdiscs(*q);
        // addLink reaches MakeQdiscs only on the veth / vxlan paths (common/veth.go:134,
        // daemon/vxlan/vxlan.go:40); UpdateLinks' own error already folds it in
        const bool uses_q = !is_add || res.kind == KDTN_KIND_SAME_NODE ||
                            res.kind == KDTN_KIND_CROSS_NODE || res.kind == KDTN_KIND_PHYSICAL;
        if (!p.err && uses_q) p.err = q->err;
    }
    return p;
}

}  // namespace

bool LinkProperties::operator==(const LinkProperties& o) const {
    for (int k = 0; k < KDTN_NPROP; ++k)
        if (*prop_field(*this, k) != *prop_field(o, k)) return false;
    return Gap == o.Gap;
}

bool Link::operator==(const Link& o) const {
    for (int k = 0; k < KDTN_NKEY; ++k)
        if (*key_field(*this, k) != *key_field(o, k)) return false;
    return UID == o.UID && Properties == o.Properties;
}

Engine::Engine(int device, double tick_in_usec, int32_t vxlan_base) {
    kdtn_config cfg{};
    cfg.device = device;
    cfg.vxlan_base = vxlan_base;
    cfg.tick_in_usec = tick_in_usec >= 0 ? tick_in_usec : kdtn_psched_tick_in_usec();
    if (int rc = kdtn_init(&ctx_, &cfg)) fail("kdtn_init", rc);
}

Engine::~Engine() { kdtn_destroy(ctx_); }

std::vector<ReconcileResult> TopologyReconciler::Reconcile(const std::vector<Topology>& topos,
                                                           const std::vector<VxlanEntry>& vxlan) {
    Interner kd, pd;
    const uint32_t T = (uint32_t)topos.size();
    std::vector<uint32_t> ns(T), name(T), src(T), netns(T), roff(T + 1, 0), noff(T + 1, 0);
    std::vector<uint8_t> flags(T);
    LinkColumns real, des;
    for (uint32_t t = 0; t < T; ++t) {
        const Topology& tp = topos[t];
        ns[t] = kd(tp.Namespace);
        name[t] = kd(tp.Name);
        src[t] = kd(tp.SrcIP);
        netns[t] = kd(tp.NetNs);
        flags[t] = (tp.StatusLinks ? 0 : KDTN_TOPO_STATUS_NIL) | (tp.SpecLinks ? 0 : KDTN_TOPO_SPEC_NIL);
        if (tp.StatusLinks)
            for (const Link& l : *tp.StatusLinks) real.add(l, kd, pd);
        if (tp.SpecLinks)
            for (const Link& l : *tp.SpecLinks) des.add(l, kd, pd);
        roff[t + 1] = (uint32_t)real.uid.size();
        noff[t + 1] = (uint32_t)des.uid.size();
    }
    std::vector<uint32_t> vnode, vnetns;
    std::vector<int32_t> vvni;
    for (const VxlanEntry& v : vxlan) {
        vnode.push_back(kd(v.node_ip));
        vvni.push_back(v.vni);
        vnetns.push_back(kd(v.netns));
    }
    kdtn_epoch_in in{};
    in.kdict = kd.table();
    in.pdict = pd.table();
    in.topos = kdtn_topo_table{T, ns.data(), name.data(), src.data(), netns.data(), flags.data(),
                               roff.data(), noff.data()};
    in.realised = real.view();
    in.desired = des.view();
    in.vnis = kdtn_vni_table{(uint32_t)vvni.size(), vnode.data(), vvni.data(), vnetns.data()};

    const uint32_t M = roff[T], N = noff[T];
    std::vector<uint8_t> action(T);
    std::vector<uint32_t> doff(T + 1), aoff(T + 1), uoff(T + 1), didx(M), aidx(N), uidx(M);
    std::vector<kdtn_resolved> dres(M), ares(N), ures(M);
    std::vector<kdtn_qdisc> aq(N), uq(M);
    kdtn_batches out{};
    out.action = action.data();
    out.del_off = doff.data();
    out.add_off = aoff.data();
    out.upd_off = uoff.data();
    out.del_idx = didx.data();
    out.add_idx = aidx.data();
    out.upd_idx = uidx.data();
    out.del_res = dres.data();
    out.add_res = ares.data();
    out.upd_res = ures.data();
    out.add_qdisc = aq.data();
    out.upd_qdisc = uq.data();
    out.del_cap = M;
    out.add_cap = N;
    out.upd_cap = M;
    if (int rc = kdtn_reconcile_epoch(eng_.ctx(), &in, &out)) fail("kdtn_reconcile_epoch", rc);

    std::vector<ReconcileResult> res(T);
    for (uint32_t t = 0; t < T; ++t) {
        const Topology& tp = topos[t];
        ReconcileResult& r = res[t];
        r.action = action[t];
        for (uint32_t e = doff[t]; e < doff[t + 1]; ++e) {
            r.del.push_back((*tp.StatusLinks)[didx[e] - roff[t]]);
            r.del_plan.push_back(to_plan(dres[e], nullptr, false, kd));
        }
        for (uint32_t e = aoff[t]; e < aoff[t + 1]; ++e) {
            r.add.push_back((*tp.SpecLinks)[aidx[e] - noff[t]]);
            r.add_plan.push_back(to_plan(ares[e], &aq[e], true, kd));
        }
        for (uint32_t e = uoff[t]; e < uoff[t + 1]; ++e) {
            r.propertiesChanged.push_back((*tp.SpecLinks)[uidx[e] - noff[t]]);
            r.upd_plan.push_back(to_plan(ures[e], &uq[e], false, kd));
        }
    }
    return res;
}

void TopologyReconciler::CalcDiff(const std::vector<Link>& old_links, const std::vector<Link>& new_links,
                                  std::vector<Link>* add, std::vector<Link>* del,
                                  std::vector<Link>* propertiesChanged) {
    Topology tp;
    tp.Name = "calc-diff";
    tp.StatusLinks = old_links;
    tp.SpecLinks = new_links;
    ReconcileResult r = Reconcile({tp})[0];
    // CalcDiff itself is ungated: identical lists diff to nothing, which is what SKIP means
    if (add) *add = std::move(r.add);
    if (del) *del = std::move(r.del);
    if (propertiesChanged) *propertiesChanged = std::move(r.propertiesChanged);
}

std::vector<Qdiscs> MakeQdiscs(Engine& e, const std::vector<LinkProperties>& props) {
    Interner pd;
    const uint32_t n = (uint32_t)props.size();
    std::vector<uint32_t> col[KDTN_NPROP], gap(n);
    for (int k = 0; k < KDTN_NPROP; ++k) col[k].resize(n);
    for (uint32_t i = 0; i < n; ++i) {
        for (int k = 0; k < KDTN_NPROP; ++k) col[k][i] = pd(*prop_field(props[i], k));
        gap[i] = props[i].Gap;
    }
    kdtn_props_table t{};
    t.n = n;
    for (int k = 0; k < KDTN_NPROP; ++k) t.prop[k] = col[k].data();
    t.gap = gap.data();
    const kdtn_strtab tab = pd.table();
    std::vector<kdtn_qdisc> q(n);
    if (int rc = kdtn_make_qdiscs(e.ctx(), &tab, &t, q.data())) fail("kdtn_make_qdiscs", rc);
    std::vector<Qdiscs> out;
    out.reserve(n);
    for (const kdtn_qdisc& x : q) out.push_back(to_qdiscs(x));
    return out;
}

BatchResponse BatchOutcome(const std::vector<LinkPlan>& plans) {
    BatchResponse r;
    for (size_t i = 0; i < plans.size(); ++i) {
        if (plans[i].err) {                   // handler.go:600-606: first error aborts
            r.response = false;
            r.first_failed = (int)i;
            r.err = plans[i].err;
            r.error = std::string(kdtn_err_name(plans[i].err)) + ": link " + std::to_string(i);
            break;
        }
    }
    return r;
}

const char* ErrName(int code) { return kdtn_err_name(code); }

}  // namespace kubedtn
