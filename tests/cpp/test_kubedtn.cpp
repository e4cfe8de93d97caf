// test_kubedtn.cpp — tests of the C++ host layer (kube-dtn_amd/host/kubedtn.hpp) on the GPU,
// written the way the reference's Go tests would exercise CalcDiff / MakeQdiscs / the daemon
// batch handlers. Fixtures are the reference's config/samples (3node.yml, tc/latency.yaml,
// tc/bandwidth.yaml) and the hand-derived values of tests/golden/samples.json.
// Run through tests/test_host_cpp.py (pytest -m gpu); exits non-zero on the first failure.
#include <cstdio>
#include <cstdlib>
#include <functional>
#include <map>
#include <string>
#include <vector>

#include "../../kube-dtn_amd/host/kubedtn.hpp"

using namespace kubedtn;

static int g_failed = 0;
#define CHECK(cond)                                                                   \
    do {                                                                              \
        if (!(cond)) {                                                                \
            std::fprintf(stderr, "%s:%d: CHECK failed: %s\n", __FILE__, __LINE__, #cond); \
            ++g_failed;                                                               \
            return;                                                                   \
        }                                                                             \
    } while (0)

static Link mk(const char* li, const char* lip, const char* pi, const char* pip, const char* pp,
               int64_t uid, LinkProperties p = {}) {
    Link l;
    l.LocalIntf = li;
    l.LocalIP = lip;
    l.PeerIntf = pi;
    l.PeerIP = pip;
    l.PeerPod = pp;
    l.UID = uid;
    l.Properties = p;
    return l;
}
static LinkProperties lat(const char* s) { LinkProperties p; p.Latency = s; return p; }
static LinkProperties rate(const char* s) { LinkProperties p; p.Rate = s; return p; }

// config/samples/3node.yml and its tc/ variants: {r1, r2, r3} link lists per state
using State = std::map<std::string, std::vector<Link>>;
static State sample(const std::string& which) {
    auto P = [&](const char* l10, const char* l50, const char* r1g, const char* r20m, const char* r50m,
                 const char* r100m, int slot) -> LinkProperties {
        if (which == "S1") return slot == 0 ? lat(l10) : (slot == 3 ? lat(l50) : LinkProperties{});
        if (which == "S2") {
            const char* r[] = {r1g, r20m, r50m, r100m};
            return rate(r[slot]);
        }
        return {};
    };
    // slots: 0 = uid 1 (r1-r2), 1 = uid 2 on r1, 2 = uid 2 on r3, 3 = uid 3 (r2-r3)
    auto p = [&](int slot) { return P("10ms", "50ms", "1Gbit", "20Mbit", "50Mbit", "100Mbit", slot); };
    State s;
    s["r1"] = {mk("eth1", "12.12.12.1/24", "eth1", "12.12.12.2/24", "r2", 1, p(0)),
               mk("eth2", "13.13.13.1/24", "eth1", "13.13.13.3/24", "r3", 2, p(1))};
    s["r2"] = {mk("eth1", "12.12.12.2/24", "eth1", "12.12.12.1/24", "r1", 1, p(0)),
               mk("eth2", "23.23.23.2/24", "eth2", "23.23.23.3/24", "r3", 3, p(3))};
    s["r3"] = {mk("eth1", "13.13.13.3/24", "eth2", "13.13.13.1/24", "r1", 2, which == "S2" ? p(2) : p(1)),
               mk("eth2", "23.23.23.3/24", "eth2", "23.23.23.2/24", "r2", 3, p(3))};
    if (which == "S2") s["r2"][1].Properties = rate("100Mbit"), s["r3"][1].Properties = rate("100Mbit");
    if (which == "S0p")   // drop r1's uid-2 link, add uid 4 to r3
        s["r1"][1] = mk("eth3", "14.14.14.1/24", "eth3", "14.14.14.3/24", "r3", 4);
    return s;
}

static std::vector<Topology> topologies(const State* status, const State& spec) {
    const char* src[] = {"10.0.0.1", "10.0.0.1", "10.0.0.2"};
    std::vector<Topology> out;
    int i = 0;
    for (const char* n : {"r1", "r2", "r3"}) {
        Topology t;
        t.Name = n;
        t.SpecLinks = spec.at(n);
        if (status) t.StatusLinks = status->at(n);
        t.SrcIP = src[i++];
        t.NetNs = std::string("/run/netns/") + n;
        out.push_back(t);
    }
    return out;
}

static std::vector<int64_t> uids(const std::vector<Link>& v) {
    std::vector<int64_t> u;
    for (const Link& l : v) u.push_back(l.UID);
    return u;
}

// Reconcile over the sample transitions (golden "transitions")
static void TestReconcileSamples(Engine& e) {
    TopologyReconciler r(e);
    struct Want { int action; std::vector<int64_t> add, del, upd; };
    struct Case { const char* from; const char* to; std::vector<Want> want; };
    const int C = KDTN_ACT_CREATED, D = KDTN_ACT_DIFF, S = KDTN_ACT_SKIP;
    const std::vector<Case> cases = {
        {nullptr, "S0", {{C, {}, {}, {}}, {C, {}, {}, {}}, {C, {}, {}, {}}}},
        {"S0", "S1", {{D, {}, {}, {1}}, {D, {}, {}, {1, 3}}, {D, {}, {}, {3}}}},
        {"S1", "S2", {{D, {}, {}, {1, 2}}, {D, {}, {}, {1, 3}}, {D, {}, {}, {2, 3}}}},
        {"S2", "S0", {{D, {}, {}, {1, 2}}, {D, {}, {}, {1, 3}}, {D, {}, {}, {2, 3}}}},
        {"S0", "S0p", {{D, {4}, {2}, {}}, {S, {}, {}, {}}, {S, {}, {}, {}}}},
    };
    for (const Case& c : cases) {
        State from = c.from ? sample(c.from) : State{};
        auto res = r.Reconcile(topologies(c.from ? &from : nullptr, sample(c.to)));
        CHECK(res.size() == 3);
        for (int t = 0; t < 3; ++t) {
            CHECK(res[t].action == c.want[t].action);
            CHECK(uids(res[t].add) == c.want[t].add);
            CHECK(uids(res[t].del) == c.want[t].del);
            CHECK(uids(res[t].propertiesChanged) == c.want[t].upd);
        }
    }
    // S0 -> S0p on r1: AddLinks uid 4 resolves to r3 across nodes, DelLinks uid 2
    State s0 = sample("S0");
    auto res = r.Reconcile(topologies(&s0, sample("S0p")));
    CHECK(res[0].add_plan.size() == 1 && res[0].del_plan.size() == 1);
    const LinkPlan& a = res[0].add_plan[0];
    CHECK(a.kind == KDTN_KIND_CROSS_NODE && a.peer == 2 && a.vni == 5004 && a.vtep == "10.0.0.2");
    CHECK(a.err == KDTN_E_NONE && a.qdiscs.size() == 0);
    CHECK(res[0].del_plan[0].vni == 5002 && res[0].del_plan[0].err == KDTN_E_NONE);
    std::printf("PASS TestReconcileSamples\n");
}

// CalcDiff first-match and duplicate-key semantics (topology_controller.go:288-318)
static void TestCalcDiffDuplicates(Engine& e) {
    TopologyReconciler r(e);
    Link a = mk("eth1", "10.0.0.1/24", "eth1", "10.0.0.2/24", "p", 7);
    Link a_lat = a;
    a_lat.Properties = lat("5ms");
    Link b = mk("eth2", "10.0.1.1/24", "eth1", "10.0.1.2/24", "q", 8);
    std::vector<Link> add, del, chg;
    // old has the key twice (different props), new once with new props: both old records
    // find the same first new record → it is reported once per old record
    r.CalcDiff({a, a_lat}, {a_lat, b}, &add, &del, &chg);
    CHECK(uids(add) == std::vector<int64_t>{8});
    CHECK(del.empty());
    CHECK(chg.size() == 1 && chg[0] == a_lat);          // a vs a_lat differ; a_lat vs a_lat equal
    // new has the key twice: neither is an add (an old record matches), the first is compared
    r.CalcDiff({a}, {a_lat, a}, &add, &del, &chg);
    CHECK(add.empty() && del.empty());
    CHECK(chg.size() == 1 && chg[0] == a_lat);
    // identical lists: nothing
    r.CalcDiff({a, b}, {a, b}, &add, &del, &chg);
    CHECK(add.empty() && del.empty() && chg.empty());
    // disjoint: all deleted, all added, in list order
    r.CalcDiff({a}, {b}, &add, &del, &chg);
    CHECK(uids(add) == std::vector<int64_t>{8} && uids(del) == std::vector<int64_t>{7} && chg.empty());
    std::printf("PASS TestCalcDiffDuplicates\n");
}

// MakeQdiscs known answers (tick_in_usec 15.625; golden "qdisc")
static void TestMakeQdiscs(Engine& e) {
    LinkProperties jit;
    jit.Latency = "10ms";
    jit.LatencyCorr = "25";
    jit.Jitter = "1ms";
    LinkProperties reorder;
    reorder.ReorderProb = "25";
    LinkProperties bad_rate = rate("1.5Gbit");
    LinkProperties bad_loss;
    bad_loss.Loss = "101";
    bad_loss.Rate = "1.5Gbit";                     // loss is parsed first: its error wins
    auto q = MakeQdiscs(e, {LinkProperties{}, lat("10ms"), lat("50ms"), rate("1Gbit"), rate("20Mbit"),
                            rate("1Kibps"), jit, reorder, bad_rate, bad_loss, lat("1us")});
    CHECK(q.size() == 11);
    CHECK(q[0].size() == 0 && q[0].err == KDTN_E_NONE);                       // proto.Size == 0
    CHECK(q[1].netem && q[1].netem->Latency == 156250 && q[1].netem->Limit == 1000 && !q[1].tbf);
    CHECK(q[2].netem && q[2].netem->Latency == 781250);
    CHECK(q[3].tbf && q[3].tbf->Rate == 1000000000ull && q[3].tbf->Buffer == 4000000 && q[3].tbf->Minburst == 1500);
    CHECK(q[3].netem && q[3].netem->Latency == 0);                           // netem always present
    CHECK(q[4].tbf && q[4].tbf->Rate == 20000000ull && q[4].tbf->Buffer == 80000);
    CHECK(q[5].tbf && q[5].tbf->Rate == 8192 && q[5].tbf->Buffer == 5000);   // getTbfBurst floor
    CHECK(q[6].netem && q[6].netem->Latency == 156250 && q[6].netem->Jitter == 15625 &&
          q[6].netem->DelayCorr == 1073741824u);
    CHECK(q[7].netem && q[7].netem->ReorderProb == 1073741824u && q[7].netem->Gap == 1);
    CHECK(q[8].err == KDTN_E_RATE && q[8].size() == 0);
    CHECK(q[9].err == KDTN_E_LOSS);
    CHECK(q[10].netem && q[10].netem->Latency == 15);
    std::printf("PASS TestMakeQdiscs\n");
}

// Daemon batch semantics: the first failing link aborts AddLinks (handler.go:592-611)
static void TestAddLinksBatchAbort(Engine& e) {
    TopologyReconciler r(e);
    Topology a;
    a.Name = "a";
    a.SrcIP = "10.0.0.1";
    a.NetNs = "/run/netns/a";
    a.StatusLinks = std::vector<Link>{};
    a.SpecLinks = std::vector<Link>{
        mk("eth1", "10.0.0.1/24", "eth1", "10.0.0.2/24", "b", 1),
        mk("eth2", "10.0.0.1", "eth1", "10.0.0.2/24", "b", 2),           // MakeVeth: no prefix
        mk("eth3", "10.0.0.3/24", "eth1", "10.0.0.4/24", "nobody", 3),   // peer lookup fails
        mk("eth4", "10.0.0.5/24", "eth1", "", "localhost", 4),
        mk("eth5", "10.0.0.6/24", "eth1", "", "physical/192.168.1.9", 5)};
    Topology b;
    b.Name = "b";
    b.SrcIP = "10.0.0.9";
    b.NetNs = "/run/netns/b";
    b.SpecLinks = std::vector<Link>{};
    auto res = r.Reconcile({a, b});
    const auto& pl = res[0].add_plan;
    CHECK(pl.size() == 5);
    CHECK(pl[0].kind == KDTN_KIND_CROSS_NODE && pl[0].vtep == "10.0.0.9" && pl[0].err == 0);
    CHECK(pl[1].err == KDTN_E_VETH_CIDR);
    CHECK(pl[2].err == KDTN_E_PEER_LOOKUP);
    CHECK(pl[3].kind == KDTN_KIND_MACVLAN);
    CHECK(pl[4].kind == KDTN_KIND_PHYSICAL && pl[4].vtep == "192.168.1.9");
    BatchResponse br = BatchOutcome(pl);
    CHECK(!br.response && br.first_failed == 1 && br.err == KDTN_E_VETH_CIDR);
    CHECK(BatchOutcome({pl[0], pl[3], pl[4]}).response);
    std::printf("PASS TestAddLinksBatchAbort\n");
}

int main() {
    try {
        Engine e(0, 15.625);
        const std::vector<std::pair<const char*, std::function<void(Engine&)>>> tests = {
            {"TestReconcileSamples", TestReconcileSamples},
            {"TestCalcDiffDuplicates", TestCalcDiffDuplicates},
            {"TestMakeQdiscs", TestMakeQdiscs},
            {"TestAddLinksBatchAbort", TestAddLinksBatchAbort}};
        for (const auto& t : tests) {
            const int before = g_failed;
            t.second(e);
            if (g_failed != before) std::printf("FAIL %s\n", t.first);
        }
    } catch (const std::exception& ex) {
        std::fprintf(stderr, "exception: %s\n", ex.what());
        return 2;
    }
    std::printf("%s\n", g_failed ? "FAILED" : "OK");
    return g_failed ? 1 : 0;
}
