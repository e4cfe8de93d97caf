// kdtn_synth.cpp — deterministic synthetic Topology workloads.
// Bench/test infrastructure (host C++), not part of the engine: it emits exactly the
// SoA tables + deduplicated dictionaries that the C-ABI (include/kdtn.h) consumes.
//
//   config 1  fat-tree: 1,000 spines + 9,000 leaves, 50,000 edges → 100,000 records,
//             uniform props {latency:10ms, loss:0.1, rate:1Gbit}; realised = same keys
//             with empty props → every record is an UpdateLinks entry.
//   config 2  random 10-regular (multi)graph over T pods (pairing model: a keyed Feistel
//             permutation of the 10·T stubs pairs stub π(2i) with π(2i+1); computable per
//             shard), heterogeneous netem/tbf props seeded per uid, 64 nodes, 2 % dead
//             pods; realised = empty non-nil status → every record is an AddLinks entry.
//   config 3  churn on config 2: realised = config-2 desired; desired drops 1/60 of the
//             edges, re-draws the props of 1/60, and adds n_edges/60 fresh edges (5 % churn).
//   config 4  WAN twin: sites in namespaces of 100, power-law degrees (Chung-Lu inside a
//             namespace, hubs ≈1000 links), 256 nodes, 1 % physical/ and 0.5 % localhost
//             peers; realised empty → AddLinks, resolution-dominated.
// Sharding (configs 2-4): "hash" (the engine's) gives pod p to shard
// kdtn_topology_shard(namespace, name, G) = hash64(namespace/name) mod G, the shard's pods in
// ascending p; pod_slice = the largest shard's pod count (every rank uses the same) and
// pod_base = shard * pod_slice, so the engine's global pod index of the shard's t-th pod is
// pod_base + t ("t_gid" maps it back to p). "block" (legacy) gives shard k the contiguous
// pods [k*pods_per_shard, (k+1)*pods_per_shard). Pod names, namespaces, node IPs and netns
// strings carry GLOBAL ids (a shared dictionary prefix identical on every shard); per-link
// strings get shard-local ids.
#include <cstdint>
#include <cstdio>
#include <cmath>
#include <cstring>
#include <algorithm>
#include <array>
#include <string>
#include <thread>
#include <unordered_map>
#include <vector>

#include "../../include/kdtn.h"
#include "kdtn_shard.h"

namespace {

uint64_t splitmix(uint64_t& x) {
    uint64_t z = (x += 0x9E3779B97F4A7C15ull);
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}
uint64_t hmix(uint64_t a, uint64_t b) {
    uint64_t x = a * 0x9E3779B97F4A7C15ull ^ (b + 0x632BE59BD9B4E019ull);
    return splitmix(x);
}

struct Rng {
    uint64_t s;
    explicit Rng(uint64_t seed) : s(seed) {}
    uint64_t next() { return splitmix(s); }
    uint32_t below(uint32_t n) { return (uint32_t)((next() >> 11) % n); }
    double unit() { return (double)(next() >> 11) * (1.0 / 9007199254740992.0); }
};

// Keyed bijection on [0, n) : Feistel network over the next power-of-two square, cycle walking.
struct Perm {
    uint64_t n, half_bits, mask, key;
    Perm(uint64_t n_, uint64_t key_) : n(n_), key(key_) {
        uint64_t bits = 2;
        while ((1ull << bits) < n) ++bits;
        if (bits & 1) ++bits;
        half_bits = bits / 2;
        mask = (1ull << half_bits) - 1;
    }
    uint64_t round_f(uint64_t r, int k) const { return hmix(key + (uint64_t)k, r) & mask; }
    uint64_t fwd1(uint64_t x) const {
        uint64_t l = x >> half_bits, r = x & mask;
        for (int k = 0; k < 4; ++k) {
            uint64_t nl = r, nr = l ^ round_f(r, k);
            l = nl;
            r = nr;
        }
        return (l << half_bits) | r;
    }
    uint64_t inv1(uint64_t y) const {
        uint64_t l = y >> half_bits, r = y & mask;
        for (int k = 3; k >= 0; --k) {
            uint64_t pr = l, pl = r ^ round_f(l, k);
            l = pl;
            r = pr;
        }
        return (l << half_bits) | r;
    }
    uint64_t fwd(uint64_t x) const {
        do { x = fwd1(x); } while (x >= n);
        return x;
    }
    uint64_t inv(uint64_t y) const {
        do { y = inv1(y); } while (y >= n);
        return y;
    }
};

struct Dict {
    std::vector<uint8_t> bytes;
    std::vector<uint32_t> offs{0};
    std::unordered_map<std::string, uint32_t> map;
    uint32_t fixed_end = 0;  // ids < fixed_end were appended without the map
    Dict() { map.emplace(std::string(), 0u), push_raw("", 0); }
    void push_raw(const char* s, size_t n) {
        bytes.insert(bytes.end(), (const uint8_t*)s, (const uint8_t*)s + n);
        offs.push_back((uint32_t)bytes.size());
    }
    uint32_t size() const { return (uint32_t)offs.size() - 1; }
    uint32_t append_unique(const std::string& s) {  // caller guarantees uniqueness
        uint32_t id = size();
        push_raw(s.data(), s.size());
        return id;
    }
    uint32_t intern(const std::string& s) {
        auto it = map.find(s);
        if (it != map.end()) return it->second;
        uint32_t id = size();
        push_raw(s.data(), s.size());
        map.emplace(s, id);
        return id;
    }
};

struct Links {
    std::vector<uint32_t> key[7];
    std::vector<int64_t> uid;
    std::vector<uint32_t> prop[12];
    std::vector<uint32_t> gap;
    size_t size() const { return uid.size(); }
};

struct Props {
    std::string s[12];
    uint32_t gap = 0;
};

struct Synth {
    Dict kd, pd;
    std::vector<uint32_t> t_ns, t_name, t_src, t_netns, t_roff{0}, t_noff{0};
    std::vector<uint8_t> t_flags;
    Links real, des;
    std::vector<uint32_t> v_node, v_netns;
    std::vector<int32_t> v_vni;
    uint32_t pod_slice = 0, pod_base = 0, total_pods = 0;
    std::vector<uint32_t> owned;      // global pod ids of this shard, ascending ("t_gid")
    std::vector<uint32_t> local_of;   // global pod id → local topology index (~0: other shard)
    // config 3 churn sequence: per desired record its global edge id, side and props version
    struct Churn {
        bool on = false;
        uint64_t seed = 0, total = 0, n_edges = 0, q_next = 0;
        uint32_t epoch = 0;
        std::vector<uint64_t> edge;
        std::vector<uint8_t> side;
        std::vector<uint32_t> ver;
    } ch;
    // global-id bases of the shared dictionary prefix
    uint32_t id_default = 0, id_node0 = 0, id_name0 = 0, id_netns0 = 0, id_ns0 = 0;
    uint32_t n_nodes = 0;
};

std::string ip4(uint32_t a) {
    char b[32];
    std::snprintf(b, sizeof b, "10.%u.%u.%u/31", (a >> 16) & 255, (a >> 8) & 255, a & 255);
    return b;
}
std::string node_ip(uint32_t n) {
    char b[32];
    std::snprintf(b, sizeof b, "192.168.%u.%u", n / 256, n % 256);
    return b;
}
std::string num(const char* pre, uint64_t v, const char* suf = "") {
    char b[64];
    std::snprintf(b, sizeof b, "%s%llu%s", pre, (unsigned long long)v, suf);
    return b;
}

// ---- heterogeneous LinkProperties ------------------------------
std::string draw_duration(Rng& r) {
    double u = r.unit();
    if (u < 0.4) return num("", 1 + r.below(500), "ms");
    if (u < 0.8) return num("", 1 + r.below(9999), "us");
    if (u < 0.9) return "1.5s";
    return "0.25ms";
}
std::string draw_pct(Rng& r) {
    if (r.unit() < 0.01) return "100";
    std::string s = num("", r.below(100));
    if (r.unit() < 0.5) {
        int nd = 1 + (int)r.below(4);
        s += '.';
        for (int k = 0; k < nd; ++k) s += (char)('0' + r.below(10));
    }
    return s;
}
std::string draw_rate(Rng& r) {
    static const char* units[] = {"bit", "kbit", "Kibit", "Mbit", "Mibit", "Gbit", "bps", "Mbps", "Gibps"};
    const char* u = units[r.below(9)];
    if (r.unit() < 0.001) return num("", 1 + r.below(1000), "") + "." + num("", r.below(10)) + u;  // err=RATE
    return num("", 1 + r.below(1000), u);
}
// props of a link are seeded by (seed, uid, version): both records of an edge agree.
Props draw_props(uint64_t seed, uint64_t uid, uint32_t version) {
    Rng r(hmix(hmix(seed, uid), version + 0x5151));
    Props p;
    if (r.unit() < 0.5) p.s[0] = draw_duration(r);   // latency
    if (r.unit() < 0.5) p.s[1] = draw_pct(r);        // latency_corr
    if (r.unit() < 0.3) p.s[2] = draw_duration(r);   // jitter
    for (int k : {3, 4, 6, 7, 8, 9, 10, 11})          // loss … corrupt_corr
        if (r.unit() < 0.5) p.s[k] = draw_pct(r);
    if (r.unit() < 0.5) p.s[5] = draw_rate(r);       // rate
    if (r.unit() < 0.2) p.gap = r.below(11);
    return p;
}

void push_link(Synth& S, Links& L, const uint32_t key[7], int64_t uid, const Props& p) {
    for (int k = 0; k < 7; ++k) L.key[k].push_back(key[k]);
    L.uid.push_back(uid);
    for (int k = 0; k < 12; ++k) L.prop[k].push_back(p.s[k].empty() ? 0u : S.pd.intern(p.s[k]));
    L.gap.push_back(p.gap);
}

// shared dictionary prefix: "", "default", node IPs, then per pod: name, netns; namespaces
void shared_prefix(Synth& S, uint32_t total_pods, uint32_t n_nodes, uint32_t n_ns,
                   const char* name_fmt) {
    S.id_default = S.kd.append_unique("default");
    S.kd.map.emplace("default", S.id_default);
    S.id_node0 = S.kd.size();
    for (uint32_t n = 0; n < n_nodes; ++n) {
        std::string s = node_ip(n);
        S.kd.map.emplace(s, S.kd.append_unique(s));
    }
    S.id_ns0 = S.kd.size();
    for (uint32_t q = 0; q < n_ns; ++q) {
        std::string s = num("ns-", q);
        S.kd.map.emplace(s, S.kd.append_unique(s));
    }
    S.id_name0 = S.kd.size();
    char b[64];
    for (uint32_t p = 0; p < total_pods; ++p) {
        std::snprintf(b, sizeof b, name_fmt, p);
        S.kd.push_raw(b, std::strlen(b));   // unique by construction; not looked up by string
    }
    S.id_netns0 = S.kd.size();
    for (uint32_t p = 0; p < total_pods; ++p) {
        std::snprintf(b, sizeof b, "/run/netns/cni-%08x", p);
        S.kd.push_raw(b, std::strlen(b));
    }
    S.n_nodes = n_nodes;
    S.total_pods = total_pods;
}

// Which pods this shard owns (see the header comment). ns_id(p) is the kdict id of pod p's
// namespace; names are the shared-prefix strings id_name0 + p.
template <typename NsOf>
void assign_shard(Synth& S, uint64_t total, uint32_t pods_per_shard, uint32_t shard, uint32_t nshards,
                  bool hash, NsOf ns_id) {
    S.local_of.assign(total, 0xFFFFFFFFu);
    if (!hash) {
        S.pod_slice = pods_per_shard;
        S.pod_base = shard * pods_per_shard;
        for (uint64_t p = S.pod_base; p < S.pod_base + (uint64_t)pods_per_shard && p < total; ++p) S.owned.push_back((uint32_t)p);
    } else {
        std::vector<uint32_t> cnt(nshards, 0);
        for (uint64_t p = 0; p < total; ++p) {
            const uint32_t ns = ns_id(p), nm = S.id_name0 + (uint32_t)p;
            const uint32_t r = kdtn::topology_shard(S.kd.bytes.data() + S.kd.offs[ns], S.kd.offs[ns + 1] - S.kd.offs[ns],
                                                    S.kd.bytes.data() + S.kd.offs[nm], S.kd.offs[nm + 1] - S.kd.offs[nm],
                                                    nshards);
            ++cnt[r];
            if (r == shard) S.owned.push_back((uint32_t)p);
        }
        S.pod_slice = 0;
        for (uint32_t c : cnt) S.pod_slice = std::max(S.pod_slice, c);
        S.pod_base = shard * S.pod_slice;
    }
    for (uint32_t t = 0; t < S.owned.size(); ++t) S.local_of[S.owned[t]] = t;
}

void push_topo(Synth& S, uint32_t p, uint32_t ns_id, bool dead, uint32_t node, uint8_t flags) {
    S.t_ns.push_back(ns_id);
    S.t_name.push_back(S.id_name0 + p);
    S.t_src.push_back(dead ? 0u : S.id_node0 + node);
    S.t_netns.push_back(dead ? 0u : S.id_netns0 + p);
    S.t_flags.push_back(flags);
}
void close_topo(Synth& S) {
    S.t_roff.push_back((uint32_t)S.real.size());
    S.t_noff.push_back((uint32_t)S.des.size());
}

// ---- config 1 --------------------------------------------------------------------------
void build_config1(Synth& S) {
    const uint32_t SP = 1000, LF = 9000, T = SP + LF;
    shared_prefix(S, T, 64, 0, "r%u");
    // edges
    struct E { uint32_t a, b; };
    std::vector<E> edges;
    for (uint32_t j = 0; j < LF; ++j)
        for (uint32_t i = 0; i < 5; ++i) edges.push_back({SP + j, (5 * j + i) % SP});
    for (uint32_t m = 0; m < LF / 2; ++m) edges.push_back({SP + 2 * m, SP + 2 * m + 1});
    for (uint32_t m = 0; m < SP / 2; ++m) edges.push_back({2 * m, 2 * m + 1});
    std::vector<std::vector<std::pair<uint32_t, uint32_t>>> adj(T);  // (edge, side)
    for (uint32_t e = 0; e < edges.size(); ++e) {
        adj[edges[e].a].push_back({e, 0});
        adj[edges[e].b].push_back({e, 1});
    }
    // interface position of each (edge, side)
    std::vector<uint32_t> pos(edges.size() * 2);
    for (uint32_t p = 0; p < T; ++p)
        for (uint32_t k = 0; k < adj[p].size(); ++k) pos[adj[p][k].first * 2 + adj[p][k].second] = k;
    Props uni;
    uni.s[0] = "10ms";
    uni.s[3] = "0.1";
    uni.s[5] = "1Gbit";
    Props empty;
    S.pod_slice = T;
    S.pod_base = 0;
    for (uint32_t p = 0; p < T; ++p) S.owned.push_back(p);
    for (uint32_t p = 0; p < T; ++p) {
        push_topo(S, p, S.id_default, false, p % 64, 0);
        for (auto [e, side] : adj[p]) {
            uint32_t peer = side ? edges[e].a : edges[e].b;
            uint32_t key[7];
            key[0] = S.kd.intern(num("eth", pos[e * 2 + side]));
            key[1] = S.kd.intern(ip4(2 * e + side));
            key[2] = 0;
            key[3] = S.kd.intern(num("eth", pos[e * 2 + (side ^ 1)]));
            key[4] = S.kd.intern(ip4(2 * e + (side ^ 1)));
            key[5] = 0;
            key[6] = S.id_name0 + peer;
            push_link(S, S.real, key, e + 1, empty);
            push_link(S, S.des, key, e + 1, uni);
        }
        close_topo(S);
    }
}

// ---- config 2 / 3 ----------------------------------------------------------------------
struct RegularGraph {
    uint64_t stubs;
    Perm perm;
    uint32_t degree;
    RegularGraph(uint64_t n_pods, uint32_t d, uint64_t seed)
        : stubs(n_pods * d), perm(n_pods * d, seed), degree(d) {}
    // stub s = pod*degree + position; returns partner stub and edge index
    void partner(uint64_t s, uint64_t* other, uint64_t* edge, uint32_t* side) const {
        uint64_t i = perm.inv(s);
        *other = perm.fwd(i ^ 1ull);
        *edge = i >> 1;
        *side = (uint32_t)(i & 1ull);
    }
};

// ---- config 3: churn epochs ---------------------------------------------------------------
// One reconcile epoch of SURVEY §8(d) config 3: realised := the previous desired; each
// alive edge is deleted (both records) with p = 1/60 or gets new props (both records) with
// p = 1/60, decided by hash(seed, epoch, edge) so every shard agrees; n_edges/60 fresh edges
// (new uid, random endpoints, both records appended to their pods' lists) are added. About
// 5 % of the edges churn per epoch: ≈ 167k del, 167k upd and 167k add records at 10M links.
// Status order = the previous spec order; kept records keep their positions. New strings
// (a fresh edge's IPs and interface names) are unique, so they are appended to the key
// dictionary without a lookup: every epoch's kdict extends the previous one.
void churn_advance(Synth& S) {
    auto& C = S.ch;
    C.epoch++;
    const uint64_t seed = C.seed, total = C.total;
    auto decide = [&](uint64_t e) -> int {
        const double u = (double)(hmix(hmix(seed ^ 0xC4124ull, C.epoch), e) >> 11) * (1.0 / 9007199254740992.0);
        return u < 1.0 / 60 ? 1 : (u < 2.0 / 60 ? 2 : 0);
    };
    S.real = std::move(S.des);
    S.des = Links();
    std::vector<uint64_t> r_edge = std::move(C.edge);
    std::vector<uint8_t> r_side = std::move(C.side);
    std::vector<uint32_t> r_ver = std::move(C.ver);
    C.edge.clear();
    C.side.clear();
    C.ver.clear();
    S.t_roff = S.t_noff;
    S.t_noff.assign(1, 0u);
    const uint64_t n_new = C.n_edges / 60;
    std::vector<std::vector<std::pair<uint64_t, uint32_t>>> added(S.owned.size());   // (q, side)
    std::vector<uint64_t> peer_of(n_new * 2);
    Rng r(hmix(seed ^ 0xADDull, C.epoch));
    for (uint64_t k = 0; k < n_new; ++k) {
        const uint64_t a = r.next() % total;
        uint64_t b = r.next() % total;
        if (b == a) b = (b + 1) % total;
        peer_of[2 * k] = b;
        peer_of[2 * k + 1] = a;
        if (S.local_of[a] != 0xFFFFFFFFu) added[S.local_of[a]].push_back({k, 0});
        if (S.local_of[b] != 0xFFFFFFFFu) added[S.local_of[b]].push_back({k, 1});
    }
    auto copy_rec = [&](uint32_t i, const Props* np) {
        for (int k = 0; k < 7; ++k) S.des.key[k].push_back(S.real.key[k][i]);
        S.des.uid.push_back(S.real.uid[i]);
        if (np) {
            for (int k = 0; k < 12; ++k) S.des.prop[k].push_back(np->s[k].empty() ? 0u : S.pd.intern(np->s[k]));
            S.des.gap.push_back(np->gap);
        } else {
            for (int k = 0; k < 12; ++k) S.des.prop[k].push_back(S.real.prop[k][i]);
            S.des.gap.push_back(S.real.gap[i]);
        }
    };
    // a fresh edge's strings, interned once per shard (both of its records may be local)
    std::unordered_map<uint64_t, std::array<uint32_t, 4>> fresh;
    auto fresh_ids = [&](uint64_t q, uint64_t e) -> const std::array<uint32_t, 4>& {
        auto it = fresh.find(q);
        if (it != fresh.end()) return it->second;
        std::array<uint32_t, 4> v{S.kd.append_unique(num("nx", q, "-a")), S.kd.append_unique(num("nx", q, "-b")),
                                  S.kd.append_unique(ip4((uint32_t)(2 * e))), S.kd.append_unique(ip4((uint32_t)(2 * e + 1)))};
        return fresh.emplace(q, v).first->second;
    };
    for (uint32_t t = 0; t < S.owned.size(); ++t) {
        for (uint32_t i = S.t_roff[t]; i < S.t_roff[t + 1]; ++i) {
            const uint64_t e = r_edge[i];
            const int c = decide(e);
            if (c == 1) continue;                                       // deleted edge
            uint32_t ver = r_ver[i];
            if (c == 2) {
                ++ver;
                const Props np = draw_props(seed, e + 1, ver);
                copy_rec(i, &np);
            } else {
                copy_rec(i, nullptr);
            }
            C.edge.push_back(e);
            C.side.push_back(r_side[i]);
            C.ver.push_back(ver);
        }
        for (auto [k, side] : added[t]) {
            const uint64_t q = C.q_next + k, e = C.n_edges + q;
            const auto& f = fresh_ids(q, e);
            uint32_t key[7];
            key[0] = f[side];
            key[1] = f[2 + side];
            key[2] = 0;
            key[3] = f[side ^ 1];
            key[4] = f[2 + (side ^ 1)];
            key[5] = 0;
            key[6] = S.id_name0 + (uint32_t)peer_of[2 * k + side];
            push_link(S, S.des, key, (int64_t)(e + 1), draw_props(seed, e + 1, 0));
            C.edge.push_back(e);
            C.side.push_back((uint8_t)side);
            C.ver.push_back(0);
        }
        S.t_noff.push_back((uint32_t)S.des.size());
    }
    C.q_next += n_new;
}

void build_config23(Synth& S, int config, uint64_t seed, uint64_t total, uint32_t pods_per_shard, uint32_t degree,
                    uint32_t n_nodes, double dead_frac, uint32_t shard, uint32_t nshards, bool hash) {
    shared_prefix(S, (uint32_t)total, n_nodes, 0, "p%u");
    assign_shard(S, total, pods_per_shard, shard, nshards, hash, [&](uint64_t) { return S.id_default; });
    RegularGraph G(total, degree, seed);
    const uint64_t n_edges = G.stubs / 2;
    auto is_dead = [&](uint64_t p) { return (double)(hmix(seed ^ 0xDEADull, p) >> 11) * (1.0 / 9007199254740992.0) < dead_frac; };
    auto node_of = [&](uint64_t p) { return (uint32_t)(hmix(seed ^ 0x40DEull, p) % n_nodes); };
    Props empty;
    for (uint64_t lp = 0; lp < S.owned.size(); ++lp) {
        const uint64_t p = S.owned[lp];
        const bool dead = is_dead(p);
        push_topo(S, (uint32_t)p, S.id_default, dead, node_of(p), 0);
        for (uint32_t k = 0; k < degree; ++k) {
            uint64_t other, e;
            uint32_t side;
            G.partner(p * degree + k, &other, &e, &side);
            const uint64_t peer = other / degree;
            const uint32_t ppos = (uint32_t)(other % degree);
            uint32_t key[7];
            key[0] = S.kd.intern(num("eth", k));
            key[1] = S.kd.intern(ip4((uint32_t)(2 * e + side)));
            key[2] = 0;
            key[3] = S.kd.intern(num("eth", ppos));
            key[4] = S.kd.intern(ip4((uint32_t)(2 * e + (side ^ 1))));
            key[5] = 0;
            key[6] = S.id_name0 + (uint32_t)peer;
            push_link(S, S.des, key, (int64_t)(e + 1), draw_props(seed, e + 1, 0));
            if (config == 3) {
                S.ch.edge.push_back(e);
                S.ch.side.push_back((uint8_t)side);
                S.ch.ver.push_back(0);
            }
        }
        close_topo(S);
    }
    if (config == 3) {                        // realised = config 2's desired, desired = epoch 1
        S.ch.on = true;
        S.ch.seed = seed;
        S.ch.total = total;
        S.ch.n_edges = n_edges;
        churn_advance(S);
    }
}

// ---- config 4: WAN digital twin --------------------------------------------------------
void build_config4(Synth& S, uint64_t seed, uint64_t total, uint32_t sites_per_shard, uint32_t shard,
                   uint32_t nshards, bool hash) {
    const uint32_t per_ns = 100;
    const uint32_t n_ns = (uint32_t)((total + per_ns - 1) / per_ns);
    shared_prefix(S, (uint32_t)total, 256, n_ns, "site-%u");
    assign_shard(S, total, sites_per_shard, shard, nshards, hash,
                 [&](uint64_t p) { return S.id_ns0 + (uint32_t)(p / per_ns); });
    // Chung-Lu inside each namespace: weight w_i ∝ (i+1)^-1.7 (the hub of a namespace draws
    // about half of its 2,000 link ends: hubs of ~1,000 links), mean degree 20;
    // the namespace's edge list is generated from (seed, ns) so every shard agrees.
    std::vector<double> w(per_ns);
    double ws = 0;
    for (uint32_t i = 0; i < per_ns; ++i) ws += (w[i] = 1.0 / std::pow((double)(i + 1), 1.7));
    const double mean_deg = 20.0;
    const uint32_t edges_per_ns = (uint32_t)(per_ns * mean_deg / 2);
    std::vector<double> cdf(per_ns);
    double acc = 0;
    for (uint32_t i = 0; i < per_ns; ++i) cdf[i] = (acc += w[i] / ws);
    auto pick = [&](Rng& r) {
        double u = r.unit();
        uint32_t lo = 0, hi = per_ns - 1;
        while (lo < hi) {
            uint32_t mid = (lo + hi) / 2;
            if (cdf[mid] < u) lo = mid + 1;
            else hi = mid;
        }
        return lo;
    };
    auto is_dead = [&](uint64_t p) { return (hmix(seed ^ 0xDEADull, p) % 100) < 2; };
    auto node_of = [&](uint64_t p) { return (uint32_t)(hmix(seed ^ 0x40DEull, p) % 256); };
    Props empty;
    std::vector<uint8_t> ns_has(n_ns, 0);                  // namespaces holding a pod of this shard
    for (uint32_t p : S.owned) ns_has[p / per_ns] = 1;
    for (uint64_t q = 0; q < n_ns; ++q) {
        if (!ns_has[q]) continue;
        Rng r(hmix(seed, q + 0x4000));
        struct E { uint32_t a, b; uint8_t kind; };   // kind 0 pod-pod, 1 physical, 2 localhost
        std::vector<E> edges(edges_per_ns);
        for (auto& e : edges) {
            e.a = pick(r);
            e.b = pick(r);
            while (e.b == e.a) e.b = pick(r);
            double u = r.unit();
            e.kind = u < 0.01 ? 1 : (u < 0.015 ? 2 : 0);
        }
        std::vector<std::vector<std::pair<uint32_t, uint32_t>>> adj(per_ns);
        for (uint32_t k = 0; k < edges.size(); ++k) {
            adj[edges[k].a].push_back({k, 0});
            if (edges[k].kind == 0) adj[edges[k].b].push_back({k, 1});
        }
        std::vector<uint32_t> pos(edges.size() * 2, 0);
        for (uint32_t i = 0; i < per_ns; ++i)
            for (uint32_t k = 0; k < adj[i].size(); ++k) pos[adj[i][k].first * 2 + adj[i][k].second] = k;
        for (uint32_t i = 0; i < per_ns; ++i) {
            const uint64_t p = q * per_ns + i;
            if (p >= total || S.local_of[p] == 0xFFFFFFFFu) continue;
            push_topo(S, (uint32_t)p, S.id_ns0 + (uint32_t)q, is_dead(p), node_of(p), 0);
            for (auto [k, side] : adj[i]) {
                const E& e = edges[k];
                const uint64_t ge = q * edges_per_ns + k;
                uint32_t key[7];
                key[0] = S.kd.intern(num("ge-", pos[k * 2 + side]));
                key[1] = S.kd.intern(ip4((uint32_t)(2 * ge + side)));
                key[2] = 0;
                key[5] = 0;
                if (e.kind == 1) {
                    key[3] = S.kd.intern("veth1");
                    key[4] = S.kd.intern(ip4((uint32_t)(2 * ge + 1)));
                    key[6] = S.kd.intern(std::string("physical/") + node_ip(200 + (uint32_t)(ge % 50)));
                } else if (e.kind == 2) {
                    key[3] = S.kd.intern("eth0");
                    key[4] = 0;
                    key[6] = S.kd.intern("localhost");
                } else {
                    const uint32_t peer_i = side ? e.a : e.b;
                    key[3] = S.kd.intern(num("ge-", pos[k * 2 + (side ^ 1)]));
                    key[4] = S.kd.intern(ip4((uint32_t)(2 * ge + (side ^ 1))));
                    key[6] = S.id_name0 + (uint32_t)(q * per_ns + peer_i);
                }
                push_link(S, S.des, key, (int64_t)(ge + 1), draw_props(seed, ge + 1, 0));
            }
            close_topo(S);
        }
    }
    // a VxlanManager snapshot (node-global daemon state, identical on every shard): every
    // 50th edge of the whole graph already has a VNI on some node
    const uint64_t n_edges_all = (uint64_t)n_ns * edges_per_ns;
    for (uint64_t ge = 0; ge < n_edges_all; ge += 50) {
        S.v_node.push_back(S.id_node0 + (uint32_t)(ge % 256));
        S.v_vni.push_back((int32_t)(5000 + ge + 1));
        S.v_netns.push_back(S.id_netns0 + (uint32_t)(hmix(seed, ge) % total));
    }
}

}  // namespace

extern "C" {

struct kdtn_synth_params {
    uint64_t seed;
    uint32_t pods_per_shard;   // block sharding: pods per shard
    uint32_t degree;
    uint32_t n_nodes;
    double dead_frac;
    uint32_t shard;
    uint32_t nshards;
    uint32_t hash_sharding;    // 1: shard = kdtn_topology_shard(namespace, name, nshards)
    uint32_t total_pods;       // hash sharding: pods of the whole topology
};

void* kdtn_synth_new(int config, const kdtn_synth_params* prm) {
    Synth* S = new Synth();
    switch (config) {
    case 1: build_config1(*S); break;
    case 2:
    case 3:
    case 4: {
        const bool hash = prm->hash_sharding != 0;
        const uint64_t total = hash ? (uint64_t)prm->total_pods : (uint64_t)prm->pods_per_shard * prm->nshards;
        if (config == 4) build_config4(*S, prm->seed, total, prm->pods_per_shard, prm->shard, prm->nshards, hash);
        else build_config23(*S, config, prm->seed, total, prm->pods_per_shard, prm->degree, prm->n_nodes,
                            prm->dead_frac, prm->shard, prm->nshards, hash);
        break;
    }
    default: delete S; return nullptr;
    }
    if (config == 2 || config == 4) {
        // realised = non-nil empty status: every spec link is added
        S->t_roff.assign(S->t_ns.size() + 1, 0u);
    }
    S->kd.map.clear();
    if (!S->ch.on) S->pd.map.clear();          // churn epochs intern re-drawn props
    return S;
}

// config 3: advance to the next churn epoch (realised := desired, new desired). Arrays
// returned by kdtn_synth_get before the call are invalidated. -1 if not a churn workload.
int kdtn_synth_advance(void* sp) {
    Synth& S = *static_cast<Synth*>(sp);
    if (!S.ch.on) return -1;
    churn_advance(S);
    return (int)S.ch.epoch;
}

void kdtn_synth_free(void* s) { delete static_cast<Synth*>(s); }

// Named arrays: returns pointer, element count and element size.
int kdtn_synth_get(void* sp, const char* name, void** ptr, uint64_t* n, uint32_t* elem) {
    Synth& S = *static_cast<Synth*>(sp);
    auto ret = [&](auto& v) {
        *ptr = (void*)v.data();
        *n = v.size();
        *elem = (uint32_t)sizeof(v[0]);
        return 0;
    };
    std::string nm(name);
    if (nm == "kdict_bytes") return ret(S.kd.bytes);
    if (nm == "kdict_offs") return ret(S.kd.offs);
    if (nm == "pdict_bytes") return ret(S.pd.bytes);
    if (nm == "pdict_offs") return ret(S.pd.offs);
    if (nm == "t_ns") return ret(S.t_ns);
    if (nm == "t_name") return ret(S.t_name);
    if (nm == "t_src") return ret(S.t_src);
    if (nm == "t_netns") return ret(S.t_netns);
    if (nm == "t_flags") return ret(S.t_flags);
    if (nm == "t_roff") return ret(S.t_roff);
    if (nm == "t_noff") return ret(S.t_noff);
    if (nm == "v_node") return ret(S.v_node);
    if (nm == "v_vni") return ret(S.v_vni);
    if (nm == "v_netns") return ret(S.v_netns);
    if (nm == "t_gid") return ret(S.owned);
    for (int side = 0; side < 2; ++side) {
        Links& L = side ? S.des : S.real;
        const std::string pre = side ? "des_" : "real_";
        for (int k = 0; k < 7; ++k)
            if (nm == pre + "key" + std::to_string(k)) return ret(L.key[k]);
        for (int k = 0; k < 12; ++k)
            if (nm == pre + "prop" + std::to_string(k)) return ret(L.prop[k]);
        if (nm == pre + "uid") return ret(L.uid);
        if (nm == pre + "gap") return ret(L.gap);
    }
    if (nm == "meta") {
        static thread_local uint32_t meta[4];
        meta[0] = S.pod_slice;
        meta[1] = S.pod_base;
        meta[2] = S.total_pods;
        meta[3] = S.id_default;
        *ptr = meta;
        *n = 4;
        *elem = 4;
        return 0;
    }
    return -1;
}

// ---- TopologyList JSON writer (CR-ingest workloads) ------------------------------------------
// Writes the tables as the API server serves Topology CRs: keys sorted, spec link strings only
// when set (as written in a user's YAML), status links with every key (the controller's typed
// json.Marshal), properties always present with its non-empty fields, strings escaped like
// encoding/json's Marshal (\", \\, control bytes, HTML-safe \u003c \u003e \u0026,
// U+2028/2029). flags bit 0: one newline + two-space indent per item (kubectl-style).
namespace {
struct JsonW {
    std::string o;
    const kdtn_epoch_in* in;
    void raw(const char* s) { o += s; }
    void str(const kdtn_strtab& t, uint32_t id) {
        const uint8_t* p = t.bytes + t.offs[id];
        const uint32_t n = t.offs[id + 1] - t.offs[id];
        o += '"';
        static const char* hex = "0123456789abcdef";
        for (uint32_t i = 0; i < n; ++i) {
            const uint8_t c = p[i];
            if (c == '"' || c == '\\') { o += '\\'; o += (char)c; }
            else if (c == '\n') o += "\\n";
            else if (c == '\r') o += "\\r";
            else if (c == '\t') o += "\\t";
            else if (c < 0x20 || c == '<' || c == '>' || c == '&') {
                o += "\\u00"; o += hex[c >> 4]; o += hex[c & 15];
            } else if (c == 0xE2 && i + 2 < n && p[i + 1] == 0x80 && (p[i + 2] == 0xA8 || p[i + 2] == 0xA9)) {
                o += p[i + 2] == 0xA8 ? "\\u2028" : "\\u2029";
                i += 2;
            } else o += (char)c;
        }
        o += '"';
    }
    void kv(const char* k, const kdtn_strtab& t, uint32_t id, bool& first, bool always) {
        if (!id && !always) return;
        if (!first) o += ',';
        first = false;
        o += '"'; o += k; o += "\":";
        str(t, id);
    }
    void link(const kdtn_link_table& L, uint32_t i, bool all) {
        static const char* const KEY[7] = {"local_intf", "local_ip", "local_mac", "peer_intf", "peer_ip",
                                           "peer_mac", "peer_pod"};
        static const char* const PROP[12] = {"latency", "latency_corr", "jitter", "loss", "loss_corr", "rate",
                                             "duplicate", "duplicate_corr", "reorder_prob", "reorder_corr",
                                             "corrupt_prob", "corrupt_corr"};
        // sorted: corrupt_corr corrupt_prob duplicate duplicate_corr [gap] jitter latency latency_corr
        //         loss loss_corr rate reorder_corr reorder_prob
        static const int ORD[12] = {11, 10, 6, 7, 2, 0, 1, 3, 4, 5, 9, 8};
        o += '{';
        bool first = true;
        for (int k = 0; k < 7; ++k) kv(KEY[k], in->kdict, L.key[k][i], first, all);
        if (!first) o += ',';
        o += "\"properties\":{";
        bool pf = true;
        for (int q = 0; q < 12; ++q) {
            if (q == 4 && L.gap[i]) {
                if (!pf) o += ',';
                pf = false;
                o += "\"gap\":" + std::to_string(L.gap[i]);
            }
            kv(PROP[ORD[q]], in->pdict, L.prop[ORD[q]][i], pf, false);
        }
        o += "},\"uid\":" + std::to_string((long long)L.uid[i]) + "}";
    }
};

std::string json_range(const kdtn_epoch_in* in, uint32_t t0, uint32_t t1, uint32_t flags) {
    JsonW w;
    w.in = in;
    const kdtn_topo_table& T = in->topos;
    for (uint32_t t = t0; t < t1; ++t) {
        if (t) w.o += ',';
        if (flags & 1) w.o += "\n  ";
        w.raw("{\"apiVersion\":\"y-young.github.io/v1\",\"kind\":\"Topology\",\"metadata\":{");
        bool f = true;
        w.kv("name", in->kdict, T.name[t], f, true);
        w.kv("namespace", in->kdict, T.ns[t], f, true);
        w.raw("},\"spec\":{\"links\":");
        if (T.flags[t] & KDTN_TOPO_SPEC_NIL) w.raw("null");
        else {
            w.o += '[';
            for (uint32_t i = T.des_off[t]; i < T.des_off[t + 1]; ++i) {
                if (i != T.des_off[t]) w.o += ',';
                w.link(in->desired, i, false);
            }
            w.o += ']';
        }
        w.raw("},\"status\":{\"links\":");
        if (T.flags[t] & KDTN_TOPO_STATUS_NIL) w.raw("null");
        else {
            w.o += '[';
            for (uint32_t i = T.real_off[t]; i < T.real_off[t + 1]; ++i) {
                if (i != T.real_off[t]) w.o += ',';
                w.link(in->realised, i, true);
            }
            w.o += ']';
        }
        f = false;
        w.kv("net_ns", in->kdict, T.net_ns[t], f, true);
        w.raw(",\"skipped\":null");
        f = false;
        w.kv("src_ip", in->kdict, T.src_ip[t], f, true);
        w.raw("}}");
    }
    return w.o;
}
}  // namespace

// Builds the document (threads over topology ranges); kdtn_synth_json_copy / _free.
void* kdtn_synth_json_new(const kdtn_epoch_in* in, uint32_t flags, uint64_t* size) {
    auto* parts = new std::vector<std::string>();
    const uint32_t T = in->topos.n;
    const uint32_t P = T > 4096 ? std::min(16u, std::max(1u, std::thread::hardware_concurrency())) : 1;
    parts->assign(P + 2, std::string());
    (*parts)[0] = "{\"apiVersion\":\"y-young.github.io/v1\",\"items\":[";
    std::vector<std::thread> th;
    for (uint32_t p = 0; p < P; ++p) {
        const uint32_t t0 = (uint32_t)((uint64_t)T * p / P), t1 = (uint32_t)((uint64_t)T * (p + 1) / P);
        th.emplace_back([=] { (*parts)[p + 1] = json_range(in, t0, t1, flags); });
    }
    for (auto& x : th) x.join();
    (*parts)[P + 1] = std::string(flags & 1 ? "\n" : "") +
                      "],\"kind\":\"TopologyList\",\"metadata\":{\"resourceVersion\":\"1\"}}";
    uint64_t n = 0;
    for (auto& x : *parts) n += x.size();
    *size = n;
    return parts;
}
void kdtn_synth_json_copy(void* h, uint8_t* out) {
    uint64_t at = 0;
    for (auto& x : *static_cast<std::vector<std::string>*>(h)) {
        std::memcpy(out + at, x.data(), x.size());
        at += x.size();
    }
}
void kdtn_synth_json_free(void* h) { delete static_cast<std::vector<std::string>*>(h); }

}  // extern "C"
