// kubedtn.hpp — C++ host layer over the C-ABI (include/kdtn.h), shaped like the reference's
// Go types and entry points for the reconcile path, so a port of the controller/daemon (or
// a test) reads like the reference:
//
//   kubedtn::Link, LinkProperties, Topology    ↔ api/v1/topology_types.go:28-206
//   TopologyReconciler::CalcDiff               ↔ controllers/topology_controller.go:288-318
//   TopologyReconciler::Reconcile              ↔ Reconcile :61-156, all dirty Topologies at once
//   kubedtn::MakeQdiscs                        ↔ common/qdisc.go:20-126 (+ netlink.NewNetem)
//   KubeDTN::AddLinks / DelLinks / UpdateLinks ↔ daemon/kubedtn/handler.go:592-671, the pure
//                                                prefix before the first syscall: per-link plan
//                                                and the batch's BoolResponse/error
//
// Nothing here computes: it interns strings, lays out the SoA tables, calls libkdtn.so
// (HIP, gfx950) and maps indices back to records. Errors are reported the reference's way
// where it has one (first failing link of a batch, Go error text shape), otherwise as
// std::runtime_error carrying the engine's kdtn_strerror.
#pragma once
#include <cstdint>
#include <optional>
#include <stdexcept>
#include <string>
#include <vector>

#include "../../include/kdtn.h"

namespace kubedtn {

struct LinkProperties {        // api/v1/topology_types.go:119-176
    std::string Latency, LatencyCorr, Jitter, Loss, LossCorr, Rate;
    uint32_t Gap = 0;
    std::string Duplicate, DuplicateCorr, ReorderProb, ReorderCorr, CorruptProb, CorruptCorr;
    bool operator==(const LinkProperties& o) const;
    bool operator!=(const LinkProperties& o) const { return !(*this == o); }
};

struct Link {                  // api/v1/topology_types.go:59-95
    std::string LocalIntf, LocalIP, LocalMAC, PeerIntf, PeerIP, PeerMAC, PeerPod;
    int64_t UID = 0;
    LinkProperties Properties;
    bool operator==(const Link& o) const;
    bool operator!=(const Link& o) const { return !(*this == o); }
};

using Links = std::optional<std::vector<Link>>;   // nullopt = nil slice (JSON null/absent)

struct Topology {              // metadata + Spec.Links + Status{Links, SrcIP, NetNs}
    std::string Namespace = "default", Name;
    Links SpecLinks, StatusLinks;
    std::string SrcIP, NetNs;
};

struct Netem {                 // netlink.Netem fields set by NewNetem
    uint32_t Latency = 0, DelayCorr = 0, Limit = 0, Loss = 0, LossCorr = 0, Gap = 0,
             Duplicate = 0, DuplicateCorr = 0, Jitter = 0, ReorderProb = 0, ReorderCorr = 0,
             CorruptProb = 0, CorruptCorr = 0;
};
struct Tbf { uint64_t Rate = 0; uint32_t Buffer = 0, Minburst = 0; };

// MakeQdiscs result: (nil, err) when err != KDTN_E_NONE; empty list when neither is set.
struct Qdiscs {
    std::optional<Netem> netem;
    std::optional<Tbf> tbf;
    int err = KDTN_E_NONE;
    size_t size() const { return (netem ? 1 : 0) + (tbf ? 1 : 0); }
};

// Pure-prefix plan of one batch entry (what addLink / delLink / UpdateLinks would do).
struct LinkPlan {
    int kind = KDTN_KIND_NONE;     // addLink classification (handler.go:333-453)
    int64_t peer = -1;             // global index of the peer Topology, -1 if none
    int32_t vni = 0;               // GetVniFromUid
    std::string vtep;              // CROSS_NODE: peer status.src_ip; PHYSICAL: PeerPod[9:]
    bool vni_hit = false;
    int err = KDTN_E_NONE;         // first failing step (MakeVeth, lookup, MakeQdiscs)
    Qdiscs qdiscs;                 // add / update entries
};

struct ReconcileResult {       // one Topology of Reconcile (:77-138)
    int action = KDTN_ACT_SKIP;
    std::vector<Link> add, del, propertiesChanged;    // CalcDiff order
    std::vector<LinkPlan> add_plan, del_plan, upd_plan;
};

struct VxlanEntry { std::string node_ip; int32_t vni; std::string netns; };   // VxlanManager

// BoolResponse + error of a daemon batch call (handler.go:592-671): the first failing link
// aborts the batch (later links are not attempted).
struct BatchResponse {
    bool response = true;
    int first_failed = -1;         // index in the batch, -1 if none
    int err = KDTN_E_NONE;
    std::string error;             // "<step>: <link index>" (the Go side wraps its own text)
};

class Engine {
  public:
    explicit Engine(int device = 0, double tick_in_usec = -1.0, int32_t vxlan_base = 5000);
    ~Engine();
    Engine(const Engine&) = delete;
    Engine& operator=(const Engine&) = delete;
    kdtn_ctx* ctx() const { return ctx_; }

  private:
    kdtn_ctx* ctx_ = nullptr;
};

class TopologyReconciler {
  public:
    explicit TopologyReconciler(Engine& e) : eng_(e) {}
    // CalcDiff(old, new) (controllers/topology_controller.go:288-318)
    void CalcDiff(const std::vector<Link>& old_links, const std::vector<Link>& new_links,
                  std::vector<Link>* add, std::vector<Link>* del,
                  std::vector<Link>* propertiesChanged);
    // Reconcile (:61-156) over every Topology: action, the three batches in RPC order
    // (Del, Add, Update) and each entry's daemon-side plan.
    std::vector<ReconcileResult> Reconcile(const std::vector<Topology>& topos,
                                           const std::vector<VxlanEntry>& vxlan = {});

  private:
    Engine& eng_;
};

// common.MakeQdiscs for a batch of property sets (one GPU launch).
std::vector<Qdiscs> MakeQdiscs(Engine& e, const std::vector<LinkProperties>& props);

// Daemon handlers' batch semantics over the plans of one LinksBatchQuery.
BatchResponse BatchOutcome(const std::vector<LinkPlan>& plans);

const char* ErrName(int kdtn_err_code);

}  // namespace kubedtn
