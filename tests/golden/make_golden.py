"""Generates tests/golden/samples.json — run once in the build container:

    python tests/golden/make_golden.py [/root/reference]

Inputs: the reference's own sample Topology CRs (data files):
  config/samples/3node.yml, config/samples/tc/latency.yaml, config/samples/tc/bandwidth.yaml
Outputs (committed, so the GPU box never needs /root/reference):
  - the three Topology link sets S0/S1/S2 as plain data, and
  - hand-derived expected reconcile results and qdisc known-answer vectors (SURVEY.md
    Appendix B), written out literally below. They are derived by reading
    controllers/topology_controller.go:288-318 and common/qdisc.go, not by running any
    reference code (the Go reference cannot be built here).
"""
from __future__ import annotations

import json
import os
import sys

import yaml

REF = sys.argv[1] if len(sys.argv) > 1 else "/root/reference"
HERE = os.path.dirname(os.path.abspath(__file__))


def topologies(path):
    with open(path) as f:
        docs = list(yaml.safe_load_all(f))
    out = {}
    for doc in docs:
        for it in doc.get("items", []):
            if it.get("kind") == "Topology":
                out[it["metadata"]["name"]] = it["spec"]["links"]
    return out


S0 = topologies(os.path.join(REF, "config/samples/3node.yml"))
S1 = topologies(os.path.join(REF, "config/samples/tc/latency.yaml"))
S2 = topologies(os.path.join(REF, "config/samples/tc/bandwidth.yaml"))

# S0' : r1 drops uid 2 and adds uid 4 towards r3 (eth3/eth3)
S0p = json.loads(json.dumps(S0))
S0p["r1"] = [l for l in S0p["r1"] if l["uid"] != 2] + [
    {"uid": 4, "peer_pod": "r3", "local_intf": "eth3", "peer_intf": "eth3",
     "local_ip": "14.14.14.1/24", "peer_ip": "14.14.14.3/24"}]

# Hand-derived transitions. Lists are uids in reference order.
TRANSITIONS = [
    {"name": "nil->S0", "status": None, "spec": "S0",
     "expect": {t: {"action": "CREATED", "del": [], "add": [], "upd": []} for t in ("r1", "r2", "r3")}},
    {"name": "S0->S1", "status": "S0", "spec": "S1",
     "expect": {"r1": {"action": "DIFF", "del": [], "add": [], "upd": [1]},
                "r2": {"action": "DIFF", "del": [], "add": [], "upd": [1, 3]},
                "r3": {"action": "DIFF", "del": [], "add": [], "upd": [3]}}},
    {"name": "S1->S2", "status": "S1", "spec": "S2",
     "expect": {"r1": {"action": "DIFF", "del": [], "add": [], "upd": [1, 2]},
                "r2": {"action": "DIFF", "del": [], "add": [], "upd": [1, 3]},
                "r3": {"action": "DIFF", "del": [], "add": [], "upd": [2, 3]}}},
    {"name": "S2->S0", "status": "S2", "spec": "S0",
     "expect": {"r1": {"action": "DIFF", "del": [], "add": [], "upd": [1, 2]},
                "r2": {"action": "DIFF", "del": [], "add": [], "upd": [1, 3]},
                "r3": {"action": "DIFF", "del": [], "add": [], "upd": [2, 3]}}},
    {"name": "S0->S0p", "status": "S0", "spec": "S0p",
     "expect": {"r1": {"action": "DIFF", "del": [2], "add": [4], "upd": []},
                "r2": {"action": "SKIP", "del": [], "add": [], "upd": []},
                "r3": {"action": "SKIP", "del": [], "add": [], "upd": []}}},
]

# Pod placement for the resolve vectors: latency.yaml pins r1, r2 to node "ubuntu" and r3
# to "worker" (config/samples/tc/latency.yaml nodeName fields).
PODS = {"r1": {"src_ip": "10.0.0.1", "net_ns": "/run/netns/r1"},
        "r2": {"src_ip": "10.0.0.1", "net_ns": "/run/netns/r2"},
        "r3": {"src_ip": "10.0.0.2", "net_ns": "/run/netns/r3"}}
# S0->S0p add of uid 4 (r1 → r3): different nodes ⇒ CROSS_NODE, vni 5004, vtep = r3's src_ip
RESOLVE = [{"transition": "S0->S0p", "topology": "r1", "uid": 4, "kind": "CROSS_NODE",
            "vni": 5004, "vtep": "10.0.0.2", "peer": "r3", "err": "none"},
           {"transition": "S0->S0p", "topology": "r1", "del_uid": 2, "vni": 5002, "err": "none"}]

# Qdisc known answers, tick_in_usec = 15.625 (netem field order of include/kdtn.h).
QDISC = [
    {"props": {}, "has_netem": 0},
    {"props": {"latency": "10ms"}, "netem": {"latency": 156250, "limit": 1000}},
    {"props": {"latency": "50ms"}, "netem": {"latency": 781250, "limit": 1000}},
    {"props": {"rate": "1Gbit"}, "netem": {"limit": 1000}, "tbf": [1000000000, 4000000, 1500]},
    {"props": {"rate": "20Mbit"}, "netem": {"limit": 1000}, "tbf": [20000000, 80000, 1500]},
    {"props": {"rate": "50Mbit"}, "netem": {"limit": 1000}, "tbf": [50000000, 200000, 1500]},
    {"props": {"rate": "100Mbit"}, "netem": {"limit": 1000}, "tbf": [100000000, 400000, 1500]},
    {"props": {"rate": "1000"}, "netem": {"limit": 1000}, "tbf": [1000, 5000, 1500]},
    {"props": {"rate": "1Kibps"}, "netem": {"limit": 1000}, "tbf": [8192, 5000, 1500]},
    {"props": {"rate": "1.5Gbit"}, "err": "rate"},
    {"props": {"latency": "1us"}, "netem": {"latency": 15, "limit": 1000}},
    {"props": {"jitter": "5ms"}, "netem": {"latency": 0, "jitter": 5000, "delay_corr": 0, "limit": 1000}},
    {"props": {"latency": "10ms", "jitter": "1ms", "latency_corr": "25"},
     "netem": {"latency": 156250, "jitter": 15625, "delay_corr": 1073741824, "limit": 1000}},
    {"props": {"loss_corr": "50"}, "netem": {"loss": 0, "loss_corr": 0, "limit": 1000}},
    {"props": {"reorder_prob": "25"}, "netem": {"reorder_prob": 1073741824, "gap": 1, "limit": 1000}},
]

P2U = {"0": 0, "0.001": 42949, "0.1": 4294967, "0.5": 21474836, "1": 42949672, "1.5": 64424508,
       "2": 85899344, "5": 214748368, "10": 429496736, "12.5": 536870912, "25": 1073741824,
       "33.3": 1430224128, "50": 2147483648, "75": 3221225472, "99.9": 4290672384,
       "99.99": 4294537728, "99.99999": 4294967040, "100": 4294967295, "100.0": 4294967295}
VNI = {"1": 5001, "100": 5100, "2147478648": -2147483648}
TIME2TICK = {"274877907": 0, "274877906": 4294967281}

json.dump({"sets": {"S0": S0, "S1": S1, "S2": S2, "S0p": S0p}, "transitions": TRANSITIONS,
           "pods": PODS, "resolve": RESOLVE, "qdisc": QDISC, "p2u": P2U, "vni": VNI,
           "time2tick": TIME2TICK, "tick_in_usec": 15.625,
           "source": "config/samples/{3node.yml,tc/latency.yaml,tc/bandwidth.yaml} + SURVEY Appendix B"},
          open(os.path.join(HERE, "samples.json"), "w"), indent=1, sort_keys=True)
print("wrote", os.path.join(HERE, "samples.json"))
