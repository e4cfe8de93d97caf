"""Synthetic workloads of SURVEY.md §8(d) (configs 1-4) from libkdtn_synth.so.

Bench/test infrastructure: builds `EpochInput`s whose arrays alias the generator's memory
(the generator object is kept alive by `EpochInput.owner`).
"""
from __future__ import annotations

import ctypes as C
import os

import numpy as np

from . import abi
from .tables import EpochInput, Links, StrTab, Topos, Vnis

_HERE = os.path.dirname(os.path.abspath(__file__))
SYNTH_PATH = os.path.join(_HERE, "libkdtn_synth.so")
SEED = 0x6B64746E  # "kdtn"
_lib = None


class Params(C.Structure):
    _fields_ = [("seed", C.c_uint64), ("pods_per_shard", C.c_uint32), ("degree", C.c_uint32),
                ("n_nodes", C.c_uint32), ("dead_frac", C.c_double), ("shard", C.c_uint32),
                ("nshards", C.c_uint32), ("hash_sharding", C.c_uint32), ("total_pods", C.c_uint32)]


def _load():
    global _lib
    if _lib is None:
        if not os.path.exists(SYNTH_PATH):
            raise ImportError(f"{SYNTH_PATH} not built; run `make -C kube-dtn_amd`")
        L = C.CDLL(SYNTH_PATH)
        L.kdtn_synth_new.restype = C.c_void_p
        L.kdtn_synth_new.argtypes = [C.c_int, C.POINTER(Params)]
        L.kdtn_synth_free.argtypes = [C.c_void_p]
        L.kdtn_synth_get.restype = C.c_int
        L.kdtn_synth_get.argtypes = [C.c_void_p, C.c_char_p, C.POINTER(C.c_void_p),
                                     C.POINTER(C.c_uint64), C.POINTER(C.c_uint32)]
        L.kdtn_synth_advance.restype = C.c_int
        L.kdtn_synth_advance.argtypes = [C.c_void_p]
        _lib = L
    return _lib


class _Handle:
    def __init__(self, ptr):
        self.ptr = ptr
        self.free = _load().kdtn_synth_free   # bound now: module globals may be gone at exit

    def __del__(self):
        if self.ptr:
            self.free(self.ptr)
            self.ptr = None


_DT = {1: np.uint8, 4: np.uint32, 8: np.int64}


def _arr(h: _Handle, name: str, dtype=None) -> np.ndarray:
    p, n, e = C.c_void_p(), C.c_uint64(), C.c_uint32()
    if _load().kdtn_synth_get(h.ptr, name.encode(), C.byref(p), C.byref(n), C.byref(e)) != 0:
        raise KeyError(name)
    dt = np.dtype(dtype or _DT[e.value])
    if n.value == 0:
        return np.zeros(0, dt)
    buf = (C.c_uint8 * (n.value * e.value)).from_address(p.value)
    return np.frombuffer(buf, dtype=dt)


def _links(h: _Handle, pre: str) -> Links:
    key = np.stack([_arr(h, f"{pre}key{k}") for k in range(abi.NKEY)]) if True else None
    prop = np.stack([_arr(h, f"{pre}prop{k}") for k in range(abi.NPROP)])
    uid = _arr(h, f"{pre}uid", np.int64)
    gap = _arr(h, f"{pre}gap")
    if uid.shape[0] == 0:
        return Links.empty(0)
    return Links(np.ascontiguousarray(key), uid, np.ascontiguousarray(prop), gap)


def _cache_path(cache_dir, *key):
    return os.path.join(cache_dir, "kdtn_synth_" + "_".join(str(k) for k in key) + ".npz")


def _save(inp: EpochInput, path: str) -> None:
    arrs = {"kb": inp.kdict.bytes_, "ko": inp.kdict.offs, "pb": inp.pdict.bytes_, "po": inp.pdict.offs,
            "tns": inp.topos.ns, "tna": inp.topos.name, "tsr": inp.topos.src_ip, "tnn": inp.topos.net_ns,
            "tfl": inp.topos.flags, "tro": inp.topos.real_off, "tdo": inp.topos.des_off,
            "vno": inp.vnis.node, "vvn": inp.vnis.vni, "vnn": inp.vnis.net_ns,
            "meta": np.array([inp.pod_slice, inp.pod_base, inp.total_pods], np.int64), "gid": inp.gid}
    for side, L in (("r", inp.realised), ("d", inp.desired)):
        arrs[side + "k"], arrs[side + "u"], arrs[side + "p"], arrs[side + "g"] = L.key, L.uid, L.prop, L.gap
    tmp = path + ".tmp.npz"
    np.savez(tmp, **arrs)
    os.replace(tmp, path)


def _load_cached(path: str) -> EpochInput:
    z = np.load(path)
    m = z["meta"]
    inp = EpochInput(StrTab(z["kb"], z["ko"]), StrTab(z["pb"], z["po"]),
                     Topos(z["tns"], z["tna"], z["tsr"], z["tnn"], z["tfl"], z["tro"], z["tdo"]),
                     Links(z["rk"], z["ru"], z["rp"], z["rg"]), Links(z["dk"], z["du"], z["dp"], z["dg"]),
                     Vnis(z["vno"], z["vvn"], z["vnn"]), pod_slice=int(m[0]), pod_base=int(m[1]))
    inp.total_pods = int(m[2])
    inp.gid = z["gid"]
    return inp


def make(config: int, pods_per_shard: int = 1_000_000, degree: int = 10, n_nodes: int = 64,
         dead_frac: float = 0.02, shard: int = 0, nshards: int = 1, seed: int = SEED,
         cache_dir: str | None = None, total_pods: int | None = None) -> EpochInput:
    """Build one shard of synthetic config `config` (1: fat-tree, 2: random-regular,
    3: churn, 4: WAN twin). Config 1 ignores the size parameters.

    Sharding: with `total_pods`, the topology has total_pods pods and this shard owns those
    with kdtn_topology_shard(namespace, name, nshards) == shard (the engine's hash sharding,
    strong scaling); `inp.gid` maps local topologies to global pod ids and the engine's
    global pod index of local topology t is inp.pod_base + t. Without it, shard k owns the
    contiguous pods [k*pods_per_shard, (k+1)*pods_per_shard) (legacy block sharding). With
    `cache_dir`, the tables are memoised as an .npz there."""
    hash_sh = total_pods is not None
    if cache_dir:
        path = _cache_path(cache_dir, config, pods_per_shard, degree, n_nodes, dead_frac, shard,
                           nshards, seed, *(["h", total_pods] if hash_sh else []))
        if os.path.exists(path):
            return _load_cached(path)
        inp = make(config, pods_per_shard, degree, n_nodes, dead_frac, shard, nshards, seed,
                   total_pods=total_pods)
        os.makedirs(cache_dir, exist_ok=True)
        _save(inp, path)
        return inp
    prm = Params(seed, pods_per_shard, degree, n_nodes, dead_frac, shard, nshards, int(hash_sh),
                 int(total_pods or 0))
    ptr = _load().kdtn_synth_new(config, C.byref(prm))
    if not ptr:
        raise ValueError(f"unknown synthetic config {config}")
    return _input(_Handle(ptr))


def _input(h: _Handle) -> EpochInput:
    kdict = StrTab(_arr(h, "kdict_bytes"), _arr(h, "kdict_offs"))
    pdict = StrTab(_arr(h, "pdict_bytes"), _arr(h, "pdict_offs"))
    topos = Topos(_arr(h, "t_ns"), _arr(h, "t_name"), _arr(h, "t_src"), _arr(h, "t_netns"),
                  _arr(h, "t_flags"), _arr(h, "t_roff"), _arr(h, "t_noff"))
    vn = Vnis(_arr(h, "v_node"), _arr(h, "v_vni", np.int32), _arr(h, "v_netns"))
    meta = _arr(h, "meta")
    inp = EpochInput(kdict, pdict, topos, _links(h, "real_"), _links(h, "des_"), vn,
                     pod_slice=int(meta[0]), pod_base=int(meta[1]), owner=h)
    inp.total_pods = int(meta[2])
    inp.gid = _arr(h, "t_gid").astype(np.int64)
    return inp


class ChurnSequence:
    """SURVEY §8(d) config 3 as a sequence of reconcile epochs: epoch 1 has config 2's
    desired links as realised; each advance() makes the current desired the realised side
    and churns 5 % of the edges (1/60 deleted, 1/60 re-drawn props, n_edges/60 added). The
    key / property dictionaries only grow (append-only interning), so each epoch's kdict
    and pdict extend the previous epoch's. Arguments as make(config=3, ...)."""

    def __init__(self, pods_per_shard: int = 1_000_000, shard: int = 0, nshards: int = 1,
                 total_pods: int | None = None, seed: int = SEED, degree: int = 10, n_nodes: int = 64,
                 dead_frac: float = 0.02):
        prm = Params(seed, pods_per_shard, degree, n_nodes, dead_frac, shard, nshards,
                     int(total_pods is not None), int(total_pods or 0))
        ptr = _load().kdtn_synth_new(3, C.byref(prm))
        self._h = _Handle(ptr)
        self.epoch = 1

    def epoch_input(self, copy: bool = False) -> EpochInput:
        """This epoch's tables; without `copy` the arrays alias the generator and are only
        valid until the next advance()."""
        inp = _input(self._h)
        if not copy:
            return inp
        c = lambda a: np.array(a, copy=True)
        out = EpochInput(StrTab(c(inp.kdict.bytes_), c(inp.kdict.offs)), StrTab(c(inp.pdict.bytes_), c(inp.pdict.offs)),
                         Topos(*[c(getattr(inp.topos, f)) for f in ("ns", "name", "src_ip", "net_ns", "flags",
                                                                     "real_off", "des_off")]),
                         Links(c(inp.realised.key), c(inp.realised.uid), c(inp.realised.prop), c(inp.realised.gap)),
                         Links(c(inp.desired.key), c(inp.desired.uid), c(inp.desired.prop), c(inp.desired.gap)),
                         Vnis(c(inp.vnis.node), c(inp.vnis.vni), c(inp.vnis.net_ns)),
                         pod_slice=inp.pod_slice, pod_base=inp.pod_base)
        out.total_pods, out.gid = inp.total_pods, c(inp.gid)
        return out

    def advance(self) -> None:
        self.epoch = _load().kdtn_synth_advance(self._h.ptr)


def select_topologies(inp: EpochInput, keep: np.ndarray) -> EpochInput:
    """The epoch restricted to the Topologies with keep[t] (order kept; or an index array): their rows and both
    link segments; the dictionaries and the VXLAN snapshot are shared. Peers of a dropped
    Topology stay in the kept ones' links (their lookups then fail, as for a deleted CR)."""
    keep = np.asarray(keep)
    sel = np.nonzero(keep)[0] if keep.dtype == bool else keep.astype(np.int64)   # (indices: any order)
    T = inp.topos

    def side(L: Links, off: np.ndarray):
        off = off.astype(np.int64)
        lens = off[sel + 1] - off[sel]
        start = np.repeat(off[sel], lens)
        idx = start + np.arange(int(lens.sum()), dtype=np.int64) - np.repeat(np.cumsum(lens) - lens, lens)
        new_off = np.zeros(len(sel) + 1, np.uint32)
        np.cumsum(lens, out=new_off[1:])
        return L.take(idx) if L.n else Links.empty(0), new_off

    real, roff = side(inp.realised, T.real_off)
    des, doff = side(inp.desired, T.des_off)
    topos = Topos(T.ns[sel].copy(), T.name[sel].copy(), T.src_ip[sel].copy(), T.net_ns[sel].copy(),
                  T.flags[sel].copy(), roff, doff)
    out = EpochInput(inp.kdict, inp.pdict, topos, real, des, inp.vnis)
    out.total_pods = getattr(inp, "total_pods", 0)
    out.gid = inp.gid[sel] if inp.gid is not None else None
    return out


class TopologySetChurn:
    """Config 3 with a changing Topology set: on top of ChurnSequence's link churn, every
    advance() deletes frac/2 of the live Topologies (a CR deleted: spec and status gone,
    DestroyPod) and re-creates as many of the absent ones (a new CR with its current spec and
    no status: the CREATED path, controllers/topology_controller.go:81-85; SetupPod). The
    epoch lists the live Topologies in generator order; links to an absent pod stay and fail
    their peer lookup. frac of the Topologies start absent."""

    def __init__(self, frac: float = 0.01, seed: int = 7, **kw):
        self.cs = ChurnSequence(**kw)
        T = self.cs.epoch_input().topos.n
        self.rng = np.random.default_rng(seed)
        self.frac = frac
        self.alive = np.ones(T, bool)
        self.alive[self.rng.choice(T, int(T * frac), replace=False)] = False

    def epoch_input(self, copy: bool = True) -> EpochInput:
        return select_topologies(self.cs.epoch_input(copy=True), self.alive)

    def advance(self) -> None:
        self.cs.advance()
        k = max(1, int(len(self.alive) * self.frac / 2))
        live, dead = np.nonzero(self.alive)[0], np.nonzero(~self.alive)[0]
        kill = self.rng.choice(live, min(k, len(live)), replace=False)
        back = self.rng.choice(dead, min(k, len(dead)), replace=False)
        self.alive[kill] = False
        self.alive[back] = True


def topology_list_json(inp: EpochInput, pretty: bool = False) -> bytes:
    """The epoch's Topology CRs as a Kubernetes TopologyList JSON document, the way the API
    server serves them (sorted keys, encoding/json escaping) — the CR-ingest workload."""
    L = _load()
    if not getattr(L, "_json_bound", False):
        from . import abi
        L.kdtn_synth_json_new.restype = C.c_void_p
        L.kdtn_synth_json_new.argtypes = [C.POINTER(abi.EpochIn), C.c_uint32, C.POINTER(C.c_uint64)]
        L.kdtn_synth_json_copy.argtypes = [C.c_void_p, C.c_void_p]
        L.kdtn_synth_json_free.argtypes = [C.c_void_p]
        L._json_bound = True
    cin = inp.to_c()
    n = C.c_uint64()
    h = L.kdtn_synth_json_new(C.byref(cin), 1 if pretty else 0, C.byref(n))
    try:
        buf = C.create_string_buffer(n.value)
        L.kdtn_synth_json_copy(h, buf)
        return buf.raw[:n.value]
    finally:
        L.kdtn_synth_json_free(h)
