"""TEST INFRASTRUCTURE ONLY — ctypes wrapper of the CPU oracle (libkdtn_oracle.so).

The oracle is the plain-C restatement of the reference reconcile path (see
kdtn_oracle.h). Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg use
it, as the checker / baseline; the product (libkdtn.so, kube-dtn_amd/kdtn) never does.
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess
import sys

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(os.path.dirname(_HERE), "kube-dtn_amd"))
from kdtn import abi  # noqa: E402  (ABI struct layouts only)
from kdtn.tables import BatchesOut, EpochInput  # noqa: E402

# KDTN_ORACLE_LIB: the ASan/UBSan build (make -C oracle sanitize) for tests/test_oracle_sanitizers.py
LIB_PATH = os.environ.get("KDTN_ORACLE_LIB") or os.path.join(_HERE, "libkdtn_oracle.so")
_lib = None


class Pods(C.Structure):
    _fields_ = [("n", C.c_uint32), ("ns", abi.u32p), ("name", abi.u32p), ("src_ip", abi.u32p),
                ("net_ns", abi.u32p), ("flags", abi.u8p), ("base", C.c_uint32)]


def build() -> None:
    subprocess.run(["make", "-s", "-C", _HERE], check=True)


def lib() -> C.CDLL:
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            build()
        L = C.CDLL(LIB_PATH)
        cs, u32 = C.c_char_p, C.c_uint32
        L.or_parse_duration.argtypes = [cs, u32, C.POINTER(C.c_uint32)]
        L.or_parse_float32.argtypes = [cs, u32, C.POINTER(C.c_float)]
        L.or_parse_pct.argtypes = [cs, u32, C.POINTER(C.c_float)]
        L.or_parse_rate.argtypes = [cs, u32, C.POINTER(C.c_uint64)]
        L.or_parse_cidr.argtypes = [cs, u32]
        L.or_parse_mac.argtypes = [cs, u32]
        L.or_p2u.argtypes = [C.c_float]
        L.or_p2u.restype = C.c_uint32
        L.or_time2tick.argtypes = [C.c_uint32, C.c_double]
        L.or_time2tick.restype = C.c_uint32
        L.or_tbf_burst.argtypes = [C.c_uint64]
        L.or_tbf_burst.restype = C.c_uint32
        L.or_vni_from_uid.argtypes = [C.c_int64, C.c_int32]
        L.or_vni_from_uid.restype = C.c_int32
        L.or_make_qdisc.argtypes = [C.POINTER(C.c_char_p), C.POINTER(C.c_uint32), C.c_uint32,
                                    C.c_double, C.POINTER(abi.Qdisc)]
        L.or_reconcile_epoch.argtypes = [C.POINTER(abi.EpochIn), C.POINTER(Pods), C.c_double,
                                         C.c_int32, C.c_uint32, C.c_uint32, C.POINTER(abi.Batches)]
        L.or_reconcile_epoch_timed.argtypes = L.or_reconcile_epoch.argtypes + [C.POINTER(C.c_double)]
        _lib = L
    return _lib


def _b(s) -> bytes:
    return s.encode() if isinstance(s, str) else bytes(s)


def parse_duration(s):
    """ParseDuration (common/qdisc.go:146): (ok, microseconds)."""
    b = _b(s)
    v = C.c_uint32()
    return lib().or_parse_duration(b, len(b), C.byref(v)) == 0, v.value


def parse_float32(s):
    b = _b(s)
    v = C.c_float()
    return lib().or_parse_float32(b, len(b), C.byref(v)) == 0, v.value


def parse_pct(s):
    """ParseFloatPercentage (common/qdisc.go:128): (ok, float32 value)."""
    b = _b(s)
    v = C.c_float()
    return lib().or_parse_pct(b, len(b), C.byref(v)) == 0, v.value


def parse_rate(s):
    """ParseRate (common/qdisc.go:162): (ok, bits/s)."""
    b = _b(s)
    v = C.c_uint64()
    return lib().or_parse_rate(b, len(b), C.byref(v)) == 0, v.value


def parse_cidr(s) -> bool:
    b = _b(s)
    return lib().or_parse_cidr(b, len(b)) == 1


def parse_mac(s) -> bool:
    b = _b(s)
    return lib().or_parse_mac(b, len(b)) == 1


def p2u(p: float) -> int:
    return lib().or_p2u(p)


def time2tick(t: int, tick: float) -> int:
    return lib().or_time2tick(t, tick)


def vni_from_uid(uid: int, base: int = 5000) -> int:
    return lib().or_vni_from_uid(uid, base)


def make_qdisc(props: dict, tick: float = 15.625) -> np.ndarray:
    """MakeQdiscs (common/qdisc.go:20) of one LinkProperties given as a dict."""
    strs = [_b(props.get(f, "")) for f in abi.PROP_COLS]
    arr = (C.c_char_p * abi.NPROP)(*strs)
    lens = (C.c_uint32 * abi.NPROP)(*[len(s) for s in strs])
    q = abi.Qdisc()
    lib().or_make_qdisc(arr, lens, int(props.get("gap", 0)), tick, C.byref(q))
    return np.frombuffer(bytes(q), dtype=abi.QDISC_DTYPE)[0]


def reconcile(inp: EpochInput, tick: float = 15.625, vxlan_base: int = 5000, pods=None,
              t_begin: int = 0, t_end: int | None = None, timing: list | None = None) -> BatchesOut:
    """Full reference epoch (gate + literal CalcDiff + daemon pure prefix + MakeQdiscs).

    `pods`: optional global pod table (dict of numpy arrays ns/name/src_ip/net_ns/flags and
    int `base`) for multi-shard parity; default = the shard's own topology table."""
    T = inp.topos.n
    if t_end is None:
        t_end = T
    cin = inp.to_c()
    # a range's lists hold at most its own records: del and upd (one per realised record,
    # repeated for duplicate old keys) its realised records, add its desired records
    T0 = inp.topos
    cap_r = max(int(T0.real_off[t_end]) - int(T0.real_off[t_begin]), 1)
    cap_d = max(int(T0.des_off[t_end]) - int(T0.des_off[t_begin]), 1)
    out = BatchesOut.alloc(t_end - t_begin, cap_r, cap_d, cap_r)
    b = out.to_c((cap_r, cap_d, cap_r))
    pp = None
    if pods is not None:
        keep = {k: np.ascontiguousarray(v, dtype=np.uint8 if k == "flags" else np.uint32)
                for k, v in pods.items() if k != "base"}
        pp = Pods(len(keep["ns"]), abi.ptr(keep["ns"], abi.u32p), abi.ptr(keep["name"], abi.u32p),
                  abi.ptr(keep["src_ip"], abi.u32p), abi.ptr(keep["net_ns"], abi.u32p),
                  abi.ptr(keep["flags"], abi.u8p), int(pods.get("base", 0)))
    secs = C.c_double(0.0)
    rc = lib().or_reconcile_epoch_timed(C.byref(cin), C.byref(pp) if pp is not None else None, tick,
                                        vxlan_base, t_begin, t_end, C.byref(b), C.byref(secs))
    if timing is not None:
        timing.append(secs.value)
    if rc != 0:
        raise RuntimeError(f"oracle reconcile failed: {rc}")
    return out.trim(b.n_del, b.n_add, b.n_upd)


def reconcile_parallel(inp: EpochInput, tick: float = 15.625, vxlan_base: int = 5000, pods=None,
                       t_begin: int = 0, t_end: int | None = None, threads: int = 0) -> BatchesOut:
    """reconcile() over [t_begin, t_end) split into `threads` disjoint topology ranges of
    about equal record counts (the reference's concurrent reconcilers, each topology
    independent), run concurrently (the ctypes call releases the GIL) and concatenated: the
    same BatchesOut as one reconcile() call, so full-size epochs check bit for bit in seconds."""
    from concurrent.futures import ThreadPoolExecutor
    T = inp.topos.n
    if t_end is None:
        t_end = T
    threads = threads or max(1, min(16, len(os.sched_getaffinity(0))))
    w = (inp.topos.des_off.astype(np.int64) + inp.topos.real_off.astype(np.int64))
    cuts = np.searchsorted(w, np.linspace(w[t_begin], w[t_end], threads + 1))
    cuts = np.clip(cuts, t_begin, t_end)
    cuts[0], cuts[-1] = t_begin, t_end
    bounds = sorted(set(int(c) for c in cuts))
    parts_ = list(zip(bounds[:-1], bounds[1:]))
    if not parts_:
        return reconcile(inp, tick, vxlan_base, pods, t_begin, t_end)
    with ThreadPoolExecutor(len(parts_)) as ex:
        parts = list(ex.map(lambda r: reconcile(inp, tick, vxlan_base, pods, r[0], r[1]), parts_))

    def offs(name):
        out, base = [np.zeros(1, np.uint32)], 0
        for p in parts:
            o = getattr(p, name).astype(np.int64)
            out.append((o[1:] + base).astype(np.uint32))
            base += int(o[-1])
        return np.concatenate(out)
    cat = lambda name: np.concatenate([getattr(p, name) for p in parts])
    return BatchesOut(cat("action"), offs("del_off"), offs("add_off"), offs("upd_off"),
                      cat("del_idx"), cat("add_idx"), cat("upd_idx"), cat("del_res"), cat("add_res"),
                      cat("upd_res"), cat("add_qdisc"), cat("upd_qdisc"))


def _wire_lib():
    L = lib()
    if not getattr(L, "_wire_bound", False):
        L.or_utf8_valid.argtypes = [C.c_char_p, C.c_uint32]
        L.or_encode_batch.argtypes = [C.POINTER(abi.EpochIn), C.c_uint32, C.c_int, abi.u32p, C.c_uint32,
                                      C.c_void_p]
        L.or_encode_batch.restype = C.c_int64
        L.or_encode_epoch.argtypes = [C.POINTER(abi.EpochIn), C.POINTER(abi.Batches), C.c_uint32, C.c_void_p,
                                      C.c_void_p, C.c_void_p]
        L.or_encode_epoch.restype = C.c_uint64
        L._wire_bound = True
    return L


def utf8_valid(s) -> bool:
    b = _b(s)
    return _wire_lib().or_utf8_valid(b, len(b)) == 1


def encode_batch(inp: EpochInput, t: int, lst: int, idx) -> bytes | None:
    """proto.Marshal of the LinksBatchQuery Reconcile sends for topology t's list `lst`
    (0 DelLinks, 1 AddLinks, 2 UpdateLinks) of records `idx`; None = Marshal error."""
    L = _wire_lib()
    cin = inp.to_c()
    idx = np.ascontiguousarray(idx, dtype=np.uint32)
    ip = abi.ptr(idx if len(idx) else np.zeros(1, np.uint32), abi.u32p)
    n = L.or_encode_batch(C.byref(cin), t, lst, ip, len(idx), None)
    if n < 0:
        return None
    buf = (C.c_uint8 * max(n, 1))()
    L.or_encode_batch(C.byref(cin), t, lst, ip, len(idx), C.cast(buf, C.c_void_p))
    return bytes(buf)[:n]


def encode_epoch(inp: EpochInput, out: BatchesOut):
    """Wire bytes of every batch of an epoch: (arena uint8, off uint64[3T+1], err uint8[T])."""
    L = _wire_lib()
    T = inp.topos.n
    cin = inp.to_c()
    b = out.to_c((max(len(out.del_idx), 1), max(len(out.add_idx), 1), max(len(out.upd_idx), 1)))
    off = np.zeros(3 * T + 1, np.uint64)
    err = np.zeros(max(T, 1), np.uint8)
    n = L.or_encode_epoch(C.byref(cin), C.byref(b), T, None, off.ctypes.data, err.ctypes.data)
    arena = np.zeros(max(int(n), 1), np.uint8)
    L.or_encode_epoch(C.byref(cin), C.byref(b), T, arena.ctypes.data, off.ctypes.data, err.ctypes.data)
    return arena[:int(n)], off, err[:T]


def fanout(out: BatchesOut, T: int):
    """RemotePod fan-out per destination daemon: (node ids, off, entry idx)."""
    L = _wire_lib()
    if not getattr(L, "_fan_bound", False):
        L.or_fanout.argtypes = [C.POINTER(abi.Batches), C.c_uint32, C.c_void_p, C.c_void_p, C.c_void_p,
                                C.POINTER(C.c_uint32)]
        L.or_fanout.restype = C.c_uint32
        L._fan_bound = True
    b = out.to_c((max(len(out.del_idx), 1), max(len(out.add_idx), 1), max(len(out.upd_idx), 1)))
    n = max(len(out.add_idx), 1)
    node = np.zeros(n, np.uint32)
    off = np.zeros(n + 1, np.uint32)
    idx = np.zeros(n, np.uint32)
    nn = C.c_uint32()
    ns = L.or_fanout(C.byref(b), T, node.ctypes.data, off.ctypes.data, idx.ctypes.data, C.byref(nn))
    return node[:nn.value], off[:nn.value + 1], idx[:ns]


def tc_epoch(inp: EpochInput, out: BatchesOut):
    """tc argv arena (uint8) and command-slot offsets (uint64): two slots per add entry
    (LocalIntf, PeerIntf of a same-node veth pair), then one per update entry."""
    L = _wire_lib()
    if not getattr(L, "_tc_bound", False):
        L.or_tc_epoch.argtypes = [C.POINTER(abi.EpochIn), C.POINTER(abi.Batches), C.c_void_p, C.c_void_p]
        L.or_tc_epoch.restype = C.c_uint64
        L._tc_bound = True
    cin = inp.to_c()
    b = out.to_c((max(len(out.del_idx), 1), max(len(out.add_idx), 1), max(len(out.upd_idx), 1)))
    b.n_del, b.n_add, b.n_upd = len(out.del_idx), len(out.add_idx), len(out.upd_idx)
    off = np.zeros(2 * len(out.add_idx) + len(out.upd_idx) + 1, np.uint64)
    n = L.or_tc_epoch(C.byref(cin), C.byref(b), None, off.ctypes.data)
    arena = np.zeros(max(int(n), 1), np.uint8)
    L.or_tc_epoch(C.byref(cin), C.byref(b), arena.ctypes.data, off.ctypes.data)
    return arena[:int(n)], off


def remote_epoch(inp: EpochInput, out: BatchesOut, peer_netns=None):
    """RemotePod messages of an epoch (or_remote_epoch): (arena uint8, off uint64[n+1],
    entry uint32[n], n_remote, tc arena uint8, tc_off uint64[n+1]). The first n_remote are
    the UpdateRemote payloads in fan-out order, the rest the PHYSICAL local Updates.
    peer_netns: net_ns id per peer_topo index (default: this epoch's topologies)."""
    L = _wire_lib()
    if not getattr(L, "_remote_bound", False):
        L.or_remote_epoch.argtypes = [C.POINTER(abi.EpochIn), C.POINTER(abi.Batches), C.c_void_p, C.c_void_p,
                                      C.POINTER(C.c_uint32), C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p,
                                      C.POINTER(C.c_uint64), C.POINTER(C.c_uint64)]
        L.or_remote_epoch.restype = C.c_uint32
        L._remote_bound = True
    cin = inp.to_c()
    b = out.to_c((max(len(out.del_idx), 1), max(len(out.add_idx), 1), max(len(out.upd_idx), 1)))
    b.n_del, b.n_add, b.n_upd = len(out.del_idx), len(out.add_idx), len(out.upd_idx)
    pn = np.ascontiguousarray(inp.topos.net_ns if peer_netns is None else peer_netns, np.uint32)
    na = max(len(out.add_idx), 1)
    entry = np.zeros(na, np.uint32)
    off, tc_off = np.zeros(na + 1, np.uint64), np.zeros(na + 1, np.uint64)
    nr, nb, nt = C.c_uint32(), C.c_uint64(), C.c_uint64()
    args = lambda by, tc: (C.byref(cin), C.byref(b), pn.ctypes.data, entry.ctypes.data, C.byref(nr), by,
                           off.ctypes.data, tc, tc_off.ctypes.data, C.byref(nb), C.byref(nt))
    L.or_remote_epoch(*args(None, None))
    arena, tca = np.zeros(max(nb.value, 1), np.uint8), np.zeros(max(nt.value, 1), np.uint8)
    n = L.or_remote_epoch(*args(arena.ctypes.data, tca.ctypes.data))
    return arena[:nb.value], off[:n + 1], entry[:n], int(nr.value), tca[:nt.value], tc_off[:n + 1]


# ---- CR ingest (kdtn_oracle_json.c) ------------------------------------------------------
class JsonTables(C.Structure):
    _fields_ = [("json_err", C.c_int32), ("err_offset", C.c_uint64),
                ("T", C.c_uint32), ("N", C.c_uint32), ("M", C.c_uint32),
                ("n_kdict", C.c_uint32), ("n_pdict", C.c_uint32),
                ("kdict_bytes", C.c_uint64), ("pdict_bytes", C.c_uint64)] + [
        (f, C.c_void_p) for f in ("kd_bytes", "kd_offs", "pd_bytes", "pd_offs", "ns", "name",
                                  "src_ip", "net_ns", "flags", "real_off", "des_off",
                                  "des_key", "des_prop", "des_gap", "des_uid",
                                  "real_key", "real_prop", "real_gap", "real_uid")]


def _np(ptr, n, dtype):
    dtype = np.dtype(dtype)
    if n == 0 or not ptr:
        return np.zeros(n, dtype)
    buf = (C.c_uint8 * (n * dtype.itemsize)).from_address(ptr)
    return np.frombuffer(buf, dtype=dtype, count=n).copy()


def json_ingest(doc: bytes):
    """Go json.Unmarshal of a TopologyList document into the epoch tables.
    Returns (json_err, err_offset, EpochInput | None)."""
    from kdtn.tables import Links, StrTab, Topos
    L = lib()
    if not getattr(L, "_json_bound", False):
        L.or_json_ingest.argtypes = [C.c_char_p, C.c_uint64, C.POINTER(JsonTables)]
        L.or_json_free.argtypes = [C.POINTER(JsonTables)]
        L._json_bound = True
    t = JsonTables()
    if L.or_json_ingest(doc, len(doc), C.byref(t)) != 0:
        raise MemoryError("oracle json ingest")
    try:
        if t.json_err:
            return int(t.json_err), int(t.err_offset), None
        T, N, M = t.T, t.N, t.M

        def links(key, prop, gap, uid, n):
            return Links(_np(key, 7 * n, np.uint32).reshape(7, n),
                         _np(uid, n, np.int64),
                         _np(prop, 12 * n, np.uint32).reshape(12, n),
                         _np(gap, n, np.uint32))
        inp = EpochInput(
            StrTab(_np(t.kd_bytes, t.kdict_bytes, np.uint8), _np(t.kd_offs, t.n_kdict + 1, np.uint32)),
            StrTab(_np(t.pd_bytes, t.pdict_bytes, np.uint8), _np(t.pd_offs, t.n_pdict + 1, np.uint32)),
            Topos(_np(t.ns, T, np.uint32), _np(t.name, T, np.uint32), _np(t.src_ip, T, np.uint32),
                  _np(t.net_ns, T, np.uint32), _np(t.flags, T, np.uint8),
                  _np(t.real_off, T + 1, np.uint32), _np(t.des_off, T + 1, np.uint32)),
            links(t.real_key, t.real_prop, t.real_gap, t.real_uid, M),
            links(t.des_key, t.des_prop, t.des_gap, t.des_uid, N))
        return 0, 0, inp
    finally:
        L.or_json_free(C.byref(t))


def vni_contested(inp: EpochInput, out: BatchesOut, pod_netns=None):
    """Keys (node, vni) whose VxlanManager result depends on the goroutine order
    (or_vni_contested), in the order of their winning store."""
    L = _wire_lib()
    if not getattr(L, "_vnic_bound", False):
        L.or_vni_contested.argtypes = [C.POINTER(abi.Batches), C.c_uint32, C.c_void_p, C.c_void_p, C.c_void_p,
                                       C.c_void_p, C.c_void_p]
        L.or_vni_contested.restype = C.c_uint32
        L._vnic_bound = True
    T = inp.topos.n
    b = out.to_c((max(len(out.del_idx), 1), max(len(out.add_idx), 1), max(len(out.upd_idx), 1)))
    src = np.ascontiguousarray(inp.topos.src_ip, np.uint32)
    ns = np.ascontiguousarray(inp.topos.net_ns, np.uint32)
    pn = np.ascontiguousarray(ns if pod_netns is None else pod_netns, np.uint32)
    n = L.or_vni_contested(C.byref(b), T, src.ctypes.data, ns.ctypes.data, pn.ctypes.data, None, None)
    node, vni = np.zeros(max(n, 1), np.uint32), np.zeros(max(n, 1), np.int32)
    L.or_vni_contested(C.byref(b), T, src.ctypes.data, ns.ctypes.data, pn.ctypes.data, node.ctypes.data,
                       vni.ctypes.data)
    return node[:n], vni[:n]


def vni_apply(inp: EpochInput, out: BatchesOut, pod_netns=None):
    """VxlanManager maps after the epoch's reached entries (or_vni_apply): (node, vni, net_ns)
    arrays — the winning adds in (topology, add-list, local-before-remote) order, then the
    snapshot's surviving entries. pod_netns: net_ns id per global pod (default: this
    epoch's topologies)."""
    L = _wire_lib()
    if not getattr(L, "_vni_bound", False):
        L.or_vni_apply.argtypes = [C.POINTER(abi.Batches), C.c_uint32, C.c_void_p, C.c_void_p, C.c_void_p,
                                   C.POINTER(abi.VniTable), C.c_void_p, C.c_void_p, C.c_void_p]
        L.or_vni_apply.restype = C.c_uint32
        L._vni_bound = True
    T = inp.topos.n
    b = out.to_c((max(len(out.del_idx), 1), max(len(out.add_idx), 1), max(len(out.upd_idx), 1)))
    src = np.ascontiguousarray(inp.topos.src_ip, np.uint32)
    ns = np.ascontiguousarray(inp.topos.net_ns, np.uint32)
    pn = np.ascontiguousarray(ns if pod_netns is None else pod_netns, np.uint32)
    vt = inp.vnis.to_c()
    n = L.or_vni_apply(C.byref(b), T, src.ctypes.data, ns.ctypes.data, pn.ctypes.data, C.byref(vt), None, None, None)
    node, vni, net = np.zeros(max(n, 1), np.uint32), np.zeros(max(n, 1), np.int32), np.zeros(max(n, 1), np.uint32)
    L.or_vni_apply(C.byref(b), T, src.ctypes.data, ns.ctypes.data, pn.ctypes.data, C.byref(vt), node.ctypes.data,
                   vni.ctypes.data, net.ctypes.data)
    return node[:n], vni[:n], net[:n]
