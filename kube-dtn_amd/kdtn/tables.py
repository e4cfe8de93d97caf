"""Struct-of-arrays containers for one reconcile epoch, mirroring include/kdtn.h.

Every table is a set of contiguous numpy columns; `EpochInput.to_c()` produces the
`kdtn_epoch_in` the C-ABI expects (pointers into these arrays, which must stay alive for
the duration of the call — the engine copies them to HBM and keeps no pointer).
"""
from __future__ import annotations

from dataclasses import dataclass, field

import numpy as np

from . import abi


class Interner:
    """Python-side string interner: deduplicated dictionary, id 0 = "" (kdtn.h contract)."""

    def __init__(self) -> None:
        self._ids: dict[bytes, int] = {b"": 0}
        self._strs: list[bytes] = [b""]

    def __call__(self, s) -> int:
        b = s.encode() if isinstance(s, str) else bytes(s)
        i = self._ids.get(b)
        if i is None:
            i = len(self._strs)
            self._ids[b] = i
            self._strs.append(b)
        return i

    def __len__(self) -> int:
        return len(self._strs)

    def table(self) -> "StrTab":
        return StrTab.from_list(self._strs)


@dataclass
class StrTab:
    bytes_: np.ndarray   # uint8 arena
    offs: np.ndarray     # uint32, n + 1

    @classmethod
    def from_list(cls, strs) -> "StrTab":
        bs = [s.encode() if isinstance(s, str) else bytes(s) for s in strs]
        lens = np.fromiter((len(b) for b in bs), dtype=np.uint64, count=len(bs))
        offs = np.zeros(len(bs) + 1, dtype=np.uint64)
        np.cumsum(lens, out=offs[1:])
        assert offs[-1] < 2**32, "dictionary arena over 4 GiB"
        arena = np.frombuffer(b"".join(bs), dtype=np.uint8).copy() if bs else np.zeros(0, np.uint8)
        return cls(arena, offs.astype(np.uint32))

    @property
    def n(self) -> int:
        return len(self.offs) - 1

    def get(self, i: int) -> bytes:
        return self.bytes_[self.offs[i]:self.offs[i + 1]].tobytes()

    def to_c(self) -> abi.Strtab:
        b = self.bytes_ if len(self.bytes_) else np.zeros(1, np.uint8)
        self._keep = b
        return abi.Strtab(abi.ptr(b, abi.u8p), abi.ptr(self.offs, abi.u32p), self.n)


@dataclass
class Links:
    """Link records grouped by topology: key (NKEY,n) u32, uid (n,) i64, prop (NPROP,n) u32, gap (n,) u32."""
    key: np.ndarray
    uid: np.ndarray
    prop: np.ndarray
    gap: np.ndarray

    @classmethod
    def empty(cls, n: int = 0) -> "Links":
        return cls(np.zeros((abi.NKEY, n), np.uint32), np.zeros(n, np.int64),
                   np.zeros((abi.NPROP, n), np.uint32), np.zeros(n, np.uint32))

    @property
    def n(self) -> int:
        return int(self.uid.shape[0])

    def take(self, idx) -> "Links":
        idx = np.asarray(idx, dtype=np.int64)
        return Links(np.ascontiguousarray(self.key[:, idx]), self.uid[idx].copy(),
                     np.ascontiguousarray(self.prop[:, idx]), self.gap[idx].copy())

    def to_c(self) -> abi.LinkTable:
        self.key = np.ascontiguousarray(self.key, dtype=np.uint32)
        self.prop = np.ascontiguousarray(self.prop, dtype=np.uint32)
        self.uid = np.ascontiguousarray(self.uid, dtype=np.int64)
        self.gap = np.ascontiguousarray(self.gap, dtype=np.uint32)
        t = abi.LinkTable()
        t.n = self.n
        for k in range(abi.NKEY):
            t.key[k] = abi.ptr(self.key[k], abi.u32p)
        t.uid = abi.ptr(self.uid, abi.i64p)
        for k in range(abi.NPROP):
            t.prop[k] = abi.ptr(self.prop[k], abi.u32p)
        t.gap = abi.ptr(self.gap, abi.u32p)
        return t


@dataclass
class Topos:
    ns: np.ndarray
    name: np.ndarray
    src_ip: np.ndarray
    net_ns: np.ndarray
    flags: np.ndarray
    real_off: np.ndarray
    des_off: np.ndarray

    @property
    def n(self) -> int:
        return int(self.ns.shape[0])

    def to_c(self) -> abi.TopoTable:
        for f in ("ns", "name", "src_ip", "net_ns", "real_off", "des_off"):
            setattr(self, f, np.ascontiguousarray(getattr(self, f), dtype=np.uint32))
        self.flags = np.ascontiguousarray(self.flags, dtype=np.uint8)
        return abi.TopoTable(self.n, abi.ptr(self.ns, abi.u32p), abi.ptr(self.name, abi.u32p),
                             abi.ptr(self.src_ip, abi.u32p), abi.ptr(self.net_ns, abi.u32p),
                             abi.ptr(self.flags, abi.u8p), abi.ptr(self.real_off, abi.u32p),
                             abi.ptr(self.des_off, abi.u32p))


@dataclass
class Vnis:
    node: np.ndarray = field(default_factory=lambda: np.zeros(0, np.uint32))
    vni: np.ndarray = field(default_factory=lambda: np.zeros(0, np.int32))
    net_ns: np.ndarray = field(default_factory=lambda: np.zeros(0, np.uint32))
    resident: bool = False      # KDTN_VNI_RESIDENT: the engine keeps its own map (no upload)

    @classmethod
    def keep_resident(cls) -> "Vnis":
        return cls(resident=True)

    @property
    def n(self) -> int:
        return int(self.node.shape[0])

    def to_c(self) -> abi.VniTable:
        if self.resident:
            return abi.VniTable(abi.VNI_RESIDENT, None, None, None)
        self.node = np.ascontiguousarray(self.node, dtype=np.uint32)
        self.vni = np.ascontiguousarray(self.vni, dtype=np.int32)
        self.net_ns = np.ascontiguousarray(self.net_ns, dtype=np.uint32)
        if self.n == 0:
            return abi.VniTable(0, None, None, None)
        return abi.VniTable(self.n, abi.ptr(self.node, abi.u32p), abi.ptr(self.vni, abi.i32p),
                            abi.ptr(self.net_ns, abi.u32p))


@dataclass
class EpochInput:
    kdict: StrTab
    pdict: StrTab
    topos: Topos
    realised: Links
    desired: Links
    vnis: Vnis = field(default_factory=Vnis)
    pod_slice: int = 0
    pod_base: int = 0            # global pod index of topology 0 (multi-shard)
    owner: object = None         # keeps a generator's memory alive
    gid: np.ndarray | None = None    # synthetic workloads: global pod id of each local topology

    def to_c(self) -> abi.EpochIn:
        c = abi.EpochIn(self.kdict.to_c(), self.pdict.to_c(), self.topos.to_c(),
                        self.realised.to_c(), self.desired.to_c(), self.vnis.to_c(),
                        self.pod_slice)
        return c


@dataclass
class BatchesOut:
    """Host-side epoch outputs (kdtn_batches), trimmed to the returned counts."""
    action: np.ndarray
    del_off: np.ndarray
    add_off: np.ndarray
    upd_off: np.ndarray
    del_idx: np.ndarray
    add_idx: np.ndarray
    upd_idx: np.ndarray
    del_res: np.ndarray
    add_res: np.ndarray
    upd_res: np.ndarray
    add_qdisc: np.ndarray
    upd_qdisc: np.ndarray

    @classmethod
    def alloc(cls, T: int, cap_del: int, cap_add: int, cap_upd: int, pinned: bool = False) -> "BatchesOut":
        if pinned:                                       # page-locked host memory (kdtn_host_alloc)
            from .engine import pinned_empty
            z = pinned_empty
        else:
            z = np.zeros
        return cls(z(T, np.uint8), z(T + 1, np.uint32), z(T + 1, np.uint32), z(T + 1, np.uint32),
                   z(max(cap_del, 1), np.uint32), z(max(cap_add, 1), np.uint32),
                   z(max(cap_upd, 1), np.uint32),
                   z(max(cap_del, 1), abi.RESOLVED_DTYPE), z(max(cap_add, 1), abi.RESOLVED_DTYPE),
                   z(max(cap_upd, 1), abi.RESOLVED_DTYPE),
                   z(max(cap_add, 1), abi.QDISC_DTYPE), z(max(cap_upd, 1), abi.QDISC_DTYPE))

    def to_c(self, caps) -> abi.Batches:
        b = abi.Batches()
        b.action = abi.ptr(self.action, abi.u8p)
        b.del_off = abi.ptr(self.del_off, abi.u32p)
        b.add_off = abi.ptr(self.add_off, abi.u32p)
        b.upd_off = abi.ptr(self.upd_off, abi.u32p)
        b.del_idx = abi.ptr(self.del_idx, abi.u32p)
        b.add_idx = abi.ptr(self.add_idx, abi.u32p)
        b.upd_idx = abi.ptr(self.upd_idx, abi.u32p)
        b.del_res = self.del_res.ctypes.data
        b.add_res = self.add_res.ctypes.data
        b.upd_res = self.upd_res.ctypes.data
        b.add_qdisc = self.add_qdisc.ctypes.data
        b.upd_qdisc = self.upd_qdisc.ctypes.data
        b.del_cap, b.add_cap, b.upd_cap = caps
        return b

    def trim(self, n_del: int, n_add: int, n_upd: int) -> "BatchesOut":
        return BatchesOut(self.action, self.del_off, self.add_off, self.upd_off,
                          self.del_idx[:n_del], self.add_idx[:n_add], self.upd_idx[:n_upd],
                          self.del_res[:n_del], self.add_res[:n_add], self.upd_res[:n_upd],
                          self.add_qdisc[:n_add], self.upd_qdisc[:n_upd])

    FIELDS = ("action", "del_off", "add_off", "upd_off", "del_idx", "add_idx", "upd_idx",
              "del_res", "add_res", "upd_res", "add_qdisc", "upd_qdisc")

    def mismatches(self, other: "BatchesOut") -> list[str]:
        """Names of the fields that differ bit-for-bit from `other` (empty list = identical)."""
        bad = []
        for f in self.FIELDS:
            a, b = getattr(self, f), getattr(other, f)
            if a.shape != b.shape or a.tobytes() != b.tobytes():
                bad.append(f)
        return bad
