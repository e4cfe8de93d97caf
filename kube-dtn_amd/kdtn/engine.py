"""Python binding of libkdtn.so (the MI355X engine behind include/kdtn.h).

The library is loaded from this package directory (built in-tree by `make -C kube-dtn_amd`).
There is no fallback: if the HIP library is missing or no gfx950 device is visible the
calls raise — the reconcile path only runs on the GPU.
"""
from __future__ import annotations

import atexit
import ctypes as C
import os
import weakref

import numpy as np

from . import abi
from .tables import BatchesOut, EpochInput, StrTab, Vnis

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, "libkdtn.so")
_lib = None
PROF_LIB_PATH = os.path.join(os.path.dirname(_HERE), "prof", "libkdtn_prof.so")


def use_profiling_library() -> None:
    """tools/ only: bind the profiling build (make -C kube-dtn_amd prof), whose A/B kernel
    variants are selected from KDTN_VARIANT / KDTN_KD_SUB / KDTN_JS_VARIANT. The product
    library kdtn/libkdtn.so reads no environment variable. Call before the first Engine."""
    global LIB_PATH
    if _lib is not None and LIB_PATH != PROF_LIB_PATH:
        raise RuntimeError("libkdtn.so is already loaded in this process")
    LIB_PATH = PROF_LIB_PATH


class KdtnError(RuntimeError):
    def __init__(self, code: int, what: str):
        super().__init__(f"{what}: {code} ({lib().kdtn_strerror(code).decode()})")
        self.code = code


def lib() -> C.CDLL:
    """Load libkdtn.so; raises ImportError when it has not been built."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise ImportError(f"libkdtn.so not built ({LIB_PATH}); run `make -C kube-dtn_amd`")
    # One HIP runtime per process: PyTorch-ROCm ships libamdhip64.so.7 / librccl.so.1 with the
    # same SONAMEs libkdtn.so links against. Loading torch first makes libkdtn bind to those
    # already-loaded copies instead of mapping a second runtime from /opt/rocm.
    try:
        import torch  # noqa: F401
    except ImportError:
        pass
    L = C.CDLL(LIB_PATH)
    vp = C.c_void_p
    sig = {
        "kdtn_version": (C.c_char_p, []),
        "kdtn_strerror": (C.c_char_p, [C.c_int]),
        "kdtn_err_name": (C.c_char_p, [C.c_int]),
        "kdtn_init": (C.c_int, [C.POINTER(vp), C.POINTER(abi.Config)]),
        "kdtn_destroy": (None, [vp]),
        "kdtn_set_stream": (C.c_int, [vp, vp]),
        "kdtn_psched_tick_in_usec": (C.c_double, []),
        "kdtn_interner_new": (C.c_int, [C.POINTER(vp)]),
        "kdtn_interner_free": (None, [vp]),
        "kdtn_intern": (C.c_uint32, [vp, C.c_char_p, C.c_uint32]),
        "kdtn_intern_batch": (C.c_int, [vp, abi.u8p, abi.u64p, C.c_uint32, abi.u32p]),
        "kdtn_interner_table": (C.c_int, [vp, C.POINTER(abi.Strtab)]),
        "kdtn_reconcile_epoch": (C.c_int, [vp, C.POINTER(abi.EpochIn), C.POINTER(abi.Batches)]),
        "kdtn_epoch_upload": (C.c_int, [vp, C.POINTER(abi.EpochIn)]),
        "kdtn_epoch_run": (C.c_int, [vp, C.c_uint32]),
        "kdtn_epoch_sync": (C.c_int, [vp, C.POINTER(abi.Counts)]),
        "kdtn_epoch_download": (C.c_int, [vp, C.POINTER(abi.Batches)]),
        "kdtn_make_qdiscs": (C.c_int, [vp, C.POINTER(abi.Strtab), C.POINTER(abi.PropsTable), vp]),
        "kdtn_comm_unique_id": (C.c_int, [C.POINTER(C.c_uint8 * 128)]),
        "kdtn_comm_init": (C.c_int, [vp, C.POINTER(C.c_uint8 * 128), C.c_int, C.c_int]),
        "kdtn_set_timing": (C.c_int, [vp, C.c_int]),
        "kdtn_epoch_vni_apply": (C.c_int, [vp, C.POINTER(abi.VniState)]),
        "kdtn_vni_contested": (C.c_int, [vp, vp, vp, C.c_uint32, C.POINTER(C.c_uint32)]),
        "kdtn_vni_download": (C.c_int, [vp, C.POINTER(abi.VniState)]),
        "kdtn_last_kernel_times": (C.c_int, [vp, C.POINTER(C.c_char_p), C.POINTER(C.c_float), C.c_int]),
        "kdtn_timer_totals": (C.c_int, [vp, C.POINTER(C.c_char_p), C.POINTER(C.c_double),
                                        C.POINTER(C.c_uint32), C.c_int, C.c_int]),
        "kdtn_debug_wg_trace": (C.c_int, [vp, C.POINTER(C.c_uint64), C.c_uint32]),
        "kdtn_epoch_encode": (C.c_int, [vp, C.POINTER(C.c_uint64)]),
        "kdtn_diff": (C.c_int, [vp, C.POINTER(abi.EpochIn), C.POINTER(abi.Batches)]),
        "kdtn_resolve": (C.c_int, [vp, C.POINTER(abi.Strtab), C.POINTER(abi.Strtab), C.POINTER(abi.PodTable),
                                   C.c_uint32, C.POINTER(abi.LinkTable), C.c_int, C.POINTER(abi.VniTable),
                                   vp, vp]),
        "kdtn_host_alloc": (vp, [C.c_uint64]),
        "kdtn_epoch_fanout": (C.c_int, [vp, C.POINTER(abi.Fanout)]),
        "kdtn_epoch_tc": (C.c_int, [vp, C.POINTER(C.c_uint64)]),
        "kdtn_epoch_download_tc": (C.c_int, [vp, C.POINTER(abi.TcArgv)]),
        "kdtn_host_free": (None, [vp]),
        "kdtn_epoch_download_wire": (C.c_int, [vp, C.POINTER(abi.Wire)]),
        "kdtn_json_upload": (C.c_int, [vp, C.c_char_p, C.c_uint64]),
        "kdtn_json_ingest": (C.c_int, [vp, C.POINTER(abi.VniTable), C.POINTER(abi.IngestInfo)]),
        "kdtn_ingest_download": (C.c_int, [vp, C.POINTER(abi.IngestTables)]),
        "kdtn_json_ingest_shard": (C.c_int, [vp, C.POINTER(abi.VniTable), C.c_uint32, C.c_uint32,
                                             C.POINTER(abi.IngestInfo)]),
        "kdtn_ingest_shard_topos": (C.c_int, [vp, vp]),
        "kdtn_topology_shard": (C.c_uint32, [C.c_char_p, C.c_uint32, C.c_char_p, C.c_uint32, C.c_uint32]),
        "kdtn_comm_set_ranks": (C.c_int, [vp, C.c_int, C.c_int]),
        "kdtn_pods_export": (C.c_int, [vp, vp]),
        "kdtn_pods_import": (C.c_int, [vp, vp, C.c_uint64]),
        "kdtn_epoch_remote_encode": (C.c_int, [vp, C.POINTER(abi.RemoteInfo)]),
        "kdtn_epoch_commit": (C.c_int, [vp, vp, C.POINTER(C.c_uint32)]),
        "kdtn_vni_ops_export": (C.c_int, [vp, vp, C.c_uint32, vp, C.c_uint32, C.POINTER(C.c_uint32),
                                          C.POINTER(C.c_uint32)]),
        "kdtn_vni_ops_import": (C.c_int, [vp, vp, C.c_uint32, vp, C.c_uint32]),
        "kdtn_epoch_upload_delta": (C.c_int, [vp, C.POINTER(abi.EpochDelta)]),
        "kdtn_epoch_tables_info": (C.c_int, [vp, C.POINTER(abi.IngestInfo)]),
        "kdtn_epoch_download_remote": (C.c_int, [vp, C.POINTER(abi.RemotePods)]),
        "kdtn_json_ingest_delta": (C.c_int, [vp, vp, C.c_uint32, C.POINTER(abi.VniTable), C.POINTER(abi.IngestInfo)]),
        "kdtn_epoch_download_async": (C.c_int, [vp, C.POINTER(abi.Batches)]),
        "kdtn_epoch_download_wait": (C.c_int, [vp]),
        "kdtn_epoch_late_pods": (C.c_int, [vp, vp, C.c_uint32]),
    }
    for name, (res, args) in sig.items():
        f = getattr(L, name)
        f.restype = res
        f.argtypes = args
    _lib = L
    # registered after torch's import, so it runs before the HIP runtime's own teardown
    atexit.register(_teardown)
    return L


# Live contexts and page-locked buffers. At interpreter exit the contexts are destroyed (their
# streams drained) and only then the page-locked buffers freed, while the HIP runtime is still
# up — not from weakref finalizers in whatever order shutdown reaches them.
_engines: "weakref.WeakSet[Engine]" = weakref.WeakSet()
_pinned: dict[int, weakref.finalize] = {}


def _teardown() -> None:
    for e in list(_engines):
        try:
            e.close()
        except Exception:
            pass
    for f in list(_pinned.values()):
        f()
    _pinned.clear()


def _host_free(p: int) -> None:
    _pinned.pop(p, None)
    if _lib is not None:
        _lib.kdtn_host_free(p)


def _check(code: int, what: str) -> None:
    if code != abi.OK:
        raise KdtnError(code, what)


def pinned_empty(shape, dtype) -> np.ndarray:
    """A numpy array in page-locked host memory (kdtn_host_alloc), freed with the array."""
    dtype = np.dtype(dtype)
    n = int(np.prod(shape, dtype=np.int64)) * dtype.itemsize
    L = lib()
    p = L.kdtn_host_alloc(max(n, 1))
    if not p:
        raise MemoryError(f"kdtn_host_alloc({n})")
    buf = (C.c_uint8 * max(n, 1)).from_address(p)
    f = weakref.finalize(buf, _host_free, p)
    f.atexit = False                       # _teardown frees it, after the contexts
    _pinned[p] = f
    return np.frombuffer(buf, dtype=np.uint8, count=n).view(dtype).reshape(shape)


def pinned_copy(a: np.ndarray) -> np.ndarray:
    out = pinned_empty(a.shape, a.dtype)
    out[...] = a
    return out


def pin_input(inp: EpochInput) -> EpochInput:
    """The epoch tables copied into page-locked host memory (what a controller that packs its
    SoA straight into kdtn_host_alloc buffers uploads from)."""
    from .tables import Links, Topos
    P = pinned_copy
    links = lambda L: Links(P(np.ascontiguousarray(L.key)), P(L.uid), P(np.ascontiguousarray(L.prop)), P(L.gap))
    T = inp.topos
    out = EpochInput(StrTab(P(inp.kdict.bytes_), P(inp.kdict.offs)), StrTab(P(inp.pdict.bytes_), P(inp.pdict.offs)),
                     Topos(*[P(getattr(T, f)) for f in ("ns", "name", "src_ip", "net_ns", "flags", "real_off",
                                                        "des_off")]),
                     links(inp.realised), links(inp.desired), Vnis(P(inp.vnis.node), P(inp.vnis.vni), P(inp.vnis.net_ns)),
                     pod_slice=inp.pod_slice, pod_base=inp.pod_base)
    out.total_pods, out.gid = getattr(inp, "total_pods", 0), inp.gid
    return out


def delta_pack_layout(n: int, nref: int, remap_T: int) -> dict:
    """Byte offsets of a delta's arrays in the engine's device block (kdtn_engine.hip
    DeltaPack): arrays placed at these offsets in one host block travel in one copy."""
    o = {"topo": 0, "src_ip": 4 * n, "net_ns": 8 * n, "des_off": 12 * n}
    o["prev"] = o["des_off"] + (4 * (n + 1) if n else 0)
    o["ns"] = o["prev"] + 4 * remap_T
    o["name"] = o["ns"] + (4 * n if remap_T else 0)
    o["spec_nil"] = o["name"] + (4 * n if remap_T else 0)
    o["ref"] = (o["spec_nil"] + n + 3) // 4 * 4
    o["total"] = o["ref"] + 4 * nref
    return o


def pin_delta(d):
    """A kdtn.delta.Delta copied into page-locked host memory; its per-Topology arrays and
    references share one block in the engine's layout (delta_pack_layout)."""
    from dataclasses import replace
    from .tables import Links
    P = pinned_copy
    r = d.records
    n, nref = d.n_changed, len(d.ref)
    remap_T = 0 if d.prev is None else len(d.prev)
    lay = delta_pack_layout(n, nref, remap_T)
    block = pinned_empty((max(lay["total"], 1),), np.uint8)
    arrs = {}
    for f, dt in (("topo", np.uint32), ("src_ip", np.uint32), ("net_ns", np.uint32), ("des_off", np.uint32),
                  ("prev", np.uint32), ("ns", np.uint32), ("name", np.uint32), ("spec_nil", np.uint8),
                  ("ref", np.uint32)):
        a = getattr(d, f)
        if a is None:
            continue
        a = np.ascontiguousarray(a, dt)
        view = block[lay[f]:lay[f] + a.nbytes].view(dt)
        view[...] = a
        arrs[f] = view
    v = d.vnis
    vn = v if v.resident else Vnis(P(v.node), P(v.vni), P(v.net_ns))
    out = replace(d, kdict=StrTab(P(d.kdict.bytes_), P(d.kdict.offs)), pdict=StrTab(P(d.pdict.bytes_), P(d.pdict.offs)),
                  vnis=vn, records=Links(P(np.ascontiguousarray(r.key)), P(r.uid), P(np.ascontiguousarray(r.prop)),
                                         P(r.gap)), **arrs)
    out._block = block
    return out


def topology_shard(namespace, name, nshards: int) -> int:
    """Owner shard of a Topology: hash64(namespace/name) mod nshards (kdtn_topology_shard)."""
    ns = namespace.encode() if isinstance(namespace, str) else bytes(namespace)
    nm = name.encode() if isinstance(name, str) else bytes(name)
    return int(lib().kdtn_topology_shard(ns, len(ns), nm, len(nm), nshards))


def comm_unique_id() -> bytes:
    buf = (C.c_uint8 * 128)()
    _check(lib().kdtn_comm_unique_id(C.byref(buf)), "kdtn_comm_unique_id")
    return bytes(buf)


class Engine:
    """One kdtn_ctx: a reconcile engine bound to one MI355X (gfx950) device."""

    def __init__(self, device: int = 0, tick_in_usec: float | None = None, vxlan_base: int = 5000):
        L = lib()
        if tick_in_usec is None:
            tick_in_usec = L.kdtn_psched_tick_in_usec()
        self.tick_in_usec = float(tick_in_usec)
        self.vxlan_base = int(vxlan_base)
        cfg = abi.Config(device, vxlan_base, self.tick_in_usec)
        ctx = C.c_void_p()
        _check(L.kdtn_init(C.byref(ctx), C.byref(cfg)), "kdtn_init")
        self._ctx = ctx
        self._T = 0
        self._caps = (0, 0, 0)
        _engines.add(self)

    def close(self) -> None:
        """Drain an outstanding kdtn_epoch_download_async, then kdtn_destroy (which waits for
        every stream of the context before it frees anything)."""
        if self._ctx:
            L = lib()
            L.kdtn_epoch_download_wait(self._ctx)
            L.kdtn_destroy(self._ctx)
            self._ctx = None
            self._dl_keep = None

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    # ---- multi-GPU -------------------------------------------------------------------
    def comm_init(self, unique_id: bytes, nranks: int, rank: int) -> None:
        buf = (C.c_uint8 * 128).from_buffer_copy(unique_id)
        _check(lib().kdtn_comm_init(self._ctx, C.byref(buf), nranks, rank), "kdtn_comm_init")

    def set_ranks(self, nranks: int, rank: int) -> None:
        """Host transport for the pod-status exchange (kdtn_comm_set_ranks): per epoch,
        pods_export → all-gather by the caller → pods_import → run."""
        _check(lib().kdtn_comm_set_ranks(self._ctx, nranks, rank), "kdtn_comm_set_ranks")

    def pods_export(self, pod_slice: int) -> np.ndarray:
        """This rank's pod-status rows (pod_slice × 4 u32: ns, name, src_ip, net_ns|nil<<31)."""
        rows = np.zeros((max(pod_slice, 1), 4), np.uint32)
        _check(lib().kdtn_pods_export(self._ctx, rows.ctypes.data), "kdtn_pods_export")
        return rows[:pod_slice]

    def pods_import(self, rows: np.ndarray) -> None:
        """The gathered table of every rank's rows, rank order ((pod_slice*nranks) × 4 u32)."""
        rows = np.ascontiguousarray(rows, dtype=np.uint32)
        _check(lib().kdtn_pods_import(self._ctx, rows.ctypes.data, rows.shape[0]), "kdtn_pods_import")

    def late_pods(self, rows: np.ndarray) -> None:
        """kdtn_epoch_late_pods: pod rows (n × 4 u32 as pods_export gives them) of Topologies
        the informer store missed and the API server returned (getPod's fallback,
        handler.go:35-39); they join the peer lookup of the following runs as global pod
        indices nranks*pod_slice + i."""
        rows = np.ascontiguousarray(rows, dtype=np.uint32).reshape(-1, 4)
        _check(lib().kdtn_epoch_late_pods(self._ctx, rows.ctypes.data if len(rows) else None, len(rows)),
               "kdtn_epoch_late_pods")

    def set_stream(self, stream_handle: int | None) -> None:
        _check(lib().kdtn_set_stream(self._ctx, C.c_void_p(stream_handle or 0)), "kdtn_set_stream")

    # ---- epoch -----------------------------------------------------------------------
    def upload(self, inp: EpochInput, kdict_keep: int = 0, pdict_keep: int = 0) -> None:
        """kdtn_epoch_upload. kdict_keep / pdict_keep: the dictionaries extend the previous
        upload's first that many strings (append-only interning): only the suffix is
        uploaded and parsed."""
        cin = inp.to_c()
        cin.kdict_keep, cin.pdict_keep = kdict_keep, pdict_keep
        _check(lib().kdtn_epoch_upload(self._ctx, C.byref(cin)), "kdtn_epoch_upload")
        self._T = inp.topos.n
        self._caps = (inp.realised.n, inp.desired.n, inp.realised.n)

    def json_upload(self, doc: bytes) -> None:
        """H2D of a TopologyList JSON document (kdtn_json_upload)."""
        _check(lib().kdtn_json_upload(self._ctx, doc, len(doc)), "kdtn_json_upload")

    def json_ingest(self, vnis=None, shard=None) -> abi.IngestInfo:
        """Decode the uploaded document on the GPU into device-resident epoch inputs
        (kdtn_json_ingest). A rejected document raises KdtnError(EBADMSG) whose .info holds
        json_err / err_offset. shard=(nshards, rank): the whole document decoded, the epoch
        cut down to that rank's Topologies (kdtn_json_ingest_shard)."""
        info = abi.IngestInfo()
        cv = vnis.to_c() if vnis is not None else None
        pv = C.byref(cv) if cv is not None else None
        if shard is None:
            name, rc = "kdtn_json_ingest", lib().kdtn_json_ingest(self._ctx, pv, C.byref(info))
        else:
            name = "kdtn_json_ingest_shard"
            rc = lib().kdtn_json_ingest_shard(self._ctx, pv, int(shard[0]), int(shard[1]), C.byref(info))
        if rc == abi.EBADMSG:
            e = KdtnError(rc, name)
            e.info = info
            raise e
        _check(rc, name)
        self._T = info.n_topos
        self._caps = (info.n_realised, info.n_desired, info.n_realised)
        self._ingest = info
        return info

    def ingest_delta(self, doc: bytes, deleted=None, vnis=None) -> abi.IngestInfo:
        """kdtn_json_ingest_delta: the added / updated Topology CRs (a TopologyList document)
        and the resident indices of the deleted ones applied to the resident state; their
        strings are interned into the resident dictionaries. vnis None keeps the resident
        VXLAN map."""
        self.json_upload(doc)
        info = abi.IngestInfo()
        dl = np.ascontiguousarray(deleted if deleted is not None else np.zeros(0), dtype=np.uint32)
        cv = vnis.to_c() if vnis is not None else None
        rc = lib().kdtn_json_ingest_delta(self._ctx, dl.ctypes.data if len(dl) else None, len(dl),
                                          C.byref(cv) if cv is not None else None, C.byref(info))
        if rc == abi.EBADMSG:
            e = KdtnError(rc, "kdtn_json_ingest_delta")
            e.info = info
            raise e
        _check(rc, "kdtn_json_ingest_delta")
        self._T = info.n_topos
        self._caps = (info.n_realised, info.n_desired, info.n_realised)
        return info

    def ingest(self, doc: bytes, vnis=None, shard=None) -> abi.IngestInfo:
        self.json_upload(doc)
        return self.json_ingest(vnis, shard)

    def ingest_doc_index(self) -> np.ndarray:
        """Document index of each topology of the last ingest (kdtn_ingest_shard_topos)."""
        out = np.zeros(max(self._T, 1), np.uint32)
        _check(lib().kdtn_ingest_shard_topos(self._ctx, out.ctypes.data), "kdtn_ingest_shard_topos")
        return out[:self._T]

    def tables(self) -> EpochInput:
        """D2H of the context's current epoch tables (kdtn_epoch_tables_info +
        kdtn_ingest_download): the resident state after a commit or delta upload."""
        info = abi.IngestInfo()
        _check(lib().kdtn_epoch_tables_info(self._ctx, C.byref(info)), "kdtn_epoch_tables_info")
        self._ingest = info
        return self.ingest_tables()

    def ingest_tables(self) -> EpochInput:
        """D2H of the tables the last json_ingest decoded (kdtn_ingest_download)."""
        from .tables import Links, StrTab, Topos
        I = self._ingest
        T, N, M = I.n_topos, I.n_desired, I.n_realised
        z = np.zeros
        kd, kdo = z(max(I.kdict_bytes, 1), np.uint8), z(I.n_kdict + 1, np.uint32)
        pd, pdo = z(max(I.pdict_bytes, 1), np.uint8), z(I.n_pdict + 1, np.uint32)
        tp = [z(T, np.uint32) for _ in range(4)] + [z(T, np.uint8), z(T + 1, np.uint32), z(T + 1, np.uint32)]

        def links(n):
            return Links(z((abi.NKEY, n), np.uint32), z(n, np.int64), z((abi.NPROP, n), np.uint32),
                         z(n, np.uint32))
        des, real = links(N), links(M)
        t = abi.IngestTables()
        for f, a in (("kd_bytes", kd), ("kd_offs", kdo), ("pd_bytes", pd), ("pd_offs", pdo),
                     ("ns", tp[0]), ("name", tp[1]), ("src_ip", tp[2]), ("net_ns", tp[3]),
                     ("flags", tp[4]), ("real_off", tp[5]), ("des_off", tp[6]),
                     ("des_key", des.key), ("des_prop", des.prop), ("des_gap", des.gap), ("des_uid", des.uid),
                     ("real_key", real.key), ("real_prop", real.prop), ("real_gap", real.gap),
                     ("real_uid", real.uid)):
            setattr(t, f, a.ctypes.data if a.size else None)
        _check(lib().kdtn_ingest_download(self._ctx, C.byref(t)), "kdtn_ingest_download")
        return EpochInput(StrTab(kd[:I.kdict_bytes], kdo), StrTab(pd[:I.pdict_bytes], pdo),
                          Topos(*tp), real, des)

    # ---- resident state: status commit and delta upload -----------------------------------
    def commit(self, mask=None) -> int:
        """kdtn_epoch_commit: Status.Links = Spec.Links on the device for the committed
        Topologies (mask None: the engine's prediction; else mask[t] != 0). Returns how many."""
        n = C.c_uint32()
        m = None if mask is None else np.ascontiguousarray(mask, dtype=np.uint8)
        _check(lib().kdtn_epoch_commit(self._ctx, m.ctypes.data if m is not None else None, C.byref(n)),
               "kdtn_epoch_commit")
        info = self.state_sizes()
        self._caps = (info.n_realised, info.n_desired, info.n_realised)
        return int(n.value)

    def upload_delta(self, delta) -> None:
        """kdtn_epoch_upload_delta: the next epoch as a delta (kdtn.delta.Delta) against the
        resident state."""
        cd = delta.to_c()
        _check(lib().kdtn_epoch_upload_delta(self._ctx, C.byref(cd)), "kdtn_epoch_upload_delta")
        info = abi.IngestInfo()
        _check(lib().kdtn_epoch_tables_info(self._ctx, C.byref(info)), "kdtn_epoch_tables_info")
        self._T = info.n_topos
        self._caps = (info.n_realised, info.n_desired, info.n_realised)

    def state_sizes(self) -> abi.IngestInfo:
        info = abi.IngestInfo()
        _check(lib().kdtn_epoch_tables_info(self._ctx, C.byref(info)), "kdtn_epoch_tables_info")
        return info

    def run(self, stages: int = abi.STAGE_ALL) -> None:
        _check(lib().kdtn_epoch_run(self._ctx, stages), "kdtn_epoch_run")

    def sync(self) -> abi.Counts:
        c = abi.Counts()
        _check(lib().kdtn_epoch_sync(self._ctx, C.byref(c)), "kdtn_epoch_sync")
        return c

    def download(self, into: BatchesOut | None = None) -> BatchesOut:
        """kdtn_epoch_download into fresh arrays, or into `into` (e.g. BatchesOut.alloc with
        pinned=True, reused across epochs)."""
        cd, ca, cu = self._caps
        out = into if into is not None else BatchesOut.alloc(self._T, cd, ca, cu)
        T = self._T
        if (len(out.action) != T or any(len(getattr(out, f)) != T + 1 for f in ("del_off", "add_off", "upd_off"))
                or len(out.del_res) < len(out.del_idx) or len(out.add_res) < len(out.add_idx)
                or len(out.upd_res) < len(out.upd_idx) or len(out.add_qdisc) < len(out.add_idx)
                or len(out.upd_qdisc) < len(out.upd_idx)):
            # kdtn_epoch_download writes T action bytes and T+1 offsets per list unchecked
            raise ValueError(f"download(into=...): buffers sized for {len(out.action)} topologies, "
                             f"the epoch has {T}")
        b = out.to_c((len(out.del_idx), len(out.add_idx), len(out.upd_idx)))
        _check(lib().kdtn_epoch_download(self._ctx, C.byref(b)), "kdtn_epoch_download")
        return out.trim(b.n_del, b.n_add, b.n_upd)

    def download_async(self, into: BatchesOut) -> BatchesOut:
        """kdtn_epoch_download_async into page-locked `into` (BatchesOut.alloc(pinned=True)):
        returns the trimmed view at once; its arrays hold the outputs after download_wait()."""
        T = self._T
        if len(into.action) != T or len(into.del_off) != T + 1:
            raise ValueError(f"download_async(into=...): buffers sized for {len(into.action)} topologies, "
                             f"the epoch has {T}")
        b = into.to_c((len(into.del_idx), len(into.add_idx), len(into.upd_idx)))
        self._dl_keep = b
        _check(lib().kdtn_epoch_download_async(self._ctx, C.byref(b)), "kdtn_epoch_download_async")
        return into.trim(b.n_del, b.n_add, b.n_upd)

    def download_wait(self) -> None:
        _check(lib().kdtn_epoch_download_wait(self._ctx), "kdtn_epoch_download_wait")

    def reconcile(self, inp: EpochInput, stages: int = abi.STAGE_ALL) -> BatchesOut:
        """Reconcile gate + CalcDiff + resolve + MakeQdiscs over every topology of `inp`."""
        self.upload(inp)
        self.run(stages)
        self.sync()
        return self.download()

    def diff(self, inp: EpochInput) -> BatchesOut:
        """Gate + CalcDiff only (kdtn_diff): index lists, no resolve / qdisc records."""
        cin = inp.to_c()
        out = BatchesOut.alloc(inp.topos.n, inp.realised.n, inp.desired.n, inp.realised.n)
        b = out.to_c((max(inp.realised.n, 1), max(inp.desired.n, 1), max(inp.realised.n, 1)))
        _check(lib().kdtn_diff(self._ctx, C.byref(cin), C.byref(b)), "kdtn_diff")
        self._T = inp.topos.n
        self._caps = (inp.realised.n, inp.desired.n, inp.realised.n)
        return out.trim(b.n_del, b.n_add, b.n_upd)

    # ---- daemon side: one LinksBatchQuery ------------------------------------------------
    def resolve(self, kdict: StrTab, pdict: StrTab, pods: Topos, local: int, links, kind: int,
                vnis=None):
        """Pure prefix of AddLinks (kind=BATCH_ADD) / DelLinks (BATCH_DEL) for the links of
        pods[local] (kdtn_resolve): (resolved records, qdisc records or None)."""
        pt = abi.PodTable(pods.n, abi.ptr(np.ascontiguousarray(pods.ns, np.uint32), abi.u32p),
                          abi.ptr(np.ascontiguousarray(pods.name, np.uint32), abi.u32p),
                          abi.ptr(np.ascontiguousarray(pods.src_ip, np.uint32), abi.u32p),
                          abi.ptr(np.ascontiguousarray(pods.net_ns, np.uint32), abi.u32p),
                          abi.ptr(np.ascontiguousarray(pods.flags, np.uint8), abi.u8p))
        lt = links.to_c()
        n = links.n
        res = np.zeros(max(n, 1), abi.RESOLVED_DTYPE)
        q = np.zeros(max(n, 1), abi.QDISC_DTYPE) if kind == abi.BATCH_ADD else None
        kd, pd = kdict.to_c(), pdict.to_c()
        vt = vnis.to_c() if vnis is not None else abi.VniTable(0, None, None, None)
        _check(lib().kdtn_resolve(self._ctx, C.byref(kd), C.byref(pd), C.byref(pt), local, C.byref(lt), kind,
                                  C.byref(vt), res.ctypes.data, q.ctypes.data if q is not None else None),
               "kdtn_resolve")
        self._T = 0          # the context's epoch state now belongs to this call
        return res[:n], (q[:n] if q is not None else None)

    # ---- wire encoding of the batches (proto/v1 LinksBatchQuery) ------------------------
    def encode(self) -> int:
        """Encode every batch of the last epoch on the GPU (after run + sync); returns the
        arena size in bytes."""
        n = C.c_uint64()
        _check(lib().kdtn_epoch_encode(self._ctx, C.byref(n)), "kdtn_epoch_encode")
        return int(n.value)

    def download_wire(self):
        """(arena uint8, off uint64[3T+1], err uint32[T]) of the last kdtn_epoch_encode."""
        w = abi.Wire()
        _check(lib().kdtn_epoch_download_wire(self._ctx, C.byref(w)), "kdtn_epoch_download_wire")
        n = int(w.n_bytes)
        arena = np.zeros(max(n, 1), np.uint8)
        off = np.zeros(3 * self._T + 1, np.uint64)
        err = np.zeros(max(self._T, 1), np.uint32)
        w.bytes, w.cap, w.off, w.err = arena.ctypes.data, arena.size, off.ctypes.data, err.ctypes.data
        _check(lib().kdtn_epoch_download_wire(self._ctx, C.byref(w)), "kdtn_epoch_download_wire")
        return arena[:n], off, err[:self._T]

    def tc_argv(self, n_add: int, n_upd: int):
        """SetVethQdiscs' `tc ... tbf` argv of the last epoch's reached entries: (arena uint8
        of NUL-terminated arguments, off uint64[2*n_add + n_upd + 1]); add entry e owns
        command slots 2e (LocalIntf) and 2e+1 (PeerIntf of a same-node veth pair), update
        entry u slot 2*n_add + u."""
        n = C.c_uint64()
        _check(lib().kdtn_epoch_tc(self._ctx, C.byref(n)), "kdtn_epoch_tc")
        arena = np.zeros(max(int(n.value), 1), np.uint8)
        off = np.zeros(2 * n_add + n_upd + 1, np.uint64)
        t = abi.TcArgv(arena.ctypes.data, arena.size, off.ctypes.data, 0)
        _check(lib().kdtn_epoch_download_tc(self._ctx, C.byref(t)), "kdtn_epoch_download_tc")
        return arena[:int(n.value)], off

    def fanout(self):
        """RemotePod RPCs of the last epoch grouped per destination daemon:
        (node kdict ids, off[n_nodes+1], add-entry indices)."""
        f = abi.Fanout()
        rc = lib().kdtn_epoch_fanout(self._ctx, C.byref(f))          # sizes (no buffers yet)
        if rc not in (abi.OK, abi.ENOSPC):
            _check(rc, "kdtn_epoch_fanout")
        node = np.zeros(max(f.n_nodes, 1), np.uint32)
        off = np.zeros(f.n_nodes + 1, np.uint32)
        idx = np.zeros(max(f.n_send, 1), np.uint32)
        f.node, f.off, f.idx = node.ctypes.data, off.ctypes.data, idx.ctypes.data
        f.node_cap, f.idx_cap = node.size, idx.size
        _check(lib().kdtn_epoch_fanout(self._ctx, C.byref(f)), "kdtn_epoch_fanout")
        return node[:f.n_nodes], off, idx[:f.n_send]

    def remote_encode(self) -> abi.RemoteInfo:
        """kdtn_epoch_remote_encode: marshal the epoch's RemotePod messages on the GPU."""
        info = abi.RemoteInfo()
        _check(lib().kdtn_epoch_remote_encode(self._ctx, C.byref(info)), "kdtn_epoch_remote_encode")
        return info

    def remote_pods(self):
        """RemotePod messages of the last epoch: (arena uint8, off uint64[n+1], entry uint32[n],
        n_remote, tc arena uint8, tc_off uint64[n+1]); messages [0, n_remote) follow the
        fan-out order (fanout()), the rest are the physical peers' local Updates."""
        info = self.remote_encode()
        n = info.n_msgs
        arena, tca = np.zeros(max(info.n_bytes, 1), np.uint8), np.zeros(max(info.n_tc_bytes, 1), np.uint8)
        off, tc_off = np.zeros(n + 1, np.uint64), np.zeros(n + 1, np.uint64)
        entry = np.zeros(max(n, 1), np.uint32)
        o = abi.RemotePods(arena.ctypes.data, arena.size, off.ctypes.data, entry.ctypes.data, tca.ctypes.data,
                           tca.size, tc_off.ctypes.data, n)
        _check(lib().kdtn_epoch_download_remote(self._ctx, C.byref(o)), "kdtn_epoch_download_remote")
        return arena[:info.n_bytes], off, entry[:n], int(info.n_remote), tca[:info.n_tc_bytes], tc_off

    def vni_apply(self) -> Vnis:
        """kdtn_epoch_vni_apply: the daemons' VxlanManager maps after the last epoch's reached
        entries; the result also becomes the engine's resident map (Vnis.keep_resident())."""
        _check(lib().kdtn_epoch_vni_apply(self._ctx, None), "kdtn_epoch_vni_apply")
        return self.vni_download()

    def vni_contested(self):
        """kdtn_vni_contested: (node, vni) keys of the last vni_apply whose result depends on the
        reference's goroutine order, in the order of each key's winning store."""
        n = C.c_uint32()
        _check(lib().kdtn_vni_contested(self._ctx, None, None, 0, C.byref(n)), "kdtn_vni_contested")
        node = np.zeros(max(n.value, 1), np.uint32)
        vni = np.zeros(max(n.value, 1), np.int32)
        _check(lib().kdtn_vni_contested(self._ctx, node.ctypes.data, vni.ctypes.data, node.size, C.byref(n)),
               "kdtn_vni_contested")
        return node[:n.value], vni[:n.value]

    def vni_ops_export(self):
        """This rank's VxlanManager ops of the last run (kdtn_vni_ops_export): (dels, adds) as
        abi.VNI_OP_DTYPE arrays — the host transport's contribution to a sharded apply."""
        nd, na = C.c_uint32(), C.c_uint32()
        _check(lib().kdtn_vni_ops_export(self._ctx, None, 0, None, 0, C.byref(nd), C.byref(na)), "kdtn_vni_ops_export")
        dels = np.zeros(max(nd.value, 1), abi.VNI_OP_DTYPE)
        adds = np.zeros(max(na.value, 1), abi.VNI_OP_DTYPE)
        _check(lib().kdtn_vni_ops_export(self._ctx, dels.ctypes.data, dels.size, adds.ctypes.data, adds.size,
                                         C.byref(nd), C.byref(na)), "kdtn_vni_ops_export")
        return dels[:nd.value], adds[:na.value]

    def vni_ops_import(self, dels: np.ndarray, adds: np.ndarray) -> None:
        """Every rank's ops concatenated in rank order (kdtn_vni_ops_import)."""
        dels = np.ascontiguousarray(dels, abi.VNI_OP_DTYPE)
        adds = np.ascontiguousarray(adds, abi.VNI_OP_DTYPE)
        _check(lib().kdtn_vni_ops_import(self._ctx, dels.ctypes.data if len(dels) else None, len(dels),
                                         adds.ctypes.data if len(adds) else None, len(adds)), "kdtn_vni_ops_import")

    def vni_download(self) -> Vnis:
        """kdtn_vni_download: the engine's resident VXLAN map."""
        st = abi.VniState(0, 0, None, None, None)
        _check(lib().kdtn_vni_download(self._ctx, C.byref(st)), "kdtn_vni_download")
        n = st.n
        node, vni, ns = np.zeros(max(n, 1), np.uint32), np.zeros(max(n, 1), np.int32), np.zeros(max(n, 1), np.uint32)
        st = abi.VniState(max(n, 1), 0, abi.ptr(node, abi.u32p), abi.ptr(vni, abi.i32p), abi.ptr(ns, abi.u32p))
        _check(lib().kdtn_vni_download(self._ctx, C.byref(st)), "kdtn_vni_download")
        return Vnis(node[:n], vni[:n], ns[:n])

    def set_timing(self, level: int) -> None:
        """HIP-event timing of kdtn_epoch_run: 0 none, 1 k_reconcile (+ placement), 2 every stage."""
        _check(lib().kdtn_set_timing(self._ctx, level), "kdtn_set_timing")

    def kernel_times(self) -> dict[str, float]:
        names = (C.c_char_p * 32)()
        ms = (C.c_float * 32)()
        n = lib().kdtn_last_kernel_times(self._ctx, names, ms, 32)
        out: dict[str, float] = {}
        for i in range(max(n, 0)):               # a stage timed in several pieces is summed
            k = names[i].decode()
            out[k] = out.get(k, 0.0) + float(ms[i])
        return out

    def timer_totals(self, reset: bool = False) -> dict[str, tuple[float, int]]:
        """kdtn_timer_totals: {stage: (ms summed over the epochs synced since the last reset,
        epochs that marked it)}; reset=True clears the totals after reading."""
        names = (C.c_char_p * 32)()
        ms = (C.c_double * 32)()
        ep = (C.c_uint32 * 32)()
        n = lib().kdtn_timer_totals(self._ctx, names, ms, ep, 32, 1 if reset else 0)
        return {names[i].decode(): (float(ms[i]), int(ep[i])) for i in range(max(n, 0))}

    def wg_trace(self) -> np.ndarray:
        """(nwg, 8) uint64 phase timestamps of the last traced run (KDTN_VARIANT bit 16)."""
        cap = 1 << 26
        buf = np.zeros(cap, np.uint64)
        n = lib().kdtn_debug_wg_trace(self._ctx, buf.ctypes.data_as(C.POINTER(C.c_uint64)), cap)
        if n < 0:
            raise KdtnError(n, "kdtn_debug_wg_trace")
        return buf[:n].reshape(-1, 8)

    # ---- MakeQdiscs batch --------------------------------------------------------------
    def make_qdiscs(self, pdict: StrTab, prop: np.ndarray, gap: np.ndarray) -> np.ndarray:
        """common.MakeQdiscs for n property sets: prop (NPROP, n) pdict ids, gap (n,)."""
        prop = np.ascontiguousarray(prop, dtype=np.uint32)
        gap = np.ascontiguousarray(gap, dtype=np.uint32)
        n = int(gap.shape[0])
        t = abi.PropsTable()
        t.n = n
        for k in range(abi.NPROP):
            t.prop[k] = abi.ptr(prop[k], abi.u32p)
        t.gap = abi.ptr(gap, abi.u32p)
        out = np.zeros(max(n, 1), abi.QDISC_DTYPE)
        cp = pdict.to_c()
        _check(lib().kdtn_make_qdiscs(self._ctx, C.byref(cp), C.byref(t), out.ctypes.data),
               "kdtn_make_qdiscs")
        return out[:n]
