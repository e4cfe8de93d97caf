"""ctypes mirror of include/kdtn.h (the C-ABI of libkdtn.so).

Pure data declarations: struct layouts, enums and numpy dtypes of the output records.
Shared by the product binding (kdtn.engine) and by the test oracle wrapper.
"""
from __future__ import annotations

import ctypes as C

import numpy as np

ABI_VERSION = 1

OK, EINVAL, ENOMEM, EIO, ENOSPC, ENODEV = 0, -22, -12, -5, -28, -19

# kdtn_err (first failing step, reference order)
E_NONE, E_VETH_CIDR, E_VETH_MAC = 0, 1, 2
E_LATENCY, E_LATENCY_CORR, E_JITTER, E_LOSS, E_LOSS_CORR = 3, 4, 5, 6, 7
E_DUPLICATE, E_DUPLICATE_CORR, E_REORDER_PROB, E_REORDER_CORR = 8, 9, 10, 11
E_CORRUPT_PROB, E_CORRUPT_CORR, E_RATE = 12, 13, 14
E_PEER_LOOKUP, E_PEER_NO_LINKS, E_PEER_VETH_CIDR, E_PEER_VETH_MAC = 15, 16, 17, 18
E_REMOTE_CIDR = 19
ERR_NAMES = ["none", "veth_cidr", "veth_mac", "latency", "latency_corr", "jitter", "loss",
             "loss_corr", "duplicate", "duplicate_corr", "reorder_prob", "reorder_corr",
             "corrupt_prob", "corrupt_corr", "rate", "peer_lookup", "peer_no_links",
             "peer_veth_cidr", "peer_veth_mac", "remote_cidr"]

ACT_SKIP, ACT_CREATED, ACT_DIFF = 0, 1, 2
KIND_NONE, KIND_MACVLAN, KIND_PHYSICAL, KIND_PEER_DEAD, KIND_SAME_NODE, KIND_CROSS_NODE = range(6)

# key columns (api/v1/topology_types.go:59-95)
KEY_COLS = ["local_intf", "local_ip", "local_mac", "peer_intf", "peer_ip", "peer_mac", "peer_pod"]
# property string columns (api/v1/topology_types.go:119-176), Gap separate
PROP_COLS = ["latency", "latency_corr", "jitter", "loss", "loss_corr", "rate", "duplicate",
             "duplicate_corr", "reorder_prob", "reorder_corr", "corrupt_prob", "corrupt_corr"]
NKEY, NPROP = len(KEY_COLS), len(PROP_COLS)

TOPO_STATUS_NIL, TOPO_SPEC_NIL = 0x1, 0x2
STAGE_DIFF, STAGE_RESOLVE, STAGE_QDISC, STAGE_ALL = 0x1, 0x2, 0x4, 0x7

u8p = C.POINTER(C.c_uint8)
u32p = C.POINTER(C.c_uint32)
u64p = C.POINTER(C.c_uint64)
i32p = C.POINTER(C.c_int32)
i64p = C.POINTER(C.c_int64)


class Strtab(C.Structure):
    _fields_ = [("bytes", u8p), ("offs", u32p), ("n", C.c_uint32)]


class LinkTable(C.Structure):
    _fields_ = [("n", C.c_uint32), ("key", u32p * NKEY), ("uid", i64p),
                ("prop", u32p * NPROP), ("gap", u32p)]


class TopoTable(C.Structure):
    _fields_ = [("n", C.c_uint32), ("ns", u32p), ("name", u32p), ("src_ip", u32p),
                ("net_ns", u32p), ("flags", u8p), ("real_off", u32p), ("des_off", u32p)]


class VniTable(C.Structure):
    _fields_ = [("n", C.c_uint32), ("node", u32p), ("vni", i32p), ("net_ns", u32p)]


VNI_RESIDENT = 0xFFFFFFFF   # kdtn_epoch_in.vnis.n: use the context's resident VXLAN map


class VniState(C.Structure):
    _fields_ = [("cap", C.c_uint64), ("n", C.c_uint32), ("node", u32p), ("vni", i32p), ("net_ns", u32p)]


class EpochIn(C.Structure):
    _fields_ = [("kdict", Strtab), ("pdict", Strtab), ("topos", TopoTable),
                ("realised", LinkTable), ("desired", LinkTable), ("vnis", VniTable),
                ("pod_slice", C.c_uint32), ("kdict_keep", C.c_uint32), ("pdict_keep", C.c_uint32)]


DELTA_NEW = 0x80000000     # kdtn_epoch_delta.ref: inline record k of the delta


class EpochDelta(C.Structure):
    _fields_ = [("kdict", Strtab), ("pdict", Strtab), ("kdict_keep", C.c_uint32), ("pdict_keep", C.c_uint32),
                ("n_changed", C.c_uint32), ("topo", u32p), ("src_ip", u32p), ("net_ns", u32p), ("spec_nil", u8p),
                ("des_off", u32p), ("ref", u32p), ("records", LinkTable), ("vnis", VniTable),
                ("n_topos", C.c_uint32), ("prev", u32p), ("ns", u32p), ("name", u32p), ("pod_slice", C.c_uint32)]


class PropsTable(C.Structure):
    _fields_ = [("n", C.c_uint32), ("prop", u32p * NPROP), ("gap", u32p)]


class Qdisc(C.Structure):
    _fields_ = [("latency", C.c_uint32), ("delay_corr", C.c_uint32), ("limit", C.c_uint32),
                ("loss", C.c_uint32), ("loss_corr", C.c_uint32), ("gap", C.c_uint32),
                ("duplicate", C.c_uint32), ("duplicate_corr", C.c_uint32),
                ("jitter", C.c_uint32), ("reorder_prob", C.c_uint32),
                ("reorder_corr", C.c_uint32), ("corrupt_prob", C.c_uint32),
                ("corrupt_corr", C.c_uint32), ("tbf_buffer", C.c_uint32),
                ("tbf_rate", C.c_uint64), ("tbf_minburst", C.c_uint32),
                ("has_netem", C.c_uint8), ("has_tbf", C.c_uint8), ("err", C.c_uint8),
                ("reserved", C.c_uint8)]


class Resolved(C.Structure):
    _fields_ = [("peer_topo", C.c_uint32), ("vni", C.c_int32), ("vtep", C.c_uint32),
                ("kind", C.c_uint8), ("err", C.c_uint8), ("vni_hit", C.c_uint8),
                ("remote_err", C.c_uint8)]


class Batches(C.Structure):
    _fields_ = [("action", u8p), ("del_off", u32p), ("add_off", u32p), ("upd_off", u32p),
                ("del_idx", u32p), ("add_idx", u32p), ("upd_idx", u32p),
                ("del_res", C.c_void_p), ("add_res", C.c_void_p), ("upd_res", C.c_void_p),
                ("add_qdisc", C.c_void_p), ("upd_qdisc", C.c_void_p),
                ("del_cap", C.c_uint32), ("add_cap", C.c_uint32), ("upd_cap", C.c_uint32),
                ("n_del", C.c_uint32), ("n_add", C.c_uint32), ("n_upd", C.c_uint32)]


class Counts(C.Structure):
    _fields_ = [("n_del", C.c_uint32), ("n_add", C.c_uint32), ("n_upd", C.c_uint32),
                ("n_topos", C.c_uint32)]


class Wire(C.Structure):
    _fields_ = [("bytes", C.c_void_p), ("cap", C.c_uint64), ("off", C.c_void_p), ("err", C.c_void_p),
                ("n_bytes", C.c_uint64)]


class Fanout(C.Structure):
    _fields_ = [("node", C.c_void_p), ("off", C.c_void_p), ("idx", C.c_void_p), ("node_cap", C.c_uint32),
                ("idx_cap", C.c_uint32), ("n_nodes", C.c_uint32), ("n_send", C.c_uint32)]


class TcArgv(C.Structure):
    _fields_ = [("bytes", C.c_void_p), ("cap", C.c_uint64), ("off", C.c_void_p), ("n_bytes", C.c_uint64)]


class RemoteInfo(C.Structure):
    _fields_ = [("n_msgs", C.c_uint32), ("n_remote", C.c_uint32), ("n_bytes", C.c_uint64),
                ("n_tc_bytes", C.c_uint64)]


class RemotePods(C.Structure):
    _fields_ = [("bytes", C.c_void_p), ("cap", C.c_uint64), ("off", C.c_void_p), ("entry", C.c_void_p),
                ("tc_bytes", C.c_void_p), ("tc_cap", C.c_uint64), ("tc_off", C.c_void_p), ("msg_cap", C.c_uint32)]


class PodTable(C.Structure):
    _fields_ = [("n", C.c_uint32), ("ns", u32p), ("name", u32p), ("src_ip", u32p), ("net_ns", u32p),
                ("flags", u8p)]


BATCH_ADD, BATCH_DEL = 0, 1


class IngestInfo(C.Structure):
    _fields_ = [("n_topos", C.c_uint32), ("n_desired", C.c_uint32), ("n_realised", C.c_uint32),
                ("n_kdict", C.c_uint32), ("n_pdict", C.c_uint32), ("json_err", C.c_int32),
                ("err_offset", C.c_uint64), ("n_tokens", C.c_uint64), ("kdict_bytes", C.c_uint64),
                ("pdict_bytes", C.c_uint64)]


class IngestTables(C.Structure):
    _fields_ = [(f, C.c_void_p) for f in (
        "kd_bytes", "kd_offs", "pd_bytes", "pd_offs", "ns", "name", "src_ip", "net_ns", "flags",
        "real_off", "des_off", "des_key", "des_prop", "des_gap", "des_uid",
        "real_key", "real_prop", "real_gap", "real_uid")]


EBADMSG = -74
JSON_OK, JSON_SYNTAX, JSON_DEPTH, JSON_TYPE, JSON_DUPKEY = 0, 1, 2, 3, 4


class Config(C.Structure):
    _fields_ = [("device", C.c_int32), ("vxlan_base", C.c_int32), ("tick_in_usec", C.c_double)]


assert C.sizeof(Qdisc) == 72, C.sizeof(Qdisc)
assert C.sizeof(Resolved) == 16

QDISC_DTYPE = np.dtype([(n, np.uint64 if n == "tbf_rate" else (np.uint8 if n in (
    "has_netem", "has_tbf", "err", "reserved") else np.uint32)) for n, _ in Qdisc._fields_],
    align=True)
RESOLVED_DTYPE = np.dtype([("peer_topo", np.uint32), ("vni", np.int32), ("vtep", np.uint32),
                           ("kind", np.uint8), ("err", np.uint8), ("vni_hit", np.uint8),
                           ("remote_err", np.uint8)], align=True)
assert QDISC_DTYPE.itemsize == 72 and RESOLVED_DTYPE.itemsize == 16
VNI_OP_DTYPE = np.dtype([("node", np.uint32), ("vni", np.int32), ("net_ns", np.uint32), ("kind", np.uint32)])

# symbols include/kdtn.h declares (checked by the CPU test suite)
EXPORTS = ["kdtn_version", "kdtn_strerror", "kdtn_err_name", "kdtn_init", "kdtn_destroy",
           "kdtn_set_stream", "kdtn_psched_tick_in_usec", "kdtn_interner_new",
           "kdtn_interner_free", "kdtn_intern", "kdtn_intern_batch", "kdtn_interner_table",
           "kdtn_reconcile_epoch", "kdtn_epoch_upload", "kdtn_epoch_run", "kdtn_epoch_sync",
           "kdtn_epoch_download", "kdtn_make_qdiscs", "kdtn_comm_unique_id", "kdtn_comm_init",
           "kdtn_set_timing", "kdtn_epoch_vni_apply", "kdtn_vni_contested", "kdtn_vni_download", "kdtn_last_kernel_times", "kdtn_timer_totals", "kdtn_debug_wg_trace", "kdtn_epoch_encode",
           "kdtn_epoch_download_wire", "kdtn_diff", "kdtn_resolve", "kdtn_host_alloc",
           "kdtn_host_free", "kdtn_epoch_fanout", "kdtn_epoch_tc", "kdtn_epoch_download_tc",
           "kdtn_json_upload", "kdtn_json_ingest", "kdtn_ingest_download", "kdtn_topology_shard",
           "kdtn_comm_set_ranks", "kdtn_pods_export", "kdtn_pods_import", "kdtn_json_ingest_shard",
           "kdtn_ingest_shard_topos", "kdtn_epoch_remote_encode", "kdtn_epoch_download_remote",
           "kdtn_epoch_commit", "kdtn_epoch_upload_delta", "kdtn_epoch_tables_info",
           "kdtn_vni_ops_export", "kdtn_vni_ops_import", "kdtn_json_ingest_delta",
           "kdtn_epoch_download_async", "kdtn_epoch_download_wait", "kdtn_epoch_late_pods"]


def ptr(a: np.ndarray, t):
    """ctypes pointer to a contiguous numpy array (caller keeps `a` alive)."""
    assert a.flags["C_CONTIGUOUS"], "array must be contiguous"
    return a.ctypes.data_as(t)
