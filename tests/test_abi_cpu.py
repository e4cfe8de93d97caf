"""CPU: the C-ABI library loads and exports exactly what include/kdtn.h declares.

No compute calls here (no GPU in the build container); kdtn_init must fail cleanly."""
import ctypes as C
import os
import re

from conftest import ROOT
from kdtn import abi, engine


def header_functions():
    src = open(os.path.join(ROOT, "include", "kdtn.h")).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(kdtn_[a-z_0-9]+)\s*\(", src)))


def test_header_matches_binding_list():
    assert header_functions() == sorted(abi.EXPORTS)


def test_library_exports_every_declared_symbol():
    L = engine.lib()
    for name in header_functions():
        assert hasattr(L, name), name
    assert L.kdtn_version().decode().startswith("kdtn-mi355x")


def test_struct_layouts():
    assert C.sizeof(abi.Qdisc) == 72
    assert C.sizeof(abi.Resolved) == 16
    assert abi.Qdisc.tbf_rate.offset == 56 and abi.Qdisc.err.offset == 70
    assert C.sizeof(abi.Strtab) == 24


def test_host_interner_dedups_and_reserves_empty_id():
    L = engine.lib()
    it = C.c_void_p()
    assert L.kdtn_interner_new(C.byref(it)) == 0
    try:
        a = L.kdtn_intern(it, b"eth0", 4)
        b = L.kdtn_intern(it, b"eth1", 4)
        assert L.kdtn_intern(it, b"eth0", 4) == a and a != b
        assert L.kdtn_intern(it, b"", 0) == 0
        t = abi.Strtab()
        assert L.kdtn_interner_table(it, C.byref(t)) == 0
        assert t.n == 3 and t.offs[0] == 0 and t.offs[1] == 0 and t.offs[3] == 8
    finally:
        L.kdtn_interner_free(it)


def test_init_without_gpu_fails_loudly():
    import torch
    if torch.cuda.is_available():
        return
    cfg = abi.Config(0, 5000, 15.625)
    ctx = C.c_void_p()
    rc = engine.lib().kdtn_init(C.byref(ctx), C.byref(cfg))
    assert rc == abi.ENODEV and not ctx.value


def test_error_names():
    L = engine.lib()
    assert [L.kdtn_err_name(i).decode() for i in range(len(abi.ERR_NAMES))] == abi.ERR_NAMES
    assert abs(L.kdtn_psched_tick_in_usec() - 15.625) < 1e-12 or L.kdtn_psched_tick_in_usec() >= 0


def test_product_library_reads_no_environment():
    """The product library compiles only the parity-tested kernel paths: no A/B switch
    (KDTN_VARIANT / KDTN_KD_SUB / KDTN_JS_VARIANT) is read from the environment, and only
    the default k_reconcile instantiation is present (the variants live in the profiling
    build, kube-dtn_amd/prof/libkdtn_prof.so)."""
    data = open(engine.LIB_PATH, "rb").read()
    for knob in (b"KDTN_VARIANT", b"KDTN_KD_SUB", b"KDTN_JS_VARIANT", b"KDTN_SPLIT", b"KDTN_PD_SPLIT",
                 b"KDTN_PD_ONLY"):
        assert knob not in data, knob
    names = set(re.findall(rb"_ZN4kdtn11k_reconcileILi(\d+)E", data))
    assert names == {b"16899", b"2116099"}, names   # default and comparison-heavy builds
