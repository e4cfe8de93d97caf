"""kdtn — MI355X batch topology-reconcile engine for kube-dtn (host layer over libkdtn.so).

The hot path (Reconcile gate + CalcDiff + addLink/delLink/UpdateLinks pure prefix +
MakeQdiscs) runs as HIP kernels on gfx950 behind the C-ABI in include/kdtn.h; this
package packs tables, calls the ABI and unpacks the batches.
"""
from . import abi
from .engine import Engine, KdtnError, comm_unique_id, lib, topology_shard
from .tables import BatchesOut, EpochInput, Interner, Links, StrTab, Topos, Vnis

__all__ = ["abi", "Engine", "KdtnError", "comm_unique_id", "lib", "BatchesOut", "EpochInput",
           "Interner", "Links", "StrTab", "Topos", "Vnis"]
