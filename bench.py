#!/usr/bin/env python3
"""bench.py — links reconciled/sec of the MI355X reconcile engine (BASELINE.json metric).

One step = one reconcile epoch over this rank's shard, inputs resident in HBM:
  dictionary parse → pod-status table (+ RCCL all-gather across ranks) → lookup tables →
  Reconcile gate + CalcDiff → batch compaction → addLink/delLink/UpdateLinks pure prefix
  → MakeQdiscs; the host waits for each epoch (kdtn_epoch_sync).

Workloads; topologies are sharded across ranks as the engine shards them,
hash64(namespace/name) mod N (kdtn_topology_shard), one process per GPU:
  --config 2 (default, BASELINE configs[2], the metric's 10M-link topology): a 1M-pod random
      10-regular topology, 10M Link records with heterogeneous netem/tbf props, all AddLinks
      (realised status non-nil and empty). Strong scaling by default: the same 10M links are
      split over N GPUs; --scaling weak gives every GPU --pods pods instead.
  --config 3 (churn): the same topology as an epoch sequence; each epoch realised := the
      previous desired and 5 % of the edges churn (1/60 deleted, 1/60 new props, 1/60 new);
      --warmup epochs, then the mean over --steps epochs (default 10). Uploads happen between
      the timed epochs; the dictionaries are append-only (kdict_keep / pdict_keep), so each
      epoch parses only its new strings.
  --config 4 (WAN twin): 100k sites in namespaces of 100, power-law degrees, 256 nodes.

  --config 1 (fat-tree): 10k pods, 100k links, uniform props; realised = the same keys with
      empty props, so every record is an UpdateLinks entry (MakeQdiscs-dominated). 1 GPU.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--config C] [--scaling strong|weak]
One process per GPU. `--gpus N` (N > 1) run without a launcher spawns the N ranks itself:
the parent starts `torch.distributed.run --nproc-per-node N` as a child process before it
touches the GPU and exits with the child's status; under an external launcher (WORLD_SIZE
set) WORLD_SIZE must equal --gpus.
"""
from __future__ import annotations

import argparse
import json
import math
import os
import sys
import time

import torch  # noqa: E402  (first: one HIP runtime per process, see kdtn/engine.py)
import torch.distributed as dist

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "kube-dtn_amd"))

import numpy as np  # noqa: E402

from kdtn import Engine, KdtnError, abi, comm_unique_id, synth  # noqa: E402

HBM_PEAK_GBS = 8000.0   # MI355X HBM3E spec peak (MI355X_MICROARCH.md, chip-level parameters)
DEFAULT_PODS = {1: 10_000, 2: 1_000_000, 3: 1_000_000, 4: 100_000}
WORKLOAD = {
    1: "config1: fat-tree of {pods} pods (1000 spines + 9000 leaves, {links} Link records), uniform "
       "props {{latency 10ms, loss 0.1, rate 1Gbit}} over a realised side with the same keys and empty "
       "props: every record is an UpdateLinks entry (MakeQdiscs on every link)",
    2: "config2: random 10-regular topology of {pods} pods ({links} Link records), heterogeneous "
       "netem/tbf props, all AddLinks (resolve + qdisc on every link)",
    3: "config3: churn epochs on a random 10-regular topology of {pods} pods (~{links} Link records): "
       "per epoch 5% of the edges churn (1/60 deleted, 1/60 re-drawn props, 1/60 added), diff-dominated; "
       "mean of {steps} epochs",
    4: "config4: WAN twin of {pods} sites in namespaces of 100 (power-law degrees, 256 nodes, 1% "
       "physical/ and 0.5% localhost peers), {links} Link records, all AddLinks (resolve-dominated)",
}


def reconcile_bytes(inp, n_add: int, n_upd: int, n_del: int) -> float:
    """Algorithmic bytes of one k_reconcile launch: per AddLinks entry
    1 (flag) + 16 (local_ip, local_mac, peer_pod, peer_ip ids) + 8 (uid) + 48 (12 prop ids)
    + 4 (gap) read, 4 (index) + 16 (resolve record) + 72 (qdisc) written = 169 B; per
    topology 8 (offsets) + 1 (action) + 12 (ns, src_ip, net_ns) read + 12 (3 batch offsets)
    written = 33 B; plus the 24 B parsed record of every property string, read once; when
    realised lists are non-empty, 88 B per record of both sides (read once to compare)."""
    T = inp.topos.n
    per_add = 1 + 16 + 8 + 48 + 4 + 4 + 16 + 72
    per_upd = 1 + 4 + 12 + 48 + 4 + 8 + 4 + 16 + 72   # flag, target, ids, props, gap, uid, out
    per_del = 1 + 12 + 8 + 4 + 16
    cmp = 88.0 * (inp.realised.n + (inp.desired.n if inp.realised.n else 0))
    return (per_add * n_add + per_upd * n_upd + per_del * n_del + 33.0 * T + 24.0 * inp.pdict.n
            + cmp)


def reconcile_ms(kt: dict) -> float:
    """k_reconcile's time, plus the placement kernels of the comparison build."""
    return kt["reconcile"] + kt.get("place_scan", 0.0) + kt.get("place", 0.0)


def epoch_bytes(inp, n_add: int, n_upd: int, n_del: int) -> float:
    """SURVEY §8(d) whole-epoch model: 92·M + 92·N + 16·T + 4·lists + 36·|add| + 72·|add∪upd|
    + unique property-string bytes."""
    M, N, T = inp.realised.n, inp.desired.n, inp.topos.n
    return (92.0 * (M + N) + 16.0 * T + 4.0 * (n_add + n_upd + n_del) + 36.0 * n_add
            + 72.0 * (n_add + n_upd) + float(inp.pdict.offs[-1]))


def cpu_share():
    """CPUs this process may use: the affinity mask, capped by a cgroup v2 cpu.max quota."""
    aff = len(os.sched_getaffinity(0))
    quota = None
    try:
        q, p = open("/sys/fs/cgroup/cpu.max").read().split()
        if q != "max":
            quota = int(q) / int(p)
    except (OSError, ValueError):
        pass
    share = aff if quota is None else max(1, min(aff, int(math.ceil(quota))))
    return share, {"nproc": os.cpu_count(), "affinity": aff, "cgroup_quota_cpus": quota,
                   "omp_num_threads": os.environ.get("OMP_NUM_THREADS"), "cpu_model": cpu_model()}


def cpu_model() -> dict:
    """The host CPU as lscpu reports it (model, sockets, cores), /proc/cpuinfo
    when lscpu is absent."""
    import subprocess
    out = {}
    try:
        txt = subprocess.run(["lscpu"], capture_output=True, text=True, timeout=10).stdout
        for line in txt.splitlines():
            k, _, v = line.partition(":")
            if k.strip() in ("Model name", "Socket(s)", "Core(s) per socket", "Thread(s) per core", "CPU(s)",
                             "CPU max MHz", "L3 cache", "NUMA node(s)"):
                out[k.strip()] = v.strip()
    except (OSError, subprocess.SubprocessError):
        pass
    if "Model name" not in out:
        try:
            for line in open("/proc/cpuinfo"):
                if line.startswith("model name"):
                    out["Model name"] = line.split(":", 1)[1].strip()
                    break
        except OSError:
            pass
    return out


def cpu_baseline(inp, budget_s: float, threads: int, share_info: dict):
    """The CPU oracle (C restatement of the reference Go path) on a bounded sample of this
    workload's topologies, loop time only (informer maps pre-built). Single thread, then
    `threads` workers over disjoint topology ranges, mirroring the reference's
    MaxConcurrentReconciles: 32 worker pool (controllers/topology_controller.go:335-337),
    capped by the CPUs this process may use; the ctypes call releases the GIL, so the
    workers run concurrently."""
    from concurrent.futures import ThreadPoolExecutor
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle as O
    T = inp.topos.n
    t_end = min(T, 20_000)
    timing = []
    O.reconcile(inp, t_begin=0, t_end=t_end, timing=timing)    # warm + calibrate
    rate = (inp.topos.des_off[t_end] - inp.topos.des_off[0]) / max(timing[-1], 1e-9)
    want = int(min(T, max(t_end, budget_s * rate / max(inp.desired.n / T, 1.0))))
    timing.clear()
    O.reconcile(inp, t_begin=0, t_end=want, timing=timing)
    links = int(inp.topos.des_off[want] - inp.topos.des_off[0])
    one = links / timing[-1]
    n_par = int(min(T, want * threads))
    bounds = [n_par * k // threads for k in range(threads + 1)]
    ptim = [[] for _ in range(threads)]
    with ThreadPoolExecutor(threads) as ex:
        list(ex.map(lambda k: O.reconcile(inp, t_begin=bounds[k], t_end=bounds[k + 1],
                                          timing=ptim[k]), range(threads)))
    par_links = int(inp.topos.des_off[n_par] - inp.topos.des_off[0])
    par_s = max(t[-1] for t in ptim)
    return {"value": par_links / par_s, "unit": "links/s", "cores": threads, "kind": "port",
            "value_1thread": one, "host": share_info,
            "sample": f"oracle/kdtn_oracle.c (literal CalcDiff loops, per-link MakeQdiscs, "
                      f"map-based resolve) on rank 0's shard: {threads} threads (min(32, CPUs this "
                      f"process may use)) over topologies [0,{n_par}) = {par_links} links in "
                      f"{par_s:.2f} s (slowest worker's loop); single thread: [0,{want}) = {links} "
                      f"links in {timing[-1]:.2f} s"}


def wire_stage(eng, reps: int = 5):
    """Separate report (not part of `value`): the output stages of an epoch, in the order a
    controller calls them after each run — kdtn_epoch_encode (proto.Marshal of every
    LinksBatchQuery Reconcile sends), kdtn_epoch_fanout (RemotePod RPCs per destination
    daemon), kdtn_epoch_remote_encode (the RemotePod bodies and the receiving daemons' tc argv).
    Every rep runs the epoch first, so each stage's time includes the per-run tables it builds
    (the encoders' string tables and the lists' coarse topology indexes are built by the first
    stage, encode, and shared by the later ones). GPU kernel time from HIP events, excluding the
    host round trips that size the arenas; bytes = serialized output. Mean over `reps` after one
    warm-up epoch."""
    acc: dict[str, float] = {}
    facc: dict[str, float] = {}
    racc: dict[str, float] = {}
    n, node, idx, info = 0, [], [], None
    for rep in range(reps + 1):
        eng.run()
        eng.sync()
        n = eng.encode()
        kt = eng.kernel_times()
        node, off, idx = eng.fanout()
        ft = eng.kernel_times()
        info = eng.remote_encode()            # the fan-out is cached per run: message kernels only
        rt = eng.kernel_times()
        if rep == 0:
            continue
        for d, src in ((acc, kt), (facc, ft), (racc, rt)):
            for k, v in src.items():
                d[k] = d.get(k, 0.0) + v / reps
    gpu_ms = sum(v for k, v in acc.items() if k != "wire_host_sync")
    res = {"bytes": n, "gpu_ms": gpu_ms, "out_GBps": n / (gpu_ms * 1e-3) / 1e9,
           "kernels_ms": acc, "note": "not part of value; per epoch after its run; arena-size host round trip excluded"}
    res["fanout"] = {"daemons": int(len(node)), "remote_rpcs": int(len(idx)),
                     "gpu_ms": sum(v for k, v in facc.items() if k != "fanout_host_sync"),
                     "kernels_ms": facc}
    rms = sum(v for k, v in racc.items() if k != "remote_host_sync")
    res["remote_pods"] = {"messages": int(info.n_msgs), "remote": int(info.n_remote), "bytes": int(info.n_bytes),
                          "tc_bytes": int(info.n_tc_bytes), "gpu_ms": rms,
                          "out_GBps": (info.n_bytes + info.n_tc_bytes) / (rms * 1e-3) / 1e9, "kernels_ms": racc,
                          "note": "RemotePod request bodies and the receiving daemons' tc argv "
                                  "(kdtn_epoch_remote_encode) after the fan-out"}
    return res


def e2e_stage(eng, inp, reps: int = 3):
    """PCIe-inclusive epoch (separate report, never `value`): kdtn_reconcile_epoch's pieces —
    upload of the host tables, run + sync, download of every output — timed separately,
    median of `reps`, from page-locked host buffers (kdtn_host_alloc: the tables and the
    output arrays), and once more from pageable numpy arrays for comparison."""
    from kdtn.engine import pin_input
    from kdtn.tables import BatchesOut

    def timed(src, into):
        ups, runs, downs = [], [], []
        out = None
        for _ in range(reps):
            t0 = time.perf_counter()
            eng.upload(src)
            t1 = time.perf_counter()
            eng.run()
            eng.sync()
            t2 = time.perf_counter()
            out = eng.download(into)
            t3 = time.perf_counter()
            ups.append(t1 - t0)
            runs.append(t2 - t1)
            downs.append(t3 - t2)
        med = lambda x: sorted(x)[len(x) // 2]
        return med(ups), med(runs), med(downs), out

    up_b = (88 * (inp.realised.n + inp.desired.n) + 25 * inp.topos.n + len(inp.kdict.bytes_)
            + 4 * inp.kdict.n + len(inp.pdict.bytes_) + 4 * inp.pdict.n)
    pin = pin_input(inp)
    into = BatchesOut.alloc(inp.topos.n, inp.realised.n, inp.desired.n, inp.realised.n, pinned=True)
    u, r, d, out = timed(pin, into)
    down_b = sum(getattr(out, f).nbytes for f in out.FIELDS)
    tot = u + r + d
    res = {"links_per_s": inp.desired.n / tot, "ms": tot * 1e3, "upload_ms": u * 1e3, "run_ms": r * 1e3,
           "download_ms": d * 1e3, "upload_bytes": up_b, "download_bytes": down_b,
           "upload_GBps": up_b / u / 1e9, "download_GBps": down_b / d / 1e9, "host_memory": "pinned (kdtn_host_alloc)",
           "note": "not part of value: full upload + epoch + download of caller-owned page-locked host memory "
                   "(one kdtn_reconcile_epoch); a resident controller uploads deltas instead (config-3 "
                   "resident_chain)"}
    del pin, into
    u, r, d, out = timed(inp, None)
    res["pageable"] = {"ms": (u + r + d) * 1e3, "upload_ms": u * 1e3, "download_ms": d * 1e3,
                       "host_link_GBps": (up_b + down_b) / (u + d) / 1e9}
    return res


def resident_chain_stage(eng, cs, prev, epochs: int, topology_set: bool = False):
    """Config 3 as a resident controller runs it (separate report, never `value`): each epoch
    uploads only a delta against the engine's state (kdtn_epoch_upload_delta: the changed
    Topologies' specs as references into the previous desired store + new records), runs,
    downloads the batches, and commits the status on the device (kdtn_epoch_commit, every
    Topology's RPCs taken as succeeded, as the churn generator assumes). Host buffers
    page-locked; the delta is built on the host outside the timed region. topology_set: `cs`
    is a synth.TopologySetChurn (1 % of the Topologies deleted / re-created per epoch) and
    `prev` was fully uploaded first."""
    from kdtn.delta import build_delta
    from kdtn.engine import pin_delta
    from kdtn.tables import BatchesOut
    T = prev.topos.n
    cap = max(1 << 20, prev.desired.n // 8)              # entries per list (5 % churn: ~1.7 %)
    into = None
    rows = []
    state_T = T
    warm = 2                                             # first deltas size the rotating buffers
    # every epoch's delta built and page-locked before the loop (as a controller's informer
    # thread would have it ready): no host allocation or release next to a timed call
    work = []
    p = prev
    for ep in range(warm + epochs):
        progress(f"  resident epoch {ep}: delta")
        cs.advance()
        new = cs.epoch_input(copy=True)
        work.append((pin_delta(build_delta(p, new, p.kdict.n, p.pdict.n)), new.topos.n, new.desired.n))
        p = new
    eng.commit(np.ones(T, np.uint8))
    for ep, (d, nT, nN) in enumerate(work):
        if into is None or len(into.action) != nT:
            into = BatchesOut.alloc(nT, cap, cap, cap, pinned=True)
        ones = np.ones(nT, np.uint8)
        t0 = time.perf_counter()
        eng.upload_delta(d)
        t1 = time.perf_counter()
        eng.run()
        c = eng.sync()
        t2 = time.perf_counter()
        out = eng.download(into)
        t3 = time.perf_counter()
        eng.commit(ones)
        t4 = time.perf_counter()
        down_b = sum(getattr(out, f).nbytes for f in out.FIELDS)
        created = int((d.prev == abi.DELTA_NEW).sum()) if d.prev is not None else 0
        deleted = state_T - (nT - created)
        state_T = nT
        if ep >= warm:
            rows.append((d.upload_bytes(), t1 - t0, t2 - t1, t3 - t2, t4 - t3, down_b, nN,
                         d.n_changed, d.records.n, c.n_add + c.n_del + c.n_upd, created, deleted))
    prev = p
    del work
    a = np.array(rows, dtype=np.float64).mean(axis=0)
    full_b = 88 * (2 * prev.desired.n) + 25 * T
    e2e = a[1] + a[2] + a[3] + a[4]
    res = {"epochs": epochs, "upload_bytes": a[0], "full_upload_bytes": full_b, "upload_frac": a[0] / full_b,
           "changed_topologies": a[7], "inline_records": a[8], "entries": a[9],
           "upload_ms": a[1] * 1e3, "upload_GBps": a[0] / a[1] / 1e9, "run_ms": a[2] * 1e3,
           "download_ms": a[3] * 1e3, "download_bytes": a[5], "download_GBps": a[5] / a[3] / 1e9,
           "commit_ms": a[4] * 1e3, "e2e_ms": e2e * 1e3, "links_per_s": a[6] / e2e,
           "note": "not part of value: per epoch delta upload + run + download + on-device status commit, "
                   f"page-locked host memory (deltas built before the loop), mean over {epochs} epochs after "
                   f"{warm} warm-up epochs"}
    if topology_set:
        res["created_topologies"], res["deleted_topologies"] = a[10], a[11]
    return res


def resident_pipeline_stage(eng, cs, prev, epochs: int):
    """The same resident controller loop pipelined over the full-duplex host link (separate
    report, never `value`): epoch k's outputs are copied out asynchronously on an SDMA engine
    (kdtn_epoch_download_async into one of two page-locked buffer sets: no CUs) while epoch
    k+1's delta is uploaded; the next run waits for the copies. Per-epoch time = wall time of
    the loop / epochs, after 2 warm-up epochs; every epoch's outputs are complete in host
    memory (download_wait) before the next-but-one reuses their buffers. `cs` may change the
    Topology set (synth.TopologySetChurn) as long as the count stays."""
    from kdtn.delta import build_delta
    from kdtn.engine import pin_delta
    from kdtn.tables import BatchesOut
    T = prev.topos.n
    cap = max(1 << 20, prev.desired.n // 8)
    warm = 2
    deltas = []
    p = prev
    for _ in range(warm + epochs):
        cs.advance()
        new = cs.epoch_input(copy=True)
        deltas.append(pin_delta(build_delta(p, new, p.kdict.n, p.pdict.n)))
        p = new
    Ts = {T} | {len(d.prev) for d in deltas if d.prev is not None}
    assert len(Ts) == 1, "the pipelined loop reuses buffers sized for one topology count"
    bufs = [BatchesOut.alloc(T, cap, cap, cap, pinned=True) for _ in range(2)]
    ones = np.ones(T, np.uint8)
    eng.commit(ones)
    t0 = None
    for ep, d in enumerate(deltas):
        if ep == warm:
            eng.download_wait()
            t0 = time.perf_counter()
        eng.upload_delta(d)                   # H2D beside the previous epoch's D2H
        eng.run()
        eng.sync()
        eng.download_wait()                   # epoch ep-1's outputs are in host memory
        eng.download_async(bufs[ep % 2])
        eng.commit(ones)
    eng.download_wait()
    wall = time.perf_counter() - t0
    return {"epochs": epochs, "e2e_ms": wall / epochs * 1e3, "links_per_s": p.desired.n * epochs / wall,
            "note": "not part of value: resident loop with epoch k's download overlapping epoch k+1's delta "
                    f"upload (full-duplex link), mean over {epochs} epochs after {warm} warm-up epochs"}


def ingest_stage(eng, inp, steps: int, reps: int = 5, cpu_sample_pods: int = 20_000):
    """Separate report (not part of `value`): CR ingest of this shard's Topology CRs as a
    TopologyList JSON document (kdtn_json_ingest: json.Unmarshal + SoA + interning on the
    GPU, document resident in HBM), then the epoch run on the ingest-produced tables (ids in
    the ingest's own interning order) next to the synthetic tables of `value`."""
    doc = synth.topology_list_json(inp)
    t = time.perf_counter()
    eng.json_upload(doc)
    h2d_s = time.perf_counter() - t
    info = eng.json_ingest()
    acc: dict[str, float] = {}
    walls = []
    for _ in range(reps):
        t = time.perf_counter()
        info = eng.json_ingest()
        walls.append(time.perf_counter() - t)
        for k, v in eng.kernel_times().items():
            acc[k] = acc.get(k, 0.0) + v / reps
    wall = sorted(walls)[len(walls) // 2]
    gpu_ms = sum(v for k, v in acc.items() if k != "js_sync")
    out_bytes = (88.0 * (info.n_desired + info.n_realised) + 25.0 * info.n_topos + info.kdict_bytes
                 + info.pdict_bytes + 4.0 * (info.n_kdict + info.n_pdict + 2))
    alg = len(doc) + out_bytes
    res = {"doc_bytes": len(doc), "links": int(info.n_desired + info.n_realised), "topologies": int(info.n_topos),
           "tokens": int(info.n_tokens), "wall_ms": wall * 1e3, "gpu_ms": gpu_ms,
           "links_per_s": (info.n_desired + info.n_realised) / wall, "json_GBps": len(doc) / wall / 1e9,
           "roofline": {"bound": "hbm", "bytes": alg, "achieved": alg / (gpu_ms * 1e-3) / 1e9,
                        "peak": HBM_PEAK_GBS, "unit": "GB/s",
                        "frac": alg / (gpu_ms * 1e-3) / 1e9 / HBM_PEAK_GBS},
           "kernels_ms": acc, "h2d_GBps": len(doc) / h2d_s / 1e9,
           "note": "not part of value; the document is resident in HBM (h2d_GBps is the PCIe "
                   "upload measured separately)"}
    del doc
    # the epoch on the ingest-produced tables (first-occurrence kdict ids)
    eng.set_timing(1)
    for _ in range(2):
        eng.run()
        eng.sync()
    ksum: dict[str, float] = {}
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(steps):
        eng.run()
        eng.sync()
        for k, v in eng.kernel_times().items():
            ksum[k] = ksum.get(k, 0.0) + v / steps
    el = (time.perf_counter() - t) / steps
    eng.set_timing(2)
    res["epoch_on_ingest_tables"] = {"ms_per_step": el * 1e3, "links_per_s": info.n_desired / el,
                                     "kernels_ms": ksum, "n_kdict": int(info.n_kdict)}
    try:
        sys.path.insert(0, os.path.join(ROOT, "oracle"))
        import oracle as O
        small = synth.make(2, pods_per_shard=cpu_sample_pods)
        sdoc = synth.topology_list_json(small)
        t = time.perf_counter()
        O.json_ingest(sdoc)
        cs = time.perf_counter() - t
        res["cpu_baseline"] = {"links_per_s": small.desired.n / cs, "json_GBps": len(sdoc) / cs / 1e9,
                               "cores": 1, "kind": "port",
                               "sample": f"oracle/kdtn_oracle_json.c on a {cpu_sample_pods}-pod config-2 "
                                         f"TopologyList ({len(sdoc)} bytes, {small.desired.n} links) in "
                                         f"{cs:.2f} s"}
    except Exception as e:   # the oracle is optional for the stage report
        res["cpu_baseline"] = {"error": str(e)}
    return res


KERNEL_SOURCES = ("kube-dtn_amd/csrc/kdtn_kernels.hip", "kube-dtn_amd/csrc/kdtn_kernels.h",
                  "kube-dtn_amd/csrc/kdtn_parse.h", "kube-dtn_amd/csrc/kdtn_engine.hip")


def kernel_src_sha16() -> str:
    """Hash of the sources that define k_reconcile and its launch (tools/pmc_traffic.py
    stamps the same hash into every PMC summary it writes)."""
    import hashlib
    h = hashlib.sha256()
    for p in KERNEL_SOURCES:
        with open(os.path.join(ROOT, p), "rb") as f:
            h.update(f.read())
    return h.hexdigest()[:16]


def pmc_traffic(config: int, links: int, placed: bool):
    """HBM bytes per k_reconcile launch (+ k_place_scan / k_place for the comparison build)
    from a committed PMC summary (profiles/*pmc_traffic*.json, written by
    tools/pmc_traffic.py from separate FETCH_SIZE / WRITE_SIZE rocprofv3 passes, gfx950
    correction applied) of the same workload AND the same kernel sources (kernel_src_sha16):
    a summary measured on other sources is never attached. The k_reconcile instantiation
    must be the build this epoch ran (the comparison build comes with k_place*). Else None."""
    import glob
    sha = kernel_src_sha16()
    best = None
    for f in sorted(glob.glob(os.path.join(ROOT, "profiles", "*pmc_traffic*.json"))):
        with open(f) as fh:
            d = json.load(fh)
        if d.get("kernel_src_sha16") != sha:
            continue
        if d.get("config", 2) != config or abs(d.get("links_per_gpu", 0) - links) > 0.01 * links:
            continue
        ks = d["kernels"]
        rec = [k for k in ks if k.startswith("k_reconcile") and "traffic_bytes" in ks[k]]
        plc = [k for k in ks if k.startswith("k_place") and "traffic_bytes" in ks[k]]
        if len(rec) != 1 or bool(plc) != placed:
            continue
        best = (sum(ks[k]["traffic_bytes"] for k in rec + plc), os.path.basename(f), rec[0])
    return best


def path_stats(inp) -> dict:
    """How k_reconcile's workgroups (64 topologies each) split between its paths: bulk (no
    topology needs element comparisons), fast (CalcDiff window in LDS, <= CAP records) and
    slow (global-scratch window)."""
    T = inp.topos
    nt = T.n
    ro, no = T.real_off.astype(np.int64), T.des_off.astype(np.int64)
    ko, kn = ro[1:] - ro[:-1], no[1:] - no[:-1]
    cmp = ((T.flags & 3) == 0) & (ko > 0) & (kn > 0)
    nwg = (nt + 63) // 64
    idx = np.arange(nwg) * 64
    anyc = np.logical_or.reduceat(cmp, idx) if nt else np.zeros(0, bool)
    tot = (ro[np.minimum(idx + 64, nt)] - ro[idx]) + (no[np.minimum(idx + 64, nt)] - no[idx])
    return {"workgroups": int(nwg), "bulk": int((~anyc).sum()), "fast": int((anyc & (tot <= 2048)).sum()),
            "slow": int((anyc & (tot > 2048)).sum())}


def allmax(x: float, world: int) -> float:
    if world == 1:
        return x
    t = torch.tensor([x], dtype=torch.float64)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t[0])


def allsum(x: float, world: int) -> float:
    if world == 1:
        return x
    t = torch.tensor([x], dtype=torch.float64)
    dist.all_reduce(t, op=dist.ReduceOp.SUM)
    return float(t[0])


_T0 = time.time()


def progress(msg: str) -> None:
    """A progress line on stderr (rank 0): long stages (generation, CPU baseline, ingest,
    resident chains) keep the run visibly alive; stdout stays the one JSON line."""
    if int(os.environ.get("RANK", "0")) == 0:
        print(f"[bench +{time.time() - _T0:6.1f}s] {msg}", file=sys.stderr, flush=True)


def barrier(world: int) -> None:
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()


def dump_outputs(d: str, rank: int, world: int, eng, inp) -> None:
    """--dump: the epoch outputs of this rank (kdtn_epoch_download) with the shard's global
    pod ids, for a parity check outside the bench (the bench itself never runs the oracle
    outside cpu_baseline)."""
    out = eng.download()
    os.makedirs(d, exist_ok=True)
    np.savez(os.path.join(d, f"rank{rank}.npz"), world=world, pod_slice=inp.pod_slice,
             gid=inp.gid if inp.gid is not None else np.arange(inp.topos.n),
             **{f: getattr(out, f) for f in out.FIELDS})


def free_port() -> int:
    import socket
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def spawn_ranks(n: int) -> int:
    """`bench.py --gpus N` without a launcher: run the N ranks as children under
    torch.distributed.run (one process per GPU, rendezvous on 127.0.0.1) and return the
    launcher's exit status. This process has not touched the GPU (nothing here initialises
    HIP), so the children own the devices; it replaces the reference's worker pool
    (controllers/topology_controller.go:335-337) with one engine process per GPU."""
    import subprocess
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    env["KDTN_BENCH_LAUNCHER"] = "bench.py --gpus (torch.distributed.run child)"
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr=127.0.0.1", f"--master-port={free_port()}", os.path.abspath(__file__)]
    cmd += sys.argv[1:]
    return subprocess.run(cmd, env=env).returncode


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=None, help="timed epochs (default 20; config 3: 10)")
    ap.add_argument("--warmup", type=int, default=None, help="untimed epochs (default 3; config 3: 1)")
    ap.add_argument("--config", type=int, default=2, choices=(1, 2, 3, 4))
    ap.add_argument("--pods", type=int, default=None,
                    help="pods of the whole topology (strong) or per GPU (weak)")
    ap.add_argument("--scaling", default="strong", choices=("strong", "weak"))
    ap.add_argument("--cpu-budget-s", type=float, default=12.0)
    ap.add_argument("--cpu-threads", type=int, default=0, help="0: min(32, CPUs this process may use)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-wire", action="store_true", help="skip the wire-encoding stage report")
    ap.add_argument("--no-ingest", action="store_true", help="skip the CR-ingest stage report")
    ap.add_argument("--no-e2e", action="store_true", help="skip the PCIe-inclusive epoch reports")
    ap.add_argument("--resident-epochs", type=int, default=5, help="config 3: epochs of the resident-chain report")
    ap.add_argument("--dump", default=None,
                    help="directory: each rank saves its last timed epoch's outputs (rank<r>.npz) for "
                         "an external parity check (tests/test_bench_gpu.py)")
    args = ap.parse_args()
    churn = args.config == 3
    steps = args.steps if args.steps is not None else (10 if churn else 20)
    warmup = args.warmup if args.warmup is not None else (1 if churn else 3)
    pods = args.pods or DEFAULT_PODS[args.config]

    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        sys.exit(spawn_ranks(args.gpus))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        print(f"bench.py: WORLD_SIZE={world} but --gpus {args.gpus}: one process per GPU is required",
              file=sys.stderr, flush=True)
        sys.exit(2)
    if args.config == 1 and world > 1:
        print("bench.py: config 1 is a one-GPU workload (SURVEY §8(d))", file=sys.stderr, flush=True)
        sys.exit(2)
    launcher = os.environ.get("KDTN_BENCH_LAUNCHER", "external" if world > 1 else "none")
    if world > 1:
        dist.init_process_group("gloo")
    ndev = torch.cuda.device_count()
    dev = local % ndev if ndev else local           # (ranks share a GPU only in host-transport tests)
    torch.cuda.set_device(dev)
    total_pods = pods if args.scaling == "strong" else pods * world

    progress(f"config {args.config}: generating the workload")
    t0 = time.time()
    cs = None
    if churn:
        cs = synth.ChurnSequence(total_pods=total_pods, shard=rank, nshards=world)
        inp = cs.epoch_input()
    elif args.config == 1:
        inp = synth.make(1)
        total_pods = inp.topos.n
    else:
        inp = synth.make(args.config, total_pods=total_pods, shard=rank, nshards=world)
    gen_s = time.time() - t0
    progress(f"generated in {gen_s:.1f} s; timed epochs")
    eng = Engine(device=dev)
    exchange = "none"
    comm_ranks = 1
    host_x = False
    if world > 1:
        # production transport: RCCL all-gather of the pod-status rows on the engine's comm
        # stream. The host transport (rows all-gathered over gloo inside every timed epoch)
        # is used when KDTN_BENCH_HOST_XCHG=1, when ranks share a device (RCCL cannot put two
        # ranks of one communicator on one GPU) or when any rank's RCCL init fails: the
        # decision is all-reduced so every rank takes the same transport.
        shared = world > max(ndev, 1)
        want_host = os.environ.get("KDTN_BENCH_HOST_XCHG") == "1" or shared
        fail = 0
        if not want_host:
            uid = [comm_unique_id() if rank == 0 else None]
            dist.broadcast_object_list(uid, src=0)
            try:
                eng.comm_init(uid[0], world, rank)
            except KdtnError as e:
                print(f"rank {rank}: RCCL communicator failed ({e})", file=sys.stderr, flush=True)
                fail = 1
        flag = torch.tensor([1 if (want_host or fail) else 0], dtype=torch.int32)
        dist.all_reduce(flag, op=dist.ReduceOp.MAX)
        host_x = bool(flag[0])
        if host_x:
            eng.set_ranks(world, rank)          # also releases a communicator this rank built
            why = ("KDTN_BENCH_HOST_XCHG=1" if os.environ.get("KDTN_BENCH_HOST_XCHG") == "1" else
                   f"{world} ranks on {ndev} device(s)" if shared else "RCCL init failed on a rank")
            exchange = f"host transport (gloo all-gather per epoch; {why})"
        else:
            exchange = "rccl all-gather"
        comm_ranks = world

    def run(stages: int = abi.STAGE_ALL) -> None:
        if host_x and (stages & abi.STAGE_RESOLVE):
            mine = torch.from_numpy(eng.pods_export(inp.pod_slice).view(np.int32).copy())
            parts = [torch.empty_like(mine) for _ in range(world)]
            dist.all_gather(parts, mine)
            eng.pods_import(torch.cat(parts).numpy().view(np.uint32))
        eng.run(stages)

    eng.upload(inp)
    # timed epochs record HIP events around k_reconcile (+ placement) only: every event costs
    # ≈5 µs of stream time; the per-stage breakdown comes from separate untimed epochs
    eng.set_timing(1)

    ksum: dict[str, float] = {}
    bsum: dict[str, float] = {}
    nbreak = 0
    counts_acc = np.zeros(3)
    bytes_acc = epoch_acc = 0.0
    links_local = 0
    elapsed = 0.0
    diff_ms = []
    pstats = None
    if not churn:
        for _ in range(warmup):
            run()
            eng.sync()
        barrier(world)
        eng.timer_totals(reset=True)
        t_start = time.perf_counter()
        counts = None
        for _ in range(steps):
            run()
            counts = eng.sync()                  # also sums this epoch's HIP-event times
        torch.cuda.synchronize()
        elapsed = time.perf_counter() - t_start
        barrier(world)
        elapsed = allmax(elapsed, world)
        for k, (v, n) in eng.timer_totals(reset=True).items():
            assert n == steps, (k, n, steps)                  # every timed epoch was marked
            ksum[k] = ksum.get(k, 0.0) + v
        links_local = inp.desired.n * steps
        eng.set_timing(2)
        for _ in range(min(steps, 5)):                    # per-stage breakdown (untimed)
            run()
            eng.sync()
            for k, v in eng.kernel_times().items():
                bsum[k] = bsum.get(k, 0.0) + v
            nbreak += 1
        eng.set_timing(1)
        counts_acc += np.array([counts.n_add, counts.n_upd, counts.n_del]) * steps
        if args.dump:
            dump_outputs(args.dump, rank, world, eng, inp)
        bytes_acc = reconcile_bytes(inp, counts.n_add, counts.n_upd, counts.n_del) * steps
        epoch_acc = epoch_bytes(inp, counts.n_add, counts.n_upd, counts.n_del) * steps
        pstats = path_stats(inp)
    else:
        # one upload per epoch (untimed), each epoch timed between barriers; sum over epochs
        for ep in range(warmup + steps):
            if ep:
                keep = (inp.kdict.n, inp.pdict.n)          # the churn interner only appends
                cs.advance()
                inp = cs.epoch_input()
                eng.upload(inp, *keep)
            timed = ep >= warmup
            barrier(world)
            t = time.perf_counter()
            run()
            counts = eng.sync()
            torch.cuda.synchronize()
            dt = time.perf_counter() - t
            kt = eng.kernel_times()
            barrier(world)
            dt = allmax(dt, world)
            if not timed:
                continue
            elapsed += dt
            for k, v in kt.items():
                ksum[k] = ksum.get(k, 0.0) + v
            links_local += inp.desired.n
            counts_acc += np.array([counts.n_add, counts.n_upd, counts.n_del])
            bytes_acc += reconcile_bytes(inp, counts.n_add, counts.n_upd, counts.n_del)
            epoch_acc += epoch_bytes(inp, counts.n_add, counts.n_upd, counts.n_del)
            run(abi.STAGE_DIFF)                      # gate + CalcDiff + lists alone (report)
            eng.sync()
            diff_ms.append(reconcile_ms(eng.kernel_times()))
            eng.set_timing(2)                            # per-stage breakdown (untimed re-run)
            run()
            eng.sync()
            for k, v in eng.kernel_times().items():
                bsum[k] = bsum.get(k, 0.0) + v
            nbreak += 1
            eng.set_timing(1)
            if pstats is None:
                pstats = path_stats(inp)
    links_total = allsum(links_local, world)
    nsteps = steps
    ms_step = elapsed / nsteps * 1e3
    kavg = {k: v / nsteps for k, v in ksum.items()}           # timed epochs: k_reconcile (+ placement)
    kstage = {k: v / max(nbreak, 1) for k, v in bsum.items()}  # untimed epochs: every stage
    bytes_launch = bytes_acc / nsteps
    dom = max(kstage, key=kstage.get) if kstage else max(kavg, key=kavg.get)
    # the comparison build's deferred chunks finish in k_place_scan + k_place: one unit of work
    placed = "place" in kavg
    rec_ms = reconcile_ms(kavg)
    roof = {"kernel": "k_reconcile+k_place_scan+k_place" if placed else "k_reconcile", "bound": "hbm",
            "achieved": bytes_launch / (rec_ms * 1e-3) / 1e9,
            "peak": HBM_PEAK_GBS, "unit": "GB/s", "traffic": None,
            "bytes_per_launch": bytes_launch, "avg_ms": rec_ms, "dominant_stage": dom}
    roof["frac"] = roof["achieved"] / roof["peak"]
    tr = pmc_traffic(args.config, inp.desired.n, placed) if world == 1 else None
    roof["kernel_src_sha16"] = kernel_src_sha16()
    if tr is not None:
        roof["traffic"] = tr[0]
        roof["traffic_source"] = (f"profiles/{tr[1]} ({tr[2]}; 2*FETCH_SIZE + WRITE_SIZE per launch, "
                                  f"measured on these kernel sources)")
    else:
        roof["traffic_source"] = "no PMC summary of this workload on these kernel sources"
    eb = epoch_acc / nsteps
    links_per_epoch = links_total / nsteps
    result = {
        "metric": "links reconciled/sec (diff+qdisc) on 10M-link topology",
        "value": links_total / elapsed,
        "unit": "links/s",
        "n_gpus": world,
        "steps": nsteps,
        "warmup": warmup,
        "ms_per_step": ms_step,
        "higher_is_better": True,
        "scaling": args.scaling,
        "vs_baseline": None,
        "dtype": "u32",
        "data": f"synthetic (kdtn_synth config {args.config}, seed 0x6b64746e), hash-sharded by namespace/name",
        "config": {"workload": WORKLOAD[args.config].format(pods=total_pods, links=int(links_per_epoch),
                                                            steps=nsteps),
                   "config": args.config, "pods_total": total_pods, "links_per_epoch": int(links_per_epoch),
                   "links_rank0": int(links_local / nsteps), "pods_rank0": inp.topos.n,
                   "parallelism": f"shard{world} (hash64(ns/name) mod {world})", "exchange": exchange,
                   "comm_ranks": comm_ranks, "launcher": launcher},
        "roofline": roof,
        "epoch_roofline": {"bytes": eb, "achieved": eb / (ms_step * 1e-3) / 1e9,
                           "peak": HBM_PEAK_GBS, "unit": "GB/s",
                           "frac": eb / (ms_step * 1e-3) / 1e9 / HBM_PEAK_GBS},
        "kernels_ms": kstage,
        "kernels_ms_note": "per-stage HIP-event times of separate untimed epochs (every stage marked); the timed "
                           "epochs carry events around k_reconcile (+ placement) only (roofline.avg_ms)",
        "counts_per_epoch_rank0": dict(zip(("add", "upd", "del"), (counts_acc / nsteps).tolist())),
        "k_reconcile_paths_rank0": pstats,
        "gen_s": round(gen_s, 2),
    }
    if not churn:
        # the next epoch over the same CR set: dictionaries resident and already parsed
        # (kdict_keep / pdict_keep = everything); a separate report, not `value`
        eng.upload(inp, inp.kdict.n, inp.pdict.n)
        for _ in range(2):
            run()
            eng.sync()
        barrier(world)
        t = time.perf_counter()
        for _ in range(steps):
            run()
            eng.sync()
        torch.cuda.synchronize()
        el = allmax(time.perf_counter() - t, world)
        eng.set_timing(2)
        rsum: dict[str, float] = {}
        for _ in range(3):                                # per-stage breakdown (untimed)
            run()
            eng.sync()
            for k, v in eng.kernel_times().items():
                rsum[k] = rsum.get(k, 0.0) + v / 3
        result["epoch_dicts_parsed"] = {"ms_per_step": el / steps * 1e3, "links_per_s": links_total / el,
                                        "kernels_ms": rsum,
                                        "note": "same epoch re-run with kdict_keep/pdict_keep = all strings "
                                                "(append-only interner, nothing new to parse)"}
    if churn:
        inp = cs.epoch_input(copy=True)          # (the generator's arrays move when it advances)
    if churn and world == 1 and not args.no_e2e:
        progress("resident chain")
        result["resident_chain"] = resident_chain_stage(eng, cs, inp, args.resident_epochs)
        progress("resident chain, pipelined")
        result["resident_pipeline"] = resident_pipeline_stage(eng, cs, cs.epoch_input(copy=True), args.resident_epochs)
        del cs
        # the same with Topologies created and deleted (informer add / delete events)
        progress("resident chain with a changing Topology set")
        tc = synth.TopologySetChurn(frac=0.01, total_pods=total_pods)
        p0 = tc.epoch_input()
        eng.upload(p0)
        eng.run()
        eng.sync()
        result["resident_chain_topology_set"] = resident_chain_stage(eng, tc, p0, args.resident_epochs,
                                                                     topology_set=True)
        del tc, p0
        progress("resident chain with a changing Topology set, pipelined")
        tc = synth.TopologySetChurn(frac=0.01, total_pods=total_pods)
        p0 = tc.epoch_input()
        eng.upload(p0)
        eng.run()
        eng.sync()
        result["resident_pipeline_topology_set"] = resident_pipeline_stage(eng, tc, p0, args.resident_epochs)
        del tc, p0
    if diff_ms:
        result["diff_only_reconcile_ms"] = float(np.mean(diff_ms))
        result["diff_share_of_reconcile"] = float(np.mean(diff_ms)) / rec_ms
    if world == 1 and not args.no_e2e and not churn:
        progress("PCIe-inclusive epoch")
        result["e2e_pcie"] = e2e_stage(eng, inp)
    if world == 1 and not args.no_wire and args.config == 2:
        progress("output stages")
        result["wire_stage"] = wire_stage(eng)
    if world == 1 and not args.no_cpu_baseline:            # CPU baseline: rank 0 at N=1 only
        share, info = cpu_share()
        threads = args.cpu_threads or min(32, share)
        progress(f"CPU baseline on {threads} threads")
        result["cpu_baseline"] = cpu_baseline(inp, args.cpu_budget_s, threads, info)
    if world == 1 and args.config == 4:                    # VxlanManager maps after the epoch
        run()
        eng.sync()
        eng.vni_apply()                                    # first call sizes the work buffers
        t = time.perf_counter()
        vm = eng.vni_apply()                               # same epoch: the same map again
        wall = time.perf_counter() - t
        kt = eng.kernel_times()
        result["vni_apply_stage"] = {"entries_before": int(inp.vnis.n), "entries_after": int(vm.n),
                                     "gpu_ms": sum(kt.values()), "kernels_ms": kt, "wall_ms": wall * 1e3,
                                     "note": "not part of value: kdtn_epoch_vni_apply (deletes, then first-wins "
                                             "adds of the reached entries) + download of the map"}
    if world == 1 and not args.no_ingest and args.config == 2:
        progress("CR ingest stage")
        result["ingest_stage"] = ingest_stage(eng, inp, steps)
    if rank == 0:
        print(json.dumps(result), flush=True)
    eng.close()
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
