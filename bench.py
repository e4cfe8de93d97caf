#!/usr/bin/env python3
"""bench.py — links reconciled/sec of the MI355X reconcile engine (BASELINE.json metric).

One step = one reconcile epoch over this rank's shard, inputs resident in HBM:
  dictionary parse → pod-status table (+ RCCL all-gather across ranks) → lookup tables →
  Reconcile gate + CalcDiff → batch compaction → addLink/delLink/UpdateLinks pure prefix
  → MakeQdiscs; the host waits for each epoch (kdtn_epoch_sync).
Workload (BASELINE configs[2]): per GPU a 1M-pod shard of a random
10-regular topology — 10M Link records with heterogeneous netem/tbf properties — all
AddLinks (realised status non-nil and empty). Weak scaling: every rank owns 1M pods of a
(N × 1M)-pod graph; peers are spread over all shards, so each epoch all-gathers the
pod-status table over RCCL/xGMI.

    python bench.py [--gpus N] [--steps K] [--warmup W]
For N > 1 launch with torch.distributed.run (one process per GPU).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import torch  # noqa: E402  (first: one HIP runtime per process, see kdtn/engine.py)
import torch.distributed as dist

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "kube-dtn_amd"))

from kdtn import Engine, abi, comm_unique_id, synth  # noqa: E402

HBM_PEAK_GBS = 8000.0   # MI355X HBM3E spec peak (MI355X_MICROARCH.md, chip-level parameters)


def reconcile_bytes(inp, n_add: int, n_upd: int, n_del: int) -> float:
    """Algorithmic bytes of one k_reconcile launch: per AddLinks entry
    1 (flag) + 12 (local_ip, local_mac, peer_pod ids) + 8 (uid) + 48 (12 prop ids) + 4 (gap)
    read, 4 (index) + 16 (resolve record) + 72 (qdisc) written = 165 B; per topology
    8 (offsets) + 1 (action) + 12 (ns, src_ip, net_ns) read + 12 (3 batch offsets) written
    = 33 B; plus the 24 B parsed record of every property string, read once."""
    T = inp.topos.n
    per_add = 165.0
    per_upd = 1 + 4 + 12 + 48 + 4 + 8 + 4 + 16 + 72   # flag, target, ids, props, gap, uid, out
    per_del = 1 + 12 + 8 + 4 + 16
    # every realised record is compared (key + props) against the desired side when both
    # lists are non-empty: 88 B per record per side (only when M > 0)
    cmp = 88.0 * (inp.realised.n + (inp.desired.n if inp.realised.n else 0))
    return (per_add * n_add + per_upd * n_upd + per_del * n_del + 33.0 * T + 24.0 * inp.pdict.n
            + cmp)


def epoch_bytes(inp, n_add: int, n_upd: int, n_del: int) -> float:
    """SURVEY §8(d) whole-epoch model: 92·M + 92·N + 16·T + 4·lists + 36·|add| + 72·|add∪upd|
    + unique property-string bytes."""
    M, N, T = inp.realised.n, inp.desired.n, inp.topos.n
    return (92.0 * (M + N) + 16.0 * T + 4.0 * (n_add + n_upd + n_del) + 36.0 * n_add
            + 72.0 * (n_add + n_upd) + float(inp.pdict.offs[-1]))


def cpu_baseline(inp, budget_s: float, threads: int):
    """The CPU oracle (C restatement of the reference Go path) on a bounded sample of this
    workload's topologies, loop time only (informer maps pre-built). Single thread, then
    `threads` workers over disjoint topology ranges, mirroring the reference's
    MaxConcurrentReconciles worker pool (controllers/topology_controller.go:335-337); the
    ctypes call releases the GIL, so the workers run concurrently."""
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
    # worker pool: each worker takes an equal slice of a sample `threads` times larger
    n_par = int(min(T, want * threads))
    bounds = [n_par * k // threads for k in range(threads + 1)]
    ptim = [[] for _ in range(threads)]
    with ThreadPoolExecutor(threads) as ex:
        list(ex.map(lambda k: O.reconcile(inp, t_begin=bounds[k], t_end=bounds[k + 1],
                                          timing=ptim[k]), range(threads)))
    par_links = int(inp.topos.des_off[n_par] - inp.topos.des_off[0])
    par_s = max(t[-1] for t in ptim)
    return {"value": par_links / par_s, "unit": "links/s", "cores": threads, "kind": "port",
            "value_1thread": one,
            "sample": f"oracle/kdtn_oracle.c (literal CalcDiff loops, per-link MakeQdiscs, "
                      f"map-based resolve) on rank 0's shard: {threads} threads over "
                      f"topologies [0,{n_par}) = {par_links} links in {par_s:.2f} s (slowest "
                      f"worker's loop); single thread: [0,{want}) = {links} links in "
                      f"{timing[-1]:.2f} s (host nproc={os.cpu_count()})"}


def wire_stage(eng, reps: int = 5):
    """Separate report (not part of `value`): the protobuf wire encoding of every batch of
    the epoch (kdtn_epoch_encode: proto.Marshal of each LinksBatchQuery Reconcile sends).
    GPU kernel time from HIP events, excluding the one host round trip that sizes the
    arena; bytes = serialized output."""
    eng.run()
    eng.sync()
    eng.encode()
    acc: dict[str, float] = {}
    n = 0
    for _ in range(reps):
        n = eng.encode()
        for k, v in eng.kernel_times().items():
            acc[k] = acc.get(k, 0.0) + v / reps
    gpu_ms = sum(v for k, v in acc.items() if k != "wire_host_sync")
    res = {"bytes": n, "gpu_ms": gpu_ms, "out_GBps": n / (gpu_ms * 1e-3) / 1e9,
           "kernels_ms": acc, "note": "not part of value; arena-size host round trip excluded"}
    # RemotePod fan-out grouped per destination daemon (kdtn_epoch_fanout)
    eng.fanout()
    facc: dict[str, float] = {}
    for _ in range(reps):
        node, off, idx = eng.fanout()
        for k, v in eng.kernel_times().items():
            facc[k] = facc.get(k, 0.0) + v / reps
    res["fanout"] = {"daemons": int(len(node)), "remote_rpcs": int(len(idx)),
                     "gpu_ms": sum(v for k, v in facc.items() if k != "fanout_host_sync"),
                     "kernels_ms": facc}
    return res


def ingest_stage(eng, inp, reps: int = 5, cpu_sample_pods: int = 20_000):
    """Separate report (not part of `value`): CR ingest of this shard's Topology CRs as a
    TopologyList JSON document (kdtn_json_ingest: json.Unmarshal + SoA + interning on the
    GPU, document resident in HBM). Wall time per ingest includes its three host round
    trips (token / element counts, intern table fill); roofline bytes = document read once
    + the decoded tables written once (88 B per link record, 25 B per topology, dictionary
    arenas + offsets). CPU baseline: the oracle's decode (oracle/kdtn_oracle_json.c, the
    reference's json.Unmarshal restated) single-threaded on a bounded slice of the workload."""
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


def pmc_traffic(links_per_gpu: int):
    """HBM bytes per k_reconcile launch from the newest committed PMC summary of the same
    workload (profiles/*_pmc_traffic.json, written by tools/pmc_traffic.py from separate
    FETCH_SIZE / WRITE_SIZE rocprofv3 passes, gfx950 correction applied), else None."""
    import glob
    best = None
    for f in sorted(glob.glob(os.path.join(ROOT, "profiles", "*_pmc_traffic.json"))):
        with open(f) as fh:
            d = json.load(fh)
        if d.get("links_per_gpu") != links_per_gpu:
            continue
        for k, v in d["kernels"].items():
            if k.startswith("k_reconcile") and "traffic_bytes" in v:
                best = (v["traffic_bytes"], os.path.basename(f))
    return best


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--pods", type=int, default=1_000_000, help="pods per GPU shard")
    ap.add_argument("--config", type=int, default=2)
    ap.add_argument("--cpu-budget-s", type=float, default=12.0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-wire", action="store_true", help="skip the wire-encoding stage report")
    ap.add_argument("--no-ingest", action="store_true", help="skip the CR-ingest stage report")
    ap.add_argument("--cpu-threads", type=int, default=16,
                    help="CPU-baseline worker threads (the GPU box's CPU share is 16)")
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        dist.init_process_group("gloo")
    torch.cuda.set_device(local)

    t0 = time.time()
    inp = synth.make(args.config, pods_per_shard=args.pods, shard=rank, nshards=world)
    gen_s = time.time() - t0
    eng = Engine(device=local)
    if world > 1:
        uid = [comm_unique_id() if rank == 0 else None]
        dist.broadcast_object_list(uid, src=0)
        eng.comm_init(uid[0], world, rank)
    eng.upload(inp)

    for _ in range(args.warmup):
        eng.run()
        eng.sync()

    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    ksum: dict[str, float] = {}
    t_start = time.perf_counter()
    counts = None
    for _ in range(args.steps):
        eng.run()
        counts = eng.sync()
        for k, v in eng.kernel_times().items():
            ksum[k] = ksum.get(k, 0.0) + v
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t_start
    if world > 1:
        dist.barrier()
        t = torch.tensor([elapsed], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t[0])
        n = torch.tensor([inp.desired.n], dtype=torch.float64)
        dist.all_reduce(n, op=dist.ReduceOp.SUM)
        links_total = float(n[0])
    else:
        links_total = float(inp.desired.n)

    ms_step = elapsed / args.steps * 1e3
    kavg = {k: v / args.steps for k, v in ksum.items()}
    dom = max(kavg, key=kavg.get)
    ebytes = reconcile_bytes(inp, counts.n_add, counts.n_upd, counts.n_del)
    roof = {"kernel": "k_reconcile", "bound": "hbm",
            "achieved": ebytes / (kavg["reconcile"] * 1e-3) / 1e9,
            "peak": HBM_PEAK_GBS, "unit": "GB/s", "traffic": None,
            "bytes_per_launch": ebytes, "avg_ms": kavg["reconcile"], "dominant_stage": dom}
    roof["frac"] = roof["achieved"] / roof["peak"]
    tr = pmc_traffic(inp.desired.n)
    if tr is not None:
        roof["traffic"] = tr[0]
        roof["traffic_source"] = f"profiles/{tr[1]} (2*FETCH_SIZE + WRITE_SIZE per launch)"
    pbytes = epoch_bytes(inp, counts.n_add, counts.n_upd, counts.n_del)
    result = {
        "metric": "links reconciled/sec (diff+qdisc) on 10M-link topology",
        "value": links_total / (elapsed / args.steps),
        "unit": "links/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": ms_step,
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "u32",
        "data": "synthetic (kdtn_synth config 2, seed 0x6b64746e)",
        "config": {"workload": f"config{args.config}: {args.pods}-pod shard per GPU of a random "
                               f"10-regular topology, {inp.desired.n} links/GPU, heterogeneous "
                               f"netem/tbf props, all AddLinks (resolve + qdisc on every link)",
                   "pods_per_gpu": inp.topos.n, "links_per_gpu": inp.desired.n,
                   "global_links": int(links_total), "parallelism": f"shard{world}"},
        "roofline": roof,
        "epoch_roofline": {"bytes": pbytes, "achieved": pbytes / (ms_step * 1e-3) / 1e9,
                           "peak": HBM_PEAK_GBS, "unit": "GB/s",
                           "frac": pbytes / (ms_step * 1e-3) / 1e9 / HBM_PEAK_GBS},
        "kernels_ms": kavg,
        "counts": {"add": counts.n_add, "upd": counts.n_upd, "del": counts.n_del},
        "gen_s": round(gen_s, 2),
    }
    if not args.no_wire and world == 1:
        result["wire_stage"] = wire_stage(eng)
    if world == 1 and not args.no_cpu_baseline:            # CPU baseline: rank 0 at N=1 only
        result["cpu_baseline"] = cpu_baseline(inp, args.cpu_budget_s, args.cpu_threads)
    if not args.no_ingest and world == 1:
        result["ingest_stage"] = ingest_stage(eng, inp)
    if rank == 0:
        print(json.dumps(result), flush=True)
    eng.close()
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
