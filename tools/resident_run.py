"""The config-3 resident controller loop, epoch by epoch (profiling tool): a full upload, then
per epoch kdtn_epoch_upload_delta + run + download + commit, each phase timed on the host.
Deltas are built and pinned before the loop. Prints one JSON line per epoch and a summary.

    python tools/resident_run.py [--pods 1000000] [--epochs 6] [--topology-set FRAC]
"""
import argparse
import json
import os
import sys
import time

import torch  # noqa: F401  (one HIP runtime)

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "kube-dtn_amd"))
import numpy as np  # noqa: E402

if os.environ.get("KDTN_ALLOC_LOG") or "--sdma-engines" in sys.argv:   # profiling build only
    from kdtn import engine as _e  # noqa: E402
    _e.use_profiling_library()
from kdtn import Engine, synth  # noqa: E402
from kdtn.delta import build_delta  # noqa: E402
from kdtn.engine import pin_delta  # noqa: E402
from kdtn.tables import BatchesOut  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--pods", type=int, default=1_000_000)
ap.add_argument("--epochs", type=int, default=6)
ap.add_argument("--topology-set", type=float, default=0.0, help="fraction of Topologies deleted/created per epoch")
ap.add_argument("--pipeline", action="store_true", help="epoch k's download overlapping epoch k+1's upload")
ap.add_argument("--maps", default="", help="write /proc/self/maps here at exit (symbolising a crash's PCs)")
ap.add_argument("--sdma-engines", default="", help="(profiling build) comma list of SDMA engine bits for the "
                "download, one fresh context each")
ap.add_argument("--both", action="store_true", help="the serial loop, then the pipelined one")
a = ap.parse_args()
if a.maps:
    import atexit
    import shutil
    atexit.register(lambda: shutil.copyfile("/proc/self/maps", a.maps))
src = (synth.TopologySetChurn(frac=a.topology_set, total_pods=a.pods) if a.topology_set
       else synth.ChurnSequence(total_pods=a.pods))
prev = src.epoch_input(copy=True)
deltas = []
p = prev
for _ in range(a.epochs):
    src.advance()
    new = src.epoch_input(copy=True)
    deltas.append((pin_delta(build_delta(p, new, p.kdict.n, p.pdict.n)), new.topos.n, new.desired.n))
    p = new
def loop(pipeline: bool, label: dict):
    """One pass of the resident loop over the prebuilt deltas on a fresh context."""
    eng = Engine(device=0)
    eng.upload(prev)
    eng.run()
    eng.sync()
    eng.commit(np.ones(prev.topos.n, np.uint8))
    cap = max(1 << 20, prev.desired.n // 8)
    into = None
    rows = []
    if pipeline:
        bufs = [BatchesOut.alloc(prev.topos.n, cap, cap, cap, pinned=True) for _ in range(2)]
        for ep, (d, T, N) in enumerate(deltas):
            print(f"[resident_run] epoch {ep}", file=sys.stderr, flush=True)
            t0 = time.perf_counter()
            eng.upload_delta(d)
            t1 = time.perf_counter()
            eng.run()
            eng.sync()
            t2 = time.perf_counter()
            eng.download_wait()
            t3 = time.perf_counter()
            eng.download_async(bufs[ep % 2])
            eng.commit(np.ones(T, np.uint8))
            t4 = time.perf_counter()
            r = {"epoch": ep, "upload_ms": (t1 - t0) * 1e3, "run_ms": (t2 - t1) * 1e3,
                 "wait_prev_download_ms": (t3 - t2) * 1e3, "async_commit_ms": (t4 - t3) * 1e3,
                 "e2e_ms": (t4 - t0) * 1e3, **label}
            rows.append(r)
            print(json.dumps(r), flush=True)
        eng.download_wait()
        eng.close()
        steady = rows[1:]
        print(json.dumps({"summary_excluding_first": {k: float(np.mean([r[k] for r in steady])) for k in rows[0]
                                                      if k not in ("epoch",) and k not in label}, **label}), flush=True)
        return
    for ep, (d, T, N) in enumerate(deltas):
        if into is None or len(into.action) != T:
            into = BatchesOut.alloc(T, cap, cap, cap, pinned=True)
        print(f"[resident_run] epoch {ep}", file=sys.stderr, flush=True)
        t0 = time.perf_counter()
        eng.upload_delta(d)
        t1 = time.perf_counter()
        eng.run()
        eng.sync()
        t2 = time.perf_counter()
        out = eng.download(into)
        t3 = time.perf_counter()
        eng.commit(np.ones(T, np.uint8))
        t4 = time.perf_counter()
        down_b = sum(getattr(out, f).nbytes for f in out.FIELDS)
        r = {"epoch": ep, "upload_ms": (t1 - t0) * 1e3, "upload_bytes": d.upload_bytes(),
             "upload_GBps": d.upload_bytes() / (t1 - t0) / 1e9, "run_ms": (t2 - t1) * 1e3,
             "download_ms": (t3 - t2) * 1e3, "download_GBps": down_b / (t3 - t2) / 1e9,
             "commit_ms": (t4 - t3) * 1e3, "e2e_ms": (t4 - t0) * 1e3,
             "refs": int(len(d.ref)), "inline": int(d.records.n), "changed": d.n_changed, **label}
        rows.append(r)
        print(json.dumps(r), flush=True)
    steady = rows[1:] if len(rows) > 1 else rows
    print(json.dumps({"summary_excluding_first": {k: float(np.mean([r[k] for r in steady]))
                                                  for k in ("upload_ms", "upload_GBps", "run_ms", "download_ms",
                                                            "download_GBps", "commit_ms", "e2e_ms")}, **label}),
          flush=True)
    eng.close()


engines = [e for e in a.sdma_engines.split(",") if e] or [None]
for e in engines:
    if e is not None:
        os.environ["KDTN_SDMA_ENGINE"] = e          # read when a context first downloads by SDMA
    for pipe in ([False, True] if a.both else [a.pipeline]):
        loop(pipe, {"sdma_engine": e, "pipeline": pipe})
