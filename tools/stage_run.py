"""One config-2 epoch and its output stages in one process, for rocprofv3 runs.

    python tools/stage_run.py [--pods N] [--reps R] [--cache DIR] [--stages run,encode,fanout,remote,tc]
Prints the HIP-event kernel times per stage (mean over reps) as JSON.
"""
import argparse
import json
import os
import sys

import torch  # noqa: F401  (one HIP runtime)

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "kube-dtn_amd"))
from kdtn import Engine, synth  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--pods", type=int, default=1_000_000)
ap.add_argument("--config", type=int, default=2)
ap.add_argument("--reps", type=int, default=3)
ap.add_argument("--cache", default="/tmp/kdtn_cache")
ap.add_argument("--stages", default="run,encode,fanout,remote,tc")
ap.add_argument("--prof", action="store_true", help="load the profiling build (A/B variants)")
a = ap.parse_args()
if a.prof:
    from kdtn import engine as _kdtn_engine
    _kdtn_engine.use_profiling_library()
inp = synth.make(a.config, pods_per_shard=a.pods, cache_dir=a.cache or None)
eng = Engine(device=0)
eng.upload(inp)
stages = a.stages.split(",")
res = {}


def timed(name, fn):
    acc = res.setdefault(name, {})
    fn()
    for k, v in eng.kernel_times().items():
        acc[k] = acc.get(k, 0.0) + v / a.reps


# per epoch: the run, then the output stages in a controller's order (per-run tables are built
# by the first stage that needs them); one warm-up epoch, then the mean over reps
for rep in range(a.reps + 1):
    if rep == 1:
        res.clear()
    eng.run()
    eng.sync()
    if "encode" in stages:
        timed("encode", eng.encode)
    if "fanout" in stages:
        timed("fanout", eng.fanout)
    if "remote" in stages:
        timed("remote", eng.remote_encode)
    if "tc" in stages:
        c = eng.sync()
        timed("tc", lambda: eng.tc_argv(c.n_add, c.n_upd))
res = {s: {k: round(v, 4) for k, v in d.items()} for s, d in res.items()}
print(json.dumps({"config": a.config, "pods": a.pods, "links": inp.desired.n, "ms": res}, indent=1))
