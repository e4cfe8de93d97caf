"""Per-stage ablation of one reconcile epoch (one process, data generated once).

    python tools/ablate.py [--pods N] [--config C] [--reps R]
(--variants / --env A/B runs load the profiling library: make -C kube-dtn_amd prof)
Prints per-kernel HIP-event times for stage masks ALL, DIFF|RESOLVE, DIFF|QDISC, DIFF.
"""
import argparse
import json
import os
import sys

import torch  # noqa: F401  (one HIP runtime)

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "kube-dtn_amd"))
from kdtn import Engine, abi, synth  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--pods", type=int, default=1_000_000)
ap.add_argument("--config", type=int, default=2)
ap.add_argument("--reps", type=int, default=10)
ap.add_argument("--masks", default="ALL,DIFF|RESOLVE,DIFF|QDISC,DIFF")
ap.add_argument("--cache", default="")
ap.add_argument("--variants", default="", help="comma list of KDTN_VARIANT values, interleaved")
ap.add_argument("--env", default="", help="NAME=v1,v2,...: interleaved A/B of an env knob, all stages timed")
ap.add_argument("--wall", action="store_true", help="--env: also the wall time of run + sync at timing level 0")
ap.add_argument("--churn", type=int, default=0, help="--variants (or --env, wall time) over K epochs of the config-3 churn sequence "
                "(each epoch uploaded once, the variants interleaved on it; k_reconcile + placement)")
a = ap.parse_args()
if a.variants or a.env:                 # A/B variants live in the profiling build
    from kdtn import engine as _kdtn_engine
    _kdtn_engine.use_profiling_library()
res = {}
if a.churn and a.env:                    # churn epochs: wall time of run + sync per env value
    import time
    name, vals = a.env.split("=")
    vs = vals.split(",")
    cs = synth.ChurnSequence(pods_per_shard=a.pods)
    eng = Engine(device=0)
    eng.set_timing(0)
    per = {v: [] for v in vs}
    inp = cs.epoch_input()
    for ep in range(a.churn):
        if ep:
            keep = (inp.kdict.n, inp.pdict.n)
            cs.advance()
            inp = cs.epoch_input()
            eng.upload(inp, *keep)
        else:
            eng.upload(inp)
        acc = {v: [] for v in vs}
        for rep in range(a.reps + 2):
            for v in vs:
                os.environ[name] = v
                t = time.perf_counter()
                eng.run(abi.STAGE_ALL)
                eng.sync()
                if rep >= 2:
                    acc[v].append((time.perf_counter() - t) * 1e3)
        for v in vs:
            per[v].append(sorted(acc[v])[len(acc[v]) // 2])
    os.environ.pop(name)
    print(json.dumps({"config": 3, "pods": a.pods, "epochs": a.churn, "reps": a.reps, "env": name,
                      "epoch_wall_ms": {v: {"mean_of_epoch_medians": round(sum(x) / len(x), 4),
                                            "per_epoch": [round(y, 4) for y in x]} for v, x in per.items()}},
                     indent=1))
    sys.exit(0)
if a.churn:                              # config 3 as the bench runs it: the churn sequence
    cs = synth.ChurnSequence(pods_per_shard=a.pods)
    eng = Engine(device=0)
    vs = a.variants.split(",")
    per = {v: [] for v in vs}
    inp = cs.epoch_input()
    for ep in range(a.churn):
        if ep:
            keep = (inp.kdict.n, inp.pdict.n)
            cs.advance()
            inp = cs.epoch_input()
            eng.upload(inp, *keep)
        else:
            eng.upload(inp)
        acc = {v: [] for v in vs}
        for rep in range(a.reps + 2):
            for v in vs:
                os.environ["KDTN_VARIANT"] = v
                eng.run(abi.STAGE_ALL)
                eng.sync()
                if rep >= 2:
                    kt = eng.kernel_times()
                    acc[v].append(kt["reconcile"] + kt.get("place", 0.0))
        for v in vs:
            per[v].append(sorted(acc[v])[len(acc[v]) // 2])
    os.environ.pop("KDTN_VARIANT")
    print(json.dumps({"config": 3, "pods": a.pods, "epochs": a.churn, "reps": a.reps,
                      "reconcile_plus_place_ms": {v: {"mean_of_epoch_medians": round(sum(x) / len(x), 4),
                                                      "per_epoch": [round(y, 4) for y in x]} for v, x in per.items()}},
                     indent=1))
    sys.exit(0)
inp = synth.make(a.config, pods_per_shard=a.pods, cache_dir=a.cache or None)
eng = Engine(device=0)
eng.upload(inp)
if a.variants:
    vs = [v for v in a.variants.split(",")]
    acc = {v: [] for v in vs}
    for rep in range(a.reps + 2):
        for v in vs:                      # interleaved rounds (cdna_hip_programming.md rule 24)
            os.environ["KDTN_VARIANT"] = v
            eng.run(abi.STAGE_ALL)
            eng.sync()
            if rep >= 2:
                kt = eng.kernel_times()
                acc[v].append(kt["reconcile"] + kt.get("qdisc", 0.0))   # split-qdisc variants
    os.environ.pop("KDTN_VARIANT")
    for v in vs:
        x = sorted(acc[v])
        res["variant_" + v] = {"median": round(x[len(x) // 2], 4), "min": round(x[0], 4)}
if a.env:
    name, vals = a.env.split("=")
    acc = {v: {} for v in vals.split(",")}
    for rep in range(a.reps + 2):
        for v in acc:
            os.environ[name] = v
            eng.run(abi.STAGE_ALL)
            eng.sync()
            if rep >= 2:
                for k, t in eng.kernel_times().items():
                    acc[v].setdefault(k, []).append(t)
    if a.wall:                            # epoch wall time, no timing events
        import time
        eng.set_timing(0)
        for rep in range(a.reps + 2):
            for v in acc:
                os.environ[name] = v
                t = time.perf_counter()
                eng.run(abi.STAGE_ALL)
                eng.sync()
                if rep >= 2:
                    acc[v].setdefault("epoch_L0", []).append((time.perf_counter() - t) * 1e3)
    os.environ.pop(name)
    for v, d in acc.items():
        res[f"{name}={v}"] = {k: round(sorted(x)[len(x) // 2], 4) for k, x in d.items()}
masks = {"ALL": abi.STAGE_ALL, "DIFF|RESOLVE": abi.STAGE_DIFF | abi.STAGE_RESOLVE,
         "DIFF|QDISC": abi.STAGE_DIFF | abi.STAGE_QDISC, "DIFF": abi.STAGE_DIFF}
for name, m in masks.items():
    if name not in a.masks.split(","):
        continue
    acc = {}
    for r in range(a.reps + 2):
        eng.run(m)
        eng.sync()
        if r >= 2:
            for k, v in eng.kernel_times().items():
                acc[k] = acc.get(k, 0.0) + v / a.reps
    res[name] = {k: round(v, 4) for k, v in acc.items()}
print(json.dumps({"config": a.config, "pods": a.pods, "links": inp.desired.n, "ms": res}, indent=1))
