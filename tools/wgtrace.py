"""Per-workgroup phase timeline of k_reconcile (KDTN_VARIANT bit 16 build of the kernel).

    python tools/wgtrace.py [--pods N] [--config C] [--variant V] [--out file.npy]
Phases: 0 entry → 1 topologies loaded → 2 counts done → 3 batch bases (look-back) → 4 end.
Prints phase-duration percentiles (µs), workgroup lifetime, mean residency and XCD spread.
"""
import argparse
import json
import os
import sys

import numpy as np
import torch  # noqa: F401  (one HIP runtime)

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "kube-dtn_amd"))
from kdtn import engine as _kdtn_engine  # noqa: E402
_kdtn_engine.use_profiling_library()   # A/B variants live in the profiling build
from kdtn import Engine, abi, synth  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--pods", type=int, default=1_000_000)
ap.add_argument("--config", type=int, default=2)
ap.add_argument("--variant", type=int, default=17)
ap.add_argument("--reps", type=int, default=3)
ap.add_argument("--cache", default="")
ap.add_argument("--out", default="")
a = ap.parse_args()
assert a.variant & 16, "trace bit (16) required"
if a.config == 3:                       # the second churn epoch (dictionaries append-only)
    cs = synth.ChurnSequence(pods_per_shard=a.pods)
    inp0 = cs.epoch_input()
    keep = (inp0.kdict.n, inp0.pdict.n)
    eng0 = None
else:
    inp = synth.make(a.config, pods_per_shard=a.pods, cache_dir=a.cache or None)
eng = Engine(device=0)
if a.config == 3:
    eng.upload(inp0)
    eng.run()
    eng.sync()
    cs.advance()
    inp = cs.epoch_input()
    eng.upload(inp, *keep)
else:
    eng.upload(inp)
os.environ["KDTN_VARIANT"] = str(a.variant)
for _ in range(a.reps):
    eng.run(abi.STAGE_ALL)
    eng.sync()
tr = eng.wg_trace().astype(np.int64)
ms = eng.kernel_times()["reconcile"]
os.environ.pop("KDTN_VARIANT")
if a.out:
    np.save(a.out, tr)
t = tr[:, :5] - tr[:, 0].min()          # 10 ns ticks
us = t * 0.01
dur = {f"p{k}->{k + 1}": np.diff(us[:, k:k + 2], axis=1)[:, 0] for k in range(4)}
life = us[:, 4] - us[:, 0]
span = us[:, 4].max()
xcc = (tr[:, 5] >> 32) & 0xF
pct = lambda x: {q: round(float(np.percentile(x, q)), 2) for q in (10, 50, 90, 99)}
res = {"config": a.config, "pods": a.pods, "nwg": int(tr.shape[0]), "kernel_ms_event": round(ms, 4),
       "span_us": round(float(span), 2), "lifetime_us": pct(life),
       "mean_resident_wgs": round(float(life.sum() / span), 1),
       "phases_us": {k: pct(v) for k, v in dur.items()},
       "start_spread_us": pct(us[:, 0]),
       "wgs_per_xcc": np.bincount(xcc, minlength=8).tolist()}
# look-back wait vs ticket order: how far back does a typical workgroup wait
tw = tr.shape[1]
if tw >= 8 and (tr[:, 6] > 0).any():           # fast-path CalcDiff window phases
    m = tr[:, 6] > 0
    res["diff_phaseA_us"] = pct((tr[m, 6] - tr[m, 1]) * 0.01)
    res["diff_phaseB_us"] = pct((tr[m, 7] - tr[m, 6]) * 0.01)
    res["diff_rest_to_counts_us"] = pct((tr[m, 2] - tr[m, 7]) * 0.01)
res["lookback_by_decile_us"] = [round(float(np.median(dur["p2->3"][i::10])), 2) for i in range(10)]
print(json.dumps(res, indent=1))
