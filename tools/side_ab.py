"""A/B of the epoch front (profiling build): --knob KDTN_FUSE (0 the launches in sequence,
1 the pod-table work fused into the dictionary-parse launches; round 3 also measured KDTN_SIDE,
a side stream for the tables, since removed: profiles/r03u_side_ab.json). Config-2 epochs at
timing level 0, modes interleaved, median wall time of run + sync per epoch; every mode must
produce the same epoch.
Usage: python tools/side_ab.py [--pods 1000000] [--reps 30] [--knob KDTN_FUSE] [--modes 0,1]"""
import argparse
import json
import os
import sys
import time

import torch  # noqa: F401  (one HIP runtime per process)

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "kube-dtn_amd"))
from kdtn import Engine, synth  # noqa: E402
from kdtn import engine as _e  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--pods", type=int, default=1_000_000)
ap.add_argument("--reps", type=int, default=30)
ap.add_argument("--modes", default="0,1")
ap.add_argument("--knob", default="KDTN_FUSE")
ap.add_argument("--cache", default="")
a = ap.parse_args()
_e.use_profiling_library()
inp = synth.make(2, pods_per_shard=a.pods, cache_dir=a.cache or None)
modes = a.modes.split(",")
with Engine(device=0) as eng:
    eng.upload(inp)
    ref = None
    acc = {m: [] for m in modes}
    kt = {}
    for m in modes:                                     # level-2 stage times, one per mode
        os.environ[a.knob] = m
        eng.set_timing(2)
        for _ in range(3):
            eng.run()
            eng.sync()
        kt[m] = {k: round(v, 4) for k, v in eng.kernel_times().items()}
        out = eng.download()
        if ref is None:
            ref = out
        assert not out.mismatches(ref), m          # every mode: the same epoch
    eng.set_timing(0)
    for r in range(a.reps + 3):
        for m in modes:
            os.environ[a.knob] = m
            t0 = time.perf_counter()
            eng.run()
            eng.sync()
            if r >= 3:
                acc[m].append(time.perf_counter() - t0)
    med = lambda x: round(sorted(x)[len(x) // 2] * 1e3, 4)
    print(json.dumps({"pods": a.pods, "ms_epoch_median": {m: med(acc[m]) for m in modes},
                      "ms_epoch_min": {m: round(min(acc[m]) * 1e3, 4) for m in modes},
                      "kernels_ms_level2": kt}, indent=1))
