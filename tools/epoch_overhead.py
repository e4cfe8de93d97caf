"""Per-epoch fixed costs on one GPU: ms per epoch (run + sync) at timing levels 0/1/2 and the
host time of the kdtn_epoch_run call alone (kernel enqueue), for config 2 at several sizes.
Usage: python tools/epoch_overhead.py [--pods 1000000,125000] [--reps 30]"""
import argparse
import json
import os
import sys
import time

import torch  # noqa: F401  (one HIP runtime per process)

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "kube-dtn_amd"))
from kdtn import Engine, synth  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--pods", default="1000000,125000")
ap.add_argument("--reps", type=int, default=30)
ap.add_argument("--config", type=int, default=2)
a = ap.parse_args()
for pods in [int(x) for x in a.pods.split(",")]:
    inp = synth.make(a.config, total_pods=pods)
    with Engine(device=0) as eng:
        eng.upload(inp)
        row = {"config": a.config, "pods": pods, "links": int(inp.desired.n)}
        for level in (2, 1, 0):
            eng.set_timing(level)
            for _ in range(3):
                eng.run()
                eng.sync()
            enq, tot = [], []
            for _ in range(a.reps):
                t0 = time.perf_counter()
                eng.run()
                t1 = time.perf_counter()
                eng.sync()
                t2 = time.perf_counter()
                enq.append(t1 - t0)
                tot.append(t2 - t0)
            med = lambda x: sorted(x)[len(x) // 2] * 1e3
            row[f"L{level}"] = {"ms_epoch": med(tot), "ms_enqueue": med(enq),
                                "kernels_ms": eng.kernel_times() if level else {}}
        print(json.dumps(row), flush=True)
