"""One process of CR-ingest work for profiling: a config-2 TopologyList document (cached as
a file between runs) uploaded once and decoded --reps times by kdtn_json_ingest.

    python tools/ingest_run.py [--pods N] [--reps R] [--doc /tmp/kdtn_doc.json]
"""
import argparse
import os
import sys

import torch  # noqa: F401  (one HIP runtime)

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "kube-dtn_amd"))
from kdtn import Engine, synth  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--pods", type=int, default=200_000)
ap.add_argument("--reps", type=int, default=2)
ap.add_argument("--doc", default="/tmp/kdtn_doc.json")
a = ap.parse_args()
if os.path.exists(a.doc):
    with open(a.doc, "rb") as f:
        doc = f.read()
else:
    doc = synth.topology_list_json(synth.make(2, pods_per_shard=a.pods))
    with open(a.doc, "wb") as f:
        f.write(doc)
eng = Engine(device=0)
eng.json_upload(doc)
for _ in range(a.reps):
    info = eng.json_ingest()
print({k: round(v, 3) for k, v in eng.kernel_times().items()}, info.n_tokens, flush=True)
