"""Output equality of k_reconcile profiling variants against the default build (one process).

    python tools/variant_check.py --variants 66051,65539 [--config 2] [--pods N]
Loads the profiling library (make -C kube-dtn_amd prof); for each workload runs the default
variant, downloads every output array, then each listed variant and compares the arrays
bit for bit. Prints one JSON line per (workload, variant). A variant that is A/B-timed by
tools/ablate.py must pass this first.
"""
import argparse
import json
import os
import sys

import numpy as np
import torch  # noqa: F401  (one HIP runtime)

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "kube-dtn_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))
from kdtn import engine as _eng  # noqa: E402

_eng.use_profiling_library()
from kdtn import Engine, abi, synth  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--variants", required=True)
ap.add_argument("--configs", default="2,1,4:100000", help="config[:pods per shard], comma list")
ap.add_argument("--random", type=int, default=6, help="random adversarial epochs (tests/helpers)")
a = ap.parse_args()

FIELDS = ("action", "del_off", "add_off", "upd_off", "del_idx", "add_idx", "upd_idx", "del_res", "add_res",
          "upd_res", "add_qdisc", "upd_qdisc")


def outputs(eng, variant, stages):
    if variant is None:
        os.environ.pop("KDTN_VARIANT", None)
    else:
        os.environ["KDTN_VARIANT"] = str(variant)
    eng.run(stages)
    eng.sync()
    out = eng.download()
    return {f: np.asarray(getattr(out, f)).copy() for f in FIELDS}


def compare(want, got):
    bad = []
    for f in FIELDS:
        x, y = want[f], got[f]
        if x.shape != y.shape or x.tobytes() != y.tobytes():
            bad.append(f)
    return bad


def workloads():
    for spec in [x for x in a.configs.split(",") if x]:
        c, _, pods = spec.partition(":")
        kw = {"pods_per_shard": int(pods)} if pods else {}
        yield f"config{spec}", synth.make(int(c), **kw)
    if a.random:
        from helpers import random_epoch_input
        for seed in range(a.random):
            yield f"random{seed}", random_epoch_input(100 + seed, T=300 + 97 * seed)[1]


eng = Engine(device=0)
ok = True
for name, inp in workloads():
    eng.upload(inp)
    for stages in (abi.STAGE_ALL, abi.STAGE_DIFF | abi.STAGE_RESOLVE, abi.STAGE_DIFF | abi.STAGE_QDISC):
        want = outputs(eng, None, stages)
        for v in a.variants.split(","):
            bad = compare(want, outputs(eng, int(v), stages))
            ok &= not bad
            print(json.dumps({"workload": name, "stages": stages, "variant": int(v), "equal": not bad,
                              "differs": bad}), flush=True)
os.environ.pop("KDTN_VARIANT", None)
eng.close()
sys.exit(0 if ok else 1)
