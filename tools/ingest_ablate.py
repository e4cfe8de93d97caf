"""Ingest ablation (profiling only): time kdtn_json_ingest on config 2 under KDTN_JS_VARIANT
bits (1 coherent slot loads, 2 no duplicate-check atomics, 4 no first-occurrence atomics,
8 no interning). Variants other than 0/1 produce wrong tables and are never used otherwise."""
import json, os, sys, time
import torch  # noqa: F401
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "kube-dtn_amd"))
from kdtn import engine as _kdtn_engine  # noqa: E402
_kdtn_engine.use_profiling_library()   # A/B variants live in the profiling build
from kdtn import Engine, synth
inp = synth.make(2, pods_per_shard=int(sys.argv[1]) if len(sys.argv) > 1 else 1_000_000)
doc = synth.topology_list_json(inp)
eng = Engine(device=0)
eng.json_upload(doc)
for v in (0, 1, 2, 4, 6, 8, 14):
    os.environ["KDTN_JS_VARIANT"] = str(v)
    eng.json_ingest()
    acc = {}
    for _ in range(3):
        eng.json_ingest()
        for k, x in eng.kernel_times().items():
            acc[k] = acc.get(k, 0.0) + x / 3
    print(json.dumps({"variant": v, **{k: round(x, 3) for k, x in acc.items()}}), flush=True)
