"""Ingest ablation (profiling only): time kdtn_json_ingest on config 2 under KDTN_JS_VARIANT
bits (1 coherent slot loads, 2 no duplicate-check atomics, 4 no first-occurrence atomics,
8 no interning, 16 no inline bytes in the intern slots). Variants 2/4/8 produce wrong tables
and are never used otherwise; 0/1/16 produce the same tables.
Usage: ingest_ablate.py [pods] [variant,variant,...] — the variants run interleaved, 5 rounds."""
import json, os, sys
import torch  # noqa: F401
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "kube-dtn_amd"))
from kdtn import engine as _kdtn_engine  # noqa: E402
_kdtn_engine.use_profiling_library()   # A/B variants live in the profiling build
from kdtn import Engine, synth
pods = int(sys.argv[1]) if len(sys.argv) > 1 else 1_000_000
variants = [int(v, 0) for v in (sys.argv[2] if len(sys.argv) > 2 else "0,16").split(",")]
inp = synth.make(2, pods_per_shard=pods)
doc = synth.topology_list_json(inp)
eng = Engine(device=0)
eng.json_upload(doc)
acc = {v: {} for v in variants}
ROUNDS = 5
for r in range(ROUNDS + 1):
    for v in variants:
        os.environ["KDTN_JS_VARIANT"] = str(v)
        eng.json_ingest()
        if r == 0:
            continue                                  # warm-up round (tables sized)
        for k, x in eng.kernel_times().items():
            acc[v][k] = acc[v].get(k, 0.0) + x / ROUNDS
    print(f"round {r}", file=sys.stderr, flush=True)
for v in variants:
    tot = sum(x for k, x in acc[v].items() if k != "js_sync")
    print(json.dumps({"variant": v, "gpu_ms": round(tot, 3), **{k: round(x, 3) for k, x in acc[v].items()}}), flush=True)
