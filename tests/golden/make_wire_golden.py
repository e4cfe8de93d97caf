"""Generates tests/golden/wire.json: the proto.Marshal bytes of every LinksBatchQuery
that Reconcile sends for the sample transitions of samples.json (DelLinks | AddLinks |
UpdateLinks per topology, in the engine's del | add | upd region order), produced by the
Python protobuf runtime (tests/wire_pb.py) from batches computed by the oracle's CalcDiff.

    python tests/golden/make_wire_golden.py
"""
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path[:0] = [os.path.join(ROOT, "kube-dtn_amd"), os.path.join(ROOT, "oracle"), os.path.dirname(HERE)]

import oracle as O  # noqa: E402
import wire_pb  # noqa: E402
from helpers import golden_epoch  # noqa: E402
from kdtn.model import pack  # noqa: E402


def main():
    with open(os.path.join(HERE, "samples.json")) as f:
        golden = json.load(f)
    res = {}
    for tr in golden["transitions"]:
        inp = pack(golden_epoch(golden, tr))
        out = O.reconcile(inp)
        per = wire_pb.epoch_bytes(inp, out)
        T = inp.topos.n
        res[tr["name"]] = {
            "batches": [("" if per[(i // T, i % T)] is None else per[(i // T, i % T)].hex())
                        for i in range(3 * T)],
            "err": [sum(1 << l for l in range(3) if per[(l, t)] is None) for t in range(T)],
        }
    with open(os.path.join(HERE, "wire.json"), "w") as f:
        json.dump(res, f, indent=1)
    print("wrote", sum(len(v["batches"]) for v in res.values()), "batches")


if __name__ == "__main__":
    main()
