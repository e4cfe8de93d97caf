"""HBM traffic per k_reconcile launch from the FETCH_SIZE / WRITE_SIZE PMC passes.

    python tools/pmc_traffic.py <gpurun_out/TAG> <profiles/OUT.json> [links_per_gpu] [config] [glob]

Reads the rocprofv3 counter CSVs of tools/gpu_round.sh's `pmc` step (one pass per counter:
they cannot share a pass on gfx950) and applies MI355X_MICROARCH.md § HBM: FETCH_SIZE and
WRITE_SIZE are in KiB; on gfx950 FETCH_SIZE tallies 128-B read requests at 64 B, so it is
doubled; WRITE_SIZE is taken as is. bench.py reports the result as roofline.traffic when
the workload matches.
"""
import collections
import csv
import glob
import hashlib
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
# the sources bench.py's kernel_src_sha16() hashes: a summary is attached to a bench line only
# when it was measured on the same k_reconcile sources
KERNEL_SOURCES = ("kube-dtn_amd/csrc/kdtn_kernels.hip", "kube-dtn_amd/csrc/kdtn_kernels.h",
                  "kube-dtn_amd/csrc/kdtn_parse.h", "kube-dtn_amd/csrc/kdtn_engine.hip")


def kernel_src_sha16() -> str:
    h = hashlib.sha256()
    for p in KERNEL_SOURCES:
        with open(os.path.join(ROOT, p), "rb") as f:
            h.update(f.read())
    return h.hexdigest()[:16]


def main():
    root, dst = sys.argv[1], sys.argv[2]
    links = int(sys.argv[3]) if len(sys.argv) > 3 else 10_000_000
    config = int(sys.argv[4]) if len(sys.argv) > 4 else 2
    pat = sys.argv[5] if len(sys.argv) > 5 else "pmc*"
    vals = collections.defaultdict(list)
    for f in sorted(glob.glob(f"{root}/{pat}/**/*counter_collection.csv", recursive=True)):
        for r in csv.DictReader(open(f)):
            k = r["Kernel_Name"].split("(")[0].replace("kdtn::", "").replace("void ", "")
            vals[(k, r["Counter_Name"])].append(float(r["Counter_Value"]))
    out = {"source": root, "links_per_gpu": links, "config": config,
           "kernel_src_sha16": kernel_src_sha16(), "kernels": {}}
    for (k, c), v in sorted(vals.items()):
        if k.startswith("__amd"):
            continue
        out["kernels"].setdefault(k, {})[c + "_kib_mean"] = sum(v) / len(v)
        out["kernels"][k][c + "_n"] = len(v)
    for k, d in out["kernels"].items():
        if "FETCH_SIZE_kib_mean" in d and "WRITE_SIZE_kib_mean" in d:
            d["read_bytes"] = 2.0 * d["FETCH_SIZE_kib_mean"] * 1024.0
            d["write_bytes"] = d["WRITE_SIZE_kib_mean"] * 1024.0
            d["traffic_bytes"] = d["read_bytes"] + d["write_bytes"]
    with open(dst, "w") as f:
        json.dump(out, f, indent=1)
    rec = [k for k in out["kernels"] if k.startswith("k_reconcile")]
    for k in rec:
        print(k, json.dumps(out["kernels"][k]))


if __name__ == "__main__":
    main()
