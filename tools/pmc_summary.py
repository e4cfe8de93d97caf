"""Summarise tools/pmc_profile.sh output: mean counter value per kernel and counter."""
import collections
import csv
import glob
import sys

root = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/pmc"
agg = collections.defaultdict(list)
for f in sorted(glob.glob(f"{root}/*/**/*counter_collection.csv", recursive=True)):
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"].split("(")[0].replace("kdtn::", "")
        agg[(k, r["Counter_Name"])].append(float(r["Counter_Value"]))
for (k, c), v in sorted(agg.items()):
    if k.startswith("__amd"):
        continue
    print(f"{k:28s} {c:36s} {sum(v) / len(v):14.6g}   (n={len(v)})")
