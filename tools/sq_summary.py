"""Per-kernel SQ instruction summary of a rocprofv3 --pmc counter CSV (tools/ingest_pmc_traffic.sh
with IPMC_GROUPS=SQ_...): instructions per wave, cycles per wave, share of cycles waiting.

    python tools/sq_summary.py <run_counter_collection.csv> [kernel-prefix]
"""
import collections
import csv
import sys

agg = collections.defaultdict(lambda: collections.defaultdict(float))
for r in csv.DictReader(open(sys.argv[1])):
    k = r["Kernel_Name"].split("(")[0].replace("kdtn::", "")
    agg[k][r["Counter_Name"]] += float(r["Counter_Value"])
pre = sys.argv[2] if len(sys.argv) > 2 else "k_"
for k, d in agg.items():
    if not k.startswith(pre):
        continue
    w = max(d.get("SQ_WAVES", 1), 1)
    print(f"{k:22s} waves {w:10.0f} valu/w {d['SQ_INSTS_VALU'] / w:7.1f} salu/w {d['SQ_INSTS_SALU'] / w:7.1f} "
          f"vmem/w {d['SQ_INSTS_VMEM_RD'] / w:5.1f} lds/w {d['SQ_INSTS_LDS'] / w:6.1f} "
          f"cyc/w {d['SQ_WAVE_CYCLES'] / w:8.0f} wait% {100 * d['SQ_WAIT_ANY'] / max(d['SQ_WAVE_CYCLES'], 1):5.1f}")
