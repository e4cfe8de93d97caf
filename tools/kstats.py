"""Per-kernel summary of a rocprofv3 --stats CSV (and per-launch times of one kernel).

    python tools/kstats.py gpurun_out/<tag>/istats/run_kernel_stats.csv [kernel-substring]
"""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
for r in rows[:32]:
    print(f"{r['Name'][:60]:60s} calls={r['Calls']:>5} avg_ms={float(r['AverageNs']) / 1e6:8.3f} "
          f"tot_ms={float(r['TotalDurationNs']) / 1e6:9.2f}")
if len(sys.argv) > 2:
    tr = sys.argv[1].replace("kernel_stats", "kernel_trace")
    for r in csv.DictReader(open(tr)):
        if sys.argv[2] in r["Kernel_Name"]:
            print(sys.argv[2], (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3, "us")
