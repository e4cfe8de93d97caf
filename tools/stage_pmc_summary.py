import csv, glob, collections, sys
root = sys.argv[1]
agg = collections.defaultdict(lambda: collections.defaultdict(list))
dur = collections.defaultdict(list)
for f in glob.glob(f"{root}/pmc*/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"].split("(")[0].replace("kdtn::", "").replace("void ", "")
        agg[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
for f in glob.glob(f"{root}/pmc1/**/*kernel_trace.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"].split("(")[0].replace("kdtn::", "").replace("void ", "")
        dur[k].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
def m(d, c):
    v = d.get(c); return sum(v) / len(v) if v else float('nan')
print(f"{'kernel':34s} {'n':>3s} {'us':>8s} {'fetchMB':>8s} {'writeMB':>8s} {'L2hit':>6s} {'TAbusy':>6s} {'valu/w':>7s} {'salu/w':>7s} {'vmr/w':>6s} {'vmw/w':>6s} {'lds/w':>6s} {'wait%':>6s} {'waves':>8s}")
for k in sorted(dur, key=lambda x: -sum(dur[x]) / len(dur[x])):
    d = agg[k]; us = sum(dur[k]) / len(dur[k])
    if us < 5: continue
    w = m(d, "SQ_WAVES")
    hit = m(d, "TCC_HIT_sum"); miss = m(d, "TCC_MISS_sum")
    ta = m(d, "TA_TA_BUSY_sum"); gui = m(d, "GRBM_GUI_ACTIVE")
    print(f"{k[:34]:34s} {len(dur[k]):3d} {us:8.1f} {2*m(d,'FETCH_SIZE')/1024:8.1f} {m(d,'WRITE_SIZE')/1024:8.1f} {hit/(hit+miss):6.2f} {ta/ (gui*256/8) if gui else 0:6.2f} {m(d,'SQ_INSTS_VALU')/w:7.0f} {m(d,'SQ_INSTS_SALU')/w:7.0f} {m(d,'SQ_INSTS_VMEM_RD')/w:6.1f} {m(d,'SQ_INSTS_VMEM_WR')/w:6.1f} {m(d,'SQ_INSTS_LDS')/w:6.1f} {100*m(d,'SQ_WAIT_ANY')/max(m(d,'SQ_WAVE_CYCLES'),1):6.1f} {w:8.0f}")
