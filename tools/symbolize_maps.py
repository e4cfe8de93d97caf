"""Map the PCs of a glog-style crash trace ("@ 0x... (unknown)") to library + offset using
the /proc/self/maps a process wrote at exit (tools/resident_run.py --maps).

    python tools/symbolize_maps.py <crash.log> <maps.txt>  >  symbolized.txt
"""
import re
import sys


def load_maps(path):
    maps = []
    for line in open(path):
        p = line.split()
        if len(p) < 5:
            continue
        a, b = (int(x, 16) for x in p[0].split("-"))
        maps.append((a, b, int(p[2], 16), p[5] if len(p) > 5 else "", p[1]))
    return maps


def main():
    log, mp = sys.argv[1], sys.argv[2]
    maps = load_maps(mp)
    pcs = []
    for line in open(log):
        m = re.search(r"(?:PC: |SIGSEGV \()?@\s+(0x[0-9a-f]+)", line)
        if m:
            pcs.append((int(m.group(1), 16), line.strip()))
    for pc, line in pcs:
        hit = [m for m in maps if m[0] <= pc < m[1]]
        where = f"{hit[0][3]} {hit[0][4]} +0x{pc - hit[0][0] + hit[0][2]:x}" if hit else "unmapped"
        print(f"0x{pc:x}  {where}    [{line}]")


if __name__ == "__main__":
    main()
