import subprocess, sys
cases = [r'"\b"', r'"\n"', r'"\f"', r'"\r"', r'"a\bc"', r'"\u0008"', r'"q\u00e9\/\b\f\n\r\t\"\\"']
bad = 0
code = r'''
import sys; sys.path.insert(0, "kube-dtn_amd")
from kdtn import Engine
e = Engine(device=0, tick_in_usec=15.625)
doc = b'{"items":[{"metadata":{"name":' + sys.argv[1].encode() + b'}}]}'
info = e.ingest(doc); t = e.ingest_tables(); print("ok", t.kdict.get(int(t.topos.name[0])), flush=True)
'''
for c in cases:
    try:
        r = subprocess.run([sys.executable, "-c", code, c], capture_output=True, text=True, timeout=40)
        print(c, r.stdout.strip()[-80:], r.returncode, r.stderr.strip()[-300:] if r.returncode else "", flush=True)
        bad |= r.returncode != 0
    except subprocess.TimeoutExpired:
        print(c, "HANG", flush=True)
        sys.exit(2)
sys.exit(1 if bad else 0)
