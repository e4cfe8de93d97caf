"""Host-to-device copy rates from page-locked memory on this box (profiling tool): one copy of
S MB on one stream, and the same bytes split over 2 / 4 streams issued together.

    python tools/h2d_probe.py
"""
import json
import time

import torch

dev = torch.device("cuda:0")
res = []
for mb in (1, 4, 16, 64, 256):
    n = mb << 20
    src = torch.empty(n, dtype=torch.uint8, pin_memory=True)
    src.fill_(1)
    dst = torch.empty(n, dtype=torch.uint8, device=dev)
    for nstreams in (1, 2, 4):
        streams = [torch.cuda.Stream() for _ in range(nstreams)]
        part = n // nstreams
        best = 1e9
        for _ in range(5):
            torch.cuda.synchronize()
            t = time.perf_counter()
            for k, s in enumerate(streams):
                with torch.cuda.stream(s):
                    dst[k * part:(k + 1) * part].copy_(src[k * part:(k + 1) * part], non_blocking=True)
            torch.cuda.synchronize()
            best = min(best, time.perf_counter() - t)
        res.append({"MB": mb, "streams": nstreams, "ms": best * 1e3, "GBps": n / best / 1e9})
        print(json.dumps(res[-1]), flush=True)
