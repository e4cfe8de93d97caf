"""Device-to-host copy paths on this box (profiling tool): hipMemcpyAsync D2H of S MB into
page-locked host memory allocated with hipHostMalloc default (coherent) vs non-coherent flags,
alone and while a host-to-device copy of the same size runs on another stream (the resident
pipeline's overlap). Run under `rocprofv3 --kernel-trace --memory-copy-trace` to see which
copies are DMA engine copies and which are blit kernels.

    python tools/d2h_probe.py
"""
import ctypes as C
import json
import sys
import time

if "--torch" in sys.argv:                 # the engine's process has torch's HIP runtime loaded
    import torch  # noqa: F401
    torch.zeros(1, device="cuda")
hip = C.CDLL("libamdhip64.so")
hip.hipMalloc.argtypes = [C.POINTER(C.c_void_p), C.c_size_t]
hip.hipHostMalloc.argtypes = [C.POINTER(C.c_void_p), C.c_size_t, C.c_uint]
hip.hipMemcpyAsync.argtypes = [C.c_void_p, C.c_void_p, C.c_size_t, C.c_int, C.c_void_p]
hip.hipStreamCreate.argtypes = [C.POINTER(C.c_void_p)]
hip.hipStreamSynchronize.argtypes = [C.c_void_p]
hip.hipMemset.argtypes = [C.c_void_p, C.c_int, C.c_size_t]
H2D, D2H = 1, 2
FLAGS = {"default": 0x0, "noncoherent": 0x80000000, "coherent": 0x40000000}


def chk(e):
    assert e == 0, f"hip error {e}"


def alloc_dev(n):
    p = C.c_void_p()
    chk(hip.hipMalloc(C.byref(p), n))
    chk(hip.hipMemset(p, 1, n))
    return p


def alloc_host(n, flags):
    p = C.c_void_p()
    chk(hip.hipHostMalloc(C.byref(p), n, flags))
    C.memset(p, 2, n)
    return p


hip.hipStreamCreateWithFlags.argtypes = [C.POINTER(C.c_void_p), C.c_uint]
s1, s2 = C.c_void_p(), C.c_void_p()
flags = 1 if "--nonblocking" in sys.argv else 0      # hipStreamNonBlocking, as the engine's streams
chk(hip.hipStreamCreateWithFlags(C.byref(s1), flags))
chk(hip.hipStreamCreateWithFlags(C.byref(s2), flags))
for mb in (1, 4, 16, 64):
    n = mb << 20
    d_src, d_dst = alloc_dev(n), alloc_dev(n)
    h_up = alloc_host(n, 0)
    for name, fl in FLAGS.items():
        h = alloc_host(n, fl)
        for overlap in (False, True):
            best = 1e9
            for _ in range(5):
                t = time.perf_counter()
                if overlap:
                    chk(hip.hipMemcpyAsync(d_dst, h_up, n, H2D, s2))
                chk(hip.hipMemcpyAsync(h, d_src, n, D2H, s1))
                chk(hip.hipStreamSynchronize(s1))
                t_d2h = time.perf_counter() - t
                chk(hip.hipStreamSynchronize(s2))
                best = min(best, t_d2h)
            print(json.dumps({"MB": mb, "host_flags": name, "with_h2d": overlap, "d2h_ms": best * 1e3,
                              "d2h_GBps": n / best / 1e9}), flush=True)
