"""Diagnostic: hipMemcpyAsync H2D from registered memory on 1, 2, 4 non-blocking streams (the load's copies)."""
import ctypes
import time

import numpy as np
import torch

torch.cuda.init()
hip = ctypes.CDLL("libamdhip64.so.7")
hip.hipHostRegister.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_uint]
hip.hipMemcpyAsync.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int, ctypes.c_void_p]
hip.hipStreamCreateWithFlags.argtypes = [ctypes.POINTER(ctypes.c_void_p), ctypes.c_uint]
hip.hipStreamSynchronize.argtypes = [ctypes.c_void_p]
n = 600 << 20
d = torch.empty(n, dtype=torch.int32, device="cuda")
a = np.ones(n, np.uint32)
print("register rc", hip.hipHostRegister(a.ctypes.data, a.nbytes, 0))
streams = []
for _ in range(4):
    s = ctypes.c_void_p()
    hip.hipStreamCreateWithFlags(ctypes.byref(s), 1)
    streams.append(s)
for ns in (1, 2, 4):
    for rep in range(3):
        torch.cuda.synchronize()
        t = time.perf_counter()
        ch = n // ns
        for k in range(ns):
            hip.hipMemcpyAsync(ctypes.c_void_p(d.data_ptr() + 4 * k * ch), ctypes.c_void_p(a.ctypes.data + 4 * k * ch),
                               4 * ch, 1, streams[k])
        for k in range(ns):
            hip.hipStreamSynchronize(streams[k])
        dt = time.perf_counter() - t
    print(f"hipMemcpyAsync on {ns} stream(s): {4 * n / dt / 1e9:.1f} GB/s", flush=True)
# chunked on one stream (16 MB pieces)
for rep in range(3):
    torch.cuda.synchronize()
    t = time.perf_counter()
    ch = 4 << 20
    for k in range(0, n, ch):
        m = min(ch, n - k)
        hip.hipMemcpyAsync(ctypes.c_void_p(d.data_ptr() + 4 * k), ctypes.c_void_p(a.ctypes.data + 4 * k), 4 * m, 1,
                           streams[0])
    hip.hipStreamSynchronize(streams[0])
    dt = time.perf_counter() - t
print(f"hipMemcpyAsync 16 MB pieces, 1 stream: {4 * n / dt / 1e9:.1f} GB/s", flush=True)
