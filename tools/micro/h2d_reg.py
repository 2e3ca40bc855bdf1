"""Diagnostic: H2D rate from hipHostRegister'ed numpy memory vs hipHostMalloc'ed memory."""
import ctypes
import time

import numpy as np
import torch

torch.cuda.init()
hip = ctypes.CDLL("libamdhip64.so.7")
hip.hipHostRegister.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_uint]
hip.hipHostMalloc.argtypes = [ctypes.POINTER(ctypes.c_void_p), ctypes.c_size_t, ctypes.c_uint]
hip.hipMemcpy.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int]
n = 600 << 20  # 2.4 GB of u32
d = torch.empty(n, dtype=torch.int32, device="cuda")


def rate(src, label):
    for rep in range(3):
        torch.cuda.synchronize()
        t = time.perf_counter()
        rc = hip.hipMemcpy(ctypes.c_void_p(d.data_ptr()), ctypes.c_void_p(src), 4 * n, 1)
        torch.cuda.synchronize()
        dt = time.perf_counter() - t
    print(f"{label}: rc {rc} {4 * n / dt / 1e9:.1f} GB/s", flush=True)


a = np.ones(n, np.uint32)
print("register rc", hip.hipHostRegister(a.ctypes.data, a.nbytes, 0), "page offset", a.ctypes.data % 4096)
rate(a.ctypes.data, "hipHostRegister numpy")
p = ctypes.c_void_p()
print("hostmalloc rc", hip.hipHostMalloc(ctypes.byref(p), 4 * n, 0))
ctypes.memset(p, 1, 4 * n)
rate(p.value, "hipHostMalloc")
b = np.ones(n + 1024, np.uint32)
off = (-b.ctypes.data % 4096) // 4
b2 = b[off:off + n]
print("register aligned rc", hip.hipHostRegister(b2.ctypes.data, b2.nbytes, 0))
rate(b2.ctypes.data, "hipHostRegister numpy, 4 KiB aligned")
