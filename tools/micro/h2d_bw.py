"""Diagnostic: pinned host -> device copy rate, one stream vs several (the C5 batch upload's shape)."""
import time

import torch

n = 1 << 30  # 4 GiB of u32
h = torch.empty(n, dtype=torch.int32).pin_memory()
d = torch.empty(n, dtype=torch.int32, device="cuda")
for ns in (1, 2, 4):
    streams = [torch.cuda.Stream() for _ in range(ns)]
    chunk = n // ns
    for rep in range(3):
        torch.cuda.synchronize()
        t = time.perf_counter()
        for k, s in enumerate(streams):
            with torch.cuda.stream(s):
                d[k * chunk:(k + 1) * chunk].copy_(h[k * chunk:(k + 1) * chunk], non_blocking=True)
        torch.cuda.synchronize()
        dt = time.perf_counter() - t
    print(f"{ns} stream(s): {4 * n / dt / 1e9:.1f} GB/s", flush=True)
