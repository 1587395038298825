"""Probe of the device->host frame copy on the GPU box (diagnostic only):
pinned D2H bandwidth, pageable D2H, and host memcpy rates for a 1080p f32
frame (24.9 MB), to size rt_render's staging path."""
import time

import numpy as np
import torch

N = 1920 * 1080 * 3 * 4


def t(f, n=10):
    f()
    torch.cuda.synchronize()
    ts = []
    for _ in range(n):
        t0 = time.perf_counter()
        f()
        torch.cuda.synchronize()
        ts.append((time.perf_counter() - t0) * 1e3)
    return float(np.median(ts))


d = torch.empty(N, dtype=torch.uint8, device="cuda")
pin = torch.empty(N, dtype=torch.uint8).pin_memory()
page = torch.empty(N, dtype=torch.uint8)
print("pinned D2H ms", t(lambda: pin.copy_(d, non_blocking=True)), "GB/s", N / t(lambda: pin.copy_(d, non_blocking=True)) / 1e6)
print("pageable D2H (torch) ms", t(lambda: page.copy_(d)))
a = np.empty(N, dtype=np.uint8)
b = np.ones(N, dtype=np.uint8)
print("host memcpy warm ms", t(lambda: np.copyto(a, b)))
print("host memcpy into fresh np.zeros ms", t(lambda: np.copyto(np.zeros(N, dtype=np.uint8), b)))
print("np.zeros + touch ms", t(lambda: np.zeros(N, dtype=np.uint8).fill(1)))
pn = pin.numpy()
print("pinned->pageable memcpy ms", t(lambda: np.copyto(a, pn)))
