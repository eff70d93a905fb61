"""Practical HBM write ceiling on this GPU: time a 12.8 GB device fill (torch zero_/fill_, the
vendor vectorized kernels) -- the same byte count one C4 obs launch writes."""
import time

import torch

n = 12_813_205_504 // 4
x = torch.empty(n, dtype=torch.float32, device="cuda")
for fn, name in ((lambda: x.zero_(), "zero_"), (lambda: x.fill_(1.0), "fill_")):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    k = 20
    for _ in range(k):
        fn()
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / k
    print(f"{name}: {dt * 1e3:.3f} ms  {x.numel() * 4 / dt / 1e12:.2f} TB/s")
