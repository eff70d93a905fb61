"""Debug: chunk-mapped buffer lifetime (devmem) — do live tensors keep their DeviceBuffer?"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from nmmo_amd import devmem  # noqa: E402

devmem.MIN_BYTES = 4 << 20
dev = torch.device("cuda", 0)
for it in range(6):
    bufs = []
    for k in range(4):
        bufs.append(devmem.empty(((8 + 7 * k + it) << 18,), torch.float32, dev))
        print(it, k, hex(bufs[-1].data_ptr()), "pending", len(devmem._pending), flush=True)
    ptrs = [b.data_ptr() for b in bufs]
    print("distinct", len(set(ptrs)) == len(ptrs), flush=True)
    del bufs
    devmem.release_pending()
