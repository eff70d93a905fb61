"""Debug: chunk-mapped buffer reuse (devmem): allocate, fill, check, free, over and over."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from nmmo_amd import devmem  # noqa: E402

devmem.MIN_BYTES = 4 << 20
dev = torch.device("cuda", 0)
bad, seen = 0, set()
for it in range(24):
    bufs = [devmem.empty(((8 + 7 * k + it % 12) << 18,), torch.float32, dev) for k in range(4)]
    for k, b in enumerate(bufs):
        seen.add(b.data_ptr())
        b.fill_(float(it * 10 + k))
    torch.cuda.synchronize()
    for k, b in enumerate(bufs):
        if not bool((b == float(it * 10 + k)).all()):
            bad += 1
            print("iteration", it, "buffer", k, "ptr", hex(b.data_ptr()), "wrong content", flush=True)
    del bufs, b
    devmem.release_pending()
print("vmm reuse check done: bad buffers", bad, "distinct ranges", len(seen), flush=True)
