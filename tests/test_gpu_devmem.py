"""Chunk-mapped device buffers (nmmo_dev_alloc / nmmo_dev_free, nmmo_amd/devmem.py) on MI355X:
buffers allocated, filled, checked and freed over and over keep their contents. Freed virtual
ranges stay reserved: a range freed with hipMemAddressFree and reserved again can alias a later
hipMalloc (torch's allocator) and read back what that wrote (tools/vmm_repro.hip, the standalone
reproducer; capi.hip nmmo_dev_free), so every allocation gets addresses never used before."""

import pytest
import torch

from tests.conftest import gpu_available

pytestmark = [pytest.mark.gpu, pytest.mark.skipif(not gpu_available(), reason="needs a GPU")]


def test_alloc_fill_free_cycles(monkeypatch):
    from nmmo_amd import devmem

    monkeypatch.setattr(devmem, "MIN_BYTES", 4 << 20)
    dev = torch.device("cuda", 0)
    seen = set()
    for it in range(48):  # tools/debug/dbg_vmm.py's cycle (4 of 48 read back wrong in round 4)
        bufs = [devmem.empty(((8 + 7 * k + it % 12) << 18,), torch.float32, dev) for k in range(4)]
        for k, b in enumerate(bufs):
            seen.add(b.data_ptr())
            b.fill_(float(it * 10 + k))
        torch.cuda.synchronize()
        for k, b in enumerate(bufs):
            assert bool((b == float(it * 10 + k)).all()), f"cycle {it} buffer {k}"
        del bufs, b
        devmem.release_pending()
    assert len(seen) == 192  # no range handed out twice
