"""Chunk-mapped device buffers (nmmo_dev_alloc / nmmo_dev_free, nmmo_amd/devmem.py) on MI355X:
buffers allocated, filled, checked and freed over and over keep their contents, with freed virtual
ranges handed out again (round 4 kept them reserved after a reused range read back other contents
under a single whole-range unmap; tools/vmm_repro.hip, the same call sequence with no build code,
found no wrong word with either unmap form: profiles/r05/vmm_repro.txt)."""

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
    assert len(seen) < 192  # freed ranges were handed out again (and read back what was written)
