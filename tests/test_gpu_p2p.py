"""The learner gather's native point-to-point posting (nmmo_p2p_*, csrc/p2p.hip) on one GPU: the
library's own RCCL communicator (world size 1; RCCL allows a rank to send to itself inside a
group) moves several buffers of different sizes in one group on the caller's stream, byte-exact,
and posting a 32-op group costs a few microseconds of host time per op (torch.distributed's
batch_isend_irecv: ~13.5 us per op on the GPU box, tools/debug/p2p_host_cost.py). The multi-rank
wiring of the same calls (nmmo_amd.distributed.WireExchange._p2p) is the gather protocol tested
over gloo (tests/test_wire_oracle.py, tests/test_gpu_multirank.py)."""

import ctypes
import time

import pytest

from tests.conftest import gpu_available

pytestmark = [pytest.mark.gpu, pytest.mark.skipif(not gpu_available(), reason="needs a GPU")]


def test_native_group_moves_every_buffer():
    import torch

    from nmmo_amd import abi
    from nmmo_amd._native import check, lib
    from nmmo_amd.distributed import native_comm

    dev = torch.device("cuda", 0)
    comm = native_comm(1, 0, dev)
    stream = torch.cuda.Stream(device=dev)
    g = torch.Generator(device="cpu").manual_seed(3)
    sizes = [1, 16, 4096, 1 << 20, 3 << 20]
    src = [torch.randint(0, 256, (n,), dtype=torch.uint8, generator=g).to(dev) for n in sizes]
    dst = [torch.zeros(n, dtype=torch.uint8, device=dev) for n in sizes]
    ops = [abi.NmmoP2POp(t.data_ptr(), t.numel(), 0, 0) for t in src] + \
          [abi.NmmoP2POp(t.data_ptr(), t.numel(), 0, 1) for t in dst]
    arr = (abi.NmmoP2POp * len(ops))(*ops)
    torch.cuda.synchronize()
    check(lib().nmmo_p2p_group(comm, arr, len(ops), ctypes.c_void_p(stream.cuda_stream)), "nmmo_p2p_group")
    stream.synchronize()
    for a, b in zip(src, dst):
        assert torch.equal(a, b)
    # host cost of a 32-op group (16 sends + 16 receives of 64 KB)
    bufs = [torch.zeros(1 << 16, dtype=torch.uint8, device=dev) for _ in range(32)]
    ops = [abi.NmmoP2POp(bufs[k].data_ptr(), 1 << 16, 0, k >= 16) for k in range(32)]
    arr = (abi.NmmoP2POp * 32)(*ops)
    for _ in range(3):
        check(lib().nmmo_p2p_group(comm, arr, 32, ctypes.c_void_p(stream.cuda_stream)), "nmmo_p2p_group")
    stream.synchronize()
    reps = 50
    t0 = time.perf_counter()
    for _ in range(reps):
        lib().nmmo_p2p_group(comm, arr, 32, ctypes.c_void_p(stream.cuda_stream))
    host_us = (time.perf_counter() - t0) / reps * 1e6
    stream.synchronize()
    print(f"nmmo_p2p_group: {host_us:.1f} us of host time per 32-op group ({host_us / 32:.2f} us per op)")
    assert host_us / 32 < 8.0, host_us
    # a bad op is refused before anything is posted
    bad = (abi.NmmoP2POp * 1)(abi.NmmoP2POp(None, 16, 0, 0))
    assert lib().nmmo_p2p_group(comm, bad, 1, ctypes.c_void_p(stream.cuda_stream)) != 0
