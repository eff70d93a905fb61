"""Large device buffers mapped from 64-MB physical chunks (nmmo_dev_alloc), as torch tensors.

The flat observation tensor of 1,024 envs is 12.6 GB. A hipMalloc'd (or torch caching-allocator)
buffer that size lands on physical placements whose write rate under the obs kernel's store
pattern varied 5.4-6.5 TB/s from one allocation to the next on the same box, while buffers mapped
from 2-256 MB chunks wrote at 6.5-6.6 TB/s every time (tools/fill_patterns.hip). `empty` returns
such a buffer as a torch tensor (zero-copy, via __cuda_array_interface__).

Release is deferred: when the last tensor view of a buffer is gone, the buffer joins a pending
list instead of calling nmmo_dev_free from the garbage collector (which would synchronise the
device in the middle of whatever is running, and is not allowed while a stream captures a
graph); `release_pending()` frees them at a sync point — NmmoEngine.close() and every `empty()`
call it. A device without virtual memory management gets torch.empty buffers instead.
"""

from __future__ import annotations

import ctypes
import os

import torch

from ._native import NativeError, check, lib

MIN_BYTES = 256 << 20  # smaller buffers come from torch's allocator

_TYPESTR = {torch.float32: "<f4", torch.uint8: "|u1", torch.int32: "<i4", torch.int16: "<i2",
            torch.int64: "<i8"}


class DeviceBuffer:
    def __init__(self, nbytes: int, device: torch.device):
        self.device = device
        self.nbytes = int(nbytes)
        ptr = ctypes.c_void_p()
        check(lib().nmmo_dev_alloc(device.index, self.nbytes, ctypes.byref(ptr)), "nmmo_dev_alloc")
        self.ptr = ptr.value
        self.__cuda_array_interface__ = None

    def view(self, shape, dtype) -> torch.Tensor:
        self.__cuda_array_interface__ = {"shape": tuple(int(x) for x in shape), "typestr": _TYPESTR[dtype],
                                         "data": (self.ptr, False), "version": 3, "strides": None}
        with torch.cuda.device(self.device):
            t = torch.as_tensor(self, device=self.device)  # holds a reference to self
        assert t.data_ptr() == self.ptr and t.dtype == dtype
        return t

    def __del__(self):
        if self.ptr:
            _pending.append(self.ptr)  # freed by release_pending() at a sync point
            self.ptr = None


_pending: list = []
_unsupported: set = set()


def release_pending():
    """Free the chunk-mapped buffers no tensor uses any more (nmmo_dev_free synchronises the
    device): call at a sync point; a no-op while the current stream is capturing a graph."""
    if not _pending or torch.cuda.is_current_stream_capturing():
        return
    while _pending:
        check(lib().nmmo_dev_free(ctypes.c_void_p(_pending.pop())), "nmmo_dev_free")


def empty(shape, dtype=torch.float32, device=None) -> torch.Tensor:
    """torch.empty(shape, dtype) on `device`, chunk-mapped when it is at least MIN_BYTES."""
    device = torch.device("cuda", torch.cuda.current_device()) if device is None else torch.device(device)
    n = 1
    for x in shape:
        n *= int(x)
    nbytes = n * torch.empty((), dtype=dtype).element_size()
    if nbytes < MIN_BYTES or os.environ.get("NMMO_DEVMEM", "1") == "0" or device.index in _unsupported:
        return torch.empty(tuple(shape), dtype=dtype, device=device)  # NMMO_DEVMEM=0: A/B only
    release_pending()
    try:
        return DeviceBuffer(nbytes, device).view(shape, dtype)
    except NativeError as err:
        if "virtual memory management" not in str(err):
            raise
        _unsupported.add(device.index)
        return torch.empty(tuple(shape), dtype=dtype, device=device)
