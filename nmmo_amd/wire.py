"""Wire encoding of native observations (SPEC.md §8c): the transport form of the learner gather.

BASELINE config 5 returns every rank's observations to one learner GPU over xGMI. The native
layout (9,552 B per agent + 32 KB Market per env) is mostly padding on the wire; a wire buffer
(`nmmo_wire_pack`, csrc/wire.hip) keeps the 16-B record head, the ActionTargets as bits except
Buy.MarketItem (rebuilt from the listings), an entity-table index per visible Entity row (each
env's distinct rows travel once), the held items, the 225 window materials at 4 bits and only
the listed Market rows: ~0.3 KB per agent in the realm in C4 steady state. The receiver decodes
it back to the native layout bit-identically (`nmmo_wire_unpack`). A handle created with
obs_layout OBS_WIRE writes the same bytes straight from the state (nmmo_step / nmmo_observe into
a wire buffer), with no native buffer at all. The transfer protocol — sizes a step ahead of
their payload, then exactly the bytes the header announced — is
`nmmo_amd.distributed.WireExchange` / `WireGather`.
"""

from __future__ import annotations

import ctypes

import torch

from ._native import check, lib


def header_bytes(n_envs: int, players: int) -> int:
    return int(lib().nmmo_wire_header_bytes(n_envs, players))


def max_bytes(n_envs: int, players: int) -> int:
    return int(lib().nmmo_wire_max_bytes(n_envs, players))


def total_bytes(wire: torch.Tensor) -> int:
    """The size a packed buffer announces (its first int64). Synchronises with wire's stream."""
    return int(wire[:8].view(torch.int64).item())


def _stream(device):
    return ctypes.c_void_p(torch.cuda.current_stream(device).cuda_stream)


def pack(engine, native: torch.Tensor | None = None, out: torch.Tensor | None = None) -> torch.Tensor:
    """Encode the engine's most recent native obs (default: engine.obs) into a device uint8
    buffer of nmmo_wire_max_bytes (enqueued on the current stream)."""
    native = engine.obs if native is None else native
    cap = max_bytes(engine.n_envs, engine.P)
    out = torch.empty(cap, dtype=torch.uint8, device=engine.device) if out is None else out
    if out.numel() < cap:
        raise ValueError(f"wire buffer holds {out.numel()} B < {cap} B")
    with torch.cuda.device(engine.device):
        check(lib().nmmo_wire_pack(engine.h, ctypes.c_void_p(native.data_ptr()), ctypes.c_void_p(out.data_ptr()),
                                   _stream(engine.device)), "nmmo_wire_pack")
    return out


def unpack(wire: torch.Tensor, n_envs: int, players: int, out: torch.Tensor | None = None) -> torch.Tensor:
    """Decode a wire buffer into the native layout [n_envs, env_bytes] (enqueued)."""
    from . import abi, devmem

    if out is None:  # the learner's native obs: chunk-mapped like the engine's
        out = devmem.empty((n_envs, abi.native_env_bytes(players)), torch.uint8, wire.device)
    with torch.cuda.device(wire.device):
        check(lib().nmmo_wire_unpack(n_envs, players, ctypes.c_void_p(wire.data_ptr()),
                                     ctypes.c_void_p(out.data_ptr()), _stream(wire.device)), "nmmo_wire_unpack")
    return out


def check_buffers(bufs, players: int, status: torch.Tensor) -> torch.Tensor:
    """check_buffer over up to 16 buffers in one launch (nmmo_wire_check_many): bufs = [(wire,
    n_envs, expect_total or None)], all on status's device."""
    n = len(bufs)
    if not 1 <= n <= 16:
        raise ValueError("check_buffers takes 1..16 buffers")
    if status.dtype != torch.int32:
        raise ValueError("status must be an int32 tensor")
    for w, _, x in bufs:
        if w.device != status.device or (x is not None and (x.dtype != torch.int64 or x.device != status.device)):
            raise ValueError("wire buffers / expect_totals must be on status's device (expect_total int64)")
    wires = (ctypes.c_void_p * n)(*[w.data_ptr() for w, _, _ in bufs])
    envs = (ctypes.c_int32 * n)(*[int(ne) for _, ne, _ in bufs])
    exp = (ctypes.c_void_p * n)(*[None if x is None else x.data_ptr() for _, _, x in bufs])
    with torch.cuda.device(status.device):
        check(lib().nmmo_wire_check_many(wires, envs, exp, n, players, ctypes.c_void_p(status.data_ptr()),
                                         _stream(status.device)), "nmmo_wire_check_many")
    return status


def check_buffer(wire: torch.Tensor, n_envs: int, players: int, status: torch.Tensor,
                 expect_total: torch.Tensor | None = None) -> torch.Tensor:
    """Enqueue the consistency check of a (received) wire buffer (nmmo_wire_check): error bits
    are OR-ed into `status` (device int32 [1]; 0 = valid: 1 total != expect_total, 2 offsets, 4
    count ranges, 8 record heads, 16 entity-table indices). `expect_total`: device int64 [1] the
    sender announced."""
    if status.dtype != torch.int32 or status.device != wire.device:
        raise ValueError("status must be an int32 tensor on the wire buffer's device")
    if expect_total is not None and (expect_total.dtype != torch.int64 or expect_total.device != wire.device):
        raise ValueError("expect_total must be an int64 tensor on the wire buffer's device")
    with torch.cuda.device(wire.device):
        check(lib().nmmo_wire_check(ctypes.c_void_p(wire.data_ptr()), n_envs, players,
                                    None if expect_total is None else ctypes.c_void_p(expect_total.data_ptr()),
                                    ctypes.c_void_p(status.data_ptr()), _stream(wire.device)), "nmmo_wire_check")
    return status
