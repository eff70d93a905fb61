"""Loader for libnmmo_hip.so (the HIP path). Fails loudly: there is no CPU fallback.

torch is imported first so that the library's libamdhip64.so.7 dependency binds to the HIP
runtime torch already loaded (one runtime per process: device pointers from the torch caching
allocator and streams from torch.cuda are then valid inside the library).
"""

from __future__ import annotations

import ctypes
import os

from . import abi

_PKG = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get(
    "NMMO_LIB", os.path.join(os.path.dirname(os.path.abspath(__file__)), "lib", "libnmmo_hip.so"))
_lib = None

SYMBOLS = [
    "nmmo_default_config", "nmmo_layout", "nmmo_create", "nmmo_destroy", "nmmo_reset",
    "nmmo_step", "nmmo_scripted_actions", "nmmo_get_state", "nmmo_set_state",
    "nmmo_get_map_bank", "nmmo_set_map_bank", "nmmo_set_timing", "nmmo_read_timing", "nmmo_get_fault", "nmmo_set_counters", "nmmo_get_events", "nmmo_set_tasks",
    "nmmo_set_wrapper", "nmmo_get_wrapper_state", "nmmo_expand_obs", "nmmo_exp_scratch_ints",
    "nmmo_exp_store", "nmmo_exp_sort", "nmmo_exp_gae", "nmmo_gather_rows", "nmmo_n_envs",
    "nmmo_last_error", "nmmo_abi_version", "nmmo_end_episodes", "nmmo_build_info",
    "nmmo_get_wrapper_dropped", "nmmo_set_task_weights", "nmmo_wire_header_bytes", "nmmo_wire_max_bytes",
    "nmmo_wire_pack", "nmmo_wire_unpack", "nmmo_wire_check", "nmmo_dev_alloc", "nmmo_dev_free", "nmmo_observe",
    "nmmo_step_envs", "nmmo_inject_fault", "nmmo_fault_into", "nmmo_exp_store_records",
    "nmmo_exp_gather_records", "nmmo_exp_store_records_many", "nmmo_obs_invalidate", "nmmo_set_obs_counter",
    "nmmo_obs_bind", "nmmo_obs_invalidate_envs", "nmmo_exp_scratch_ints_many", "nmmo_set_step_records",
    "nmmo_wire_check_many", "nmmo_exp_store_records_checked", "nmmo_sizes_row",
    "nmmo_obs_invalidate_sections", "nmmo_p2p_load", "nmmo_p2p_unique_id", "nmmo_p2p_init", "nmmo_p2p_group",
    "nmmo_p2p_destroy",
]


class NativeError(RuntimeError):
    pass


def lib():
    global _lib
    if _lib is not None:
        return _lib
    import torch  # noqa: F401  (bind the HIP runtime torch ships, see module docstring)

    if not os.path.exists(LIB_PATH):
        raise NativeError(
            f"{LIB_PATH} is missing: build it with `python -c 'import __graft_entry__ as g; g.build()'`"
            " (there is no CPU fallback for the HIP stepper)")
    L = declare(ctypes.CDLL(LIB_PATH))
    if L.nmmo_abi_version() != abi.ABI_VERSION:
        raise NativeError(f"ABI mismatch: lib {L.nmmo_abi_version()} != python {abi.ABI_VERSION}")
    info = build_info(L)
    if os.environ.get("NMMO_ALLOW_STALE") != "1" and os.path.isdir(os.path.join(_PKG, "csrc")):
        from .build import source_hash

        want = source_hash()
        if info.get("src") != want:
            raise NativeError(
                f"{LIB_PATH} was built from other sources (src={info.get('src')}, tree={want}): "
                "rebuild it (`python -m nmmo_amd.build --force`)")
    _lib = L
    return L


def declare(L):
    """The ctypes signatures of include/nmmo_hip.h on a loaded library (this package's
    libnmmo_hip.so, or any library exporting the same C-ABI)."""
    vp, i32, u64, sz = ctypes.c_void_p, ctypes.c_int32, ctypes.c_uint64, ctypes.c_size_t
    cfgp = ctypes.POINTER(abi.NmmoConfig)
    L.nmmo_default_config.argtypes = [cfgp]
    L.nmmo_default_config.restype = None
    L.nmmo_layout.argtypes = [cfgp, ctypes.POINTER(abi.NmmoLayout)]
    L.nmmo_create.argtypes = [cfgp, i32, u64, i32, vp, ctypes.POINTER(vp)]
    L.nmmo_destroy.argtypes = [vp]
    L.nmmo_destroy.restype = None
    L.nmmo_reset.argtypes = [vp, vp, vp, vp, vp]
    L.nmmo_step.argtypes = [vp, vp, vp, vp, vp, vp, vp, vp]
    L.nmmo_step_envs.argtypes = [vp, vp, i32, vp, vp, vp, vp, vp, vp, vp]
    L.nmmo_inject_fault.argtypes = [vp, i32]
    L.nmmo_fault_into.argtypes = [vp, vp, vp]
    L.nmmo_scripted_actions.argtypes = [vp, u64, vp, vp]
    L.nmmo_get_state.argtypes = [vp, vp, sz]
    L.nmmo_set_state.argtypes = [vp, vp, sz]
    L.nmmo_get_map_bank.argtypes = [vp, vp, sz]
    L.nmmo_set_map_bank.argtypes = [vp, vp, sz]
    L.nmmo_set_timing.argtypes = [vp, i32]
    L.nmmo_get_fault.argtypes = [vp, ctypes.POINTER(i32)]
    L.nmmo_read_timing.argtypes = [vp, ctypes.POINTER(ctypes.c_double), ctypes.POINTER(i32)]
    L.nmmo_set_counters.argtypes = [vp, vp]
    L.nmmo_get_events.argtypes = [vp, i32, vp, i32, ctypes.POINTER(i32)]
    L.nmmo_set_tasks.argtypes = [vp, vp, i32, vp, vp]
    L.nmmo_set_task_weights.argtypes = [vp, vp, i32]
    L.nmmo_set_wrapper.argtypes = [vp, ctypes.POINTER(abi.NmmoWrapperConfig), vp]
    L.nmmo_get_wrapper_state.argtypes = [vp, vp, vp]
    L.nmmo_expand_obs.argtypes = [vp, vp, vp, i32, vp]
    L.nmmo_observe.argtypes = [vp, vp, vp]
    L.nmmo_obs_invalidate.argtypes = [vp, vp]
    L.nmmo_obs_bind.argtypes = [vp, vp]
    L.nmmo_obs_invalidate_envs.argtypes = [vp, vp, i32, vp]
    L.nmmo_obs_invalidate_sections.argtypes = [vp, vp, i32, ctypes.c_uint32, vp]
    L.nmmo_set_obs_counter.argtypes = [vp, vp]
    L.nmmo_set_step_records.argtypes = [vp, vp, vp]
    xp = ctypes.POINTER(abi.NmmoExperience)
    L.nmmo_exp_scratch_ints.argtypes = [i32, i32]
    L.nmmo_exp_scratch_ints.restype = ctypes.c_int64
    L.nmmo_exp_scratch_ints_many.argtypes = [i32, i32, i32]
    L.nmmo_exp_scratch_ints_many.restype = ctypes.c_int64
    L.nmmo_exp_store.argtypes = [vp, xp, ctypes.POINTER(abi.NmmoStoreInput), vp, vp]
    L.nmmo_exp_sort.argtypes = [xp, vp, vp, vp]
    rsp = ctypes.POINTER(abi.NmmoRecordStore)
    L.nmmo_exp_store_records.argtypes = [vp, xp, rsp, ctypes.POINTER(abi.NmmoStoreInput), vp, vp]
    L.nmmo_exp_gather_records.argtypes = [vp, xp, rsp, vp, i32, vp, vp]
    L.nmmo_exp_store_records_many.argtypes = [vp, xp, rsp, ctypes.POINTER(abi.NmmoStoreInput), i32, i32, vp, vp]
    L.nmmo_exp_store_records_checked.argtypes = [vp, xp, rsp, ctypes.POINTER(abi.NmmoStoreInput), i32, i32, vp,
                                                 ctypes.c_uint32, vp, vp, vp, vp]
    L.nmmo_exp_gae.argtypes = [xp, vp, i32, ctypes.c_double, ctypes.c_double, vp, vp]
    L.nmmo_gather_rows.argtypes = [vp, ctypes.c_int64, vp, i32, vp, vp]
    L.nmmo_n_envs.argtypes = [vp]
    L.nmmo_last_error.restype = ctypes.c_char_p
    L.nmmo_abi_version.restype = i32
    L.nmmo_end_episodes.argtypes = [vp, vp, vp]
    L.nmmo_get_wrapper_dropped.argtypes = [vp, ctypes.POINTER(ctypes.c_int64)]
    L.nmmo_wire_header_bytes.argtypes = [i32, i32]
    L.nmmo_wire_header_bytes.restype = ctypes.c_int64
    L.nmmo_wire_max_bytes.argtypes = [i32, i32]
    L.nmmo_wire_max_bytes.restype = ctypes.c_int64
    L.nmmo_wire_pack.argtypes = [vp, vp, vp, vp]
    L.nmmo_wire_unpack.argtypes = [i32, i32, vp, vp, vp]
    L.nmmo_wire_check.argtypes = [vp, i32, i32, vp, vp, vp]
    L.nmmo_wire_check_many.argtypes = [vp, vp, vp, i32, i32, vp, vp]
    L.nmmo_sizes_row.argtypes = [vp, i32, vp, vp, vp]
    L.nmmo_p2p_load.argtypes = [ctypes.c_char_p]
    L.nmmo_p2p_unique_id.argtypes = [vp]
    L.nmmo_p2p_init.argtypes = [vp, i32, i32, ctypes.POINTER(vp)]
    L.nmmo_p2p_group.argtypes = [vp, ctypes.POINTER(abi.NmmoP2POp), i32, vp]
    L.nmmo_p2p_destroy.argtypes = [vp]
    L.nmmo_dev_alloc.argtypes = [i32, u64, ctypes.POINTER(vp)]
    L.nmmo_dev_free.argtypes = [vp]
    L.nmmo_build_info.restype = ctypes.c_char_p
    return L


def build_info(L=None) -> dict:
    """nmmo_build_info() as a dict (src = source hash the library was compiled from)."""
    L = lib() if L is None else L
    return dict(kv.split("=", 1) for kv in L.nmmo_build_info().decode().split() if "=" in kv)


def check(rc: int, what: str):
    if rc != abi.NMMO_OK:
        raise NativeError(f"{what} failed ({rc}): {lib().nmmo_last_error().decode()}")


def layout(cfg: abi.NmmoConfig) -> abi.NmmoLayout:
    out = abi.NmmoLayout()
    check(lib().nmmo_layout(ctypes.byref(cfg), ctypes.byref(out)), "nmmo_layout")
    return out
