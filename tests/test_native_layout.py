"""Native observation layout (SPEC.md §8b) on the CPU: a native buffer encoded from the oracle's
flat obs decodes (nmmo_amd.layout.unflatten_native) to exactly what the flat layout decodes to."""

import numpy as np

from nmmo_amd import abi, layout
from nmmo_amd.config import Config
from oracle.oracle import OracleEnvs


def encode_native(flat: np.ndarray, players: int, task_index: np.ndarray) -> np.ndarray:
    """numpy restatement of the native writer: flat float32 [n, P, elems] -> uint8 [n, env_bytes]."""
    lay = layout.flat_layout()
    n = flat.shape[0]
    out = np.zeros((n, abi.native_env_bytes(players)), np.uint8)
    rows = out[:, :players * abi.NATIVE_ROW_BYTES].reshape(n, players, abi.NATIVE_ROW_BYTES)
    nmask = lay["AgentId"].offset
    rows[:, :, :nmask] = flat[:, :, :nmask].astype(np.uint8)
    i16 = np.zeros((n, players, abi.NATIVE_I16), np.int16)
    for name, (o, shape) in layout.native_offsets().items():
        k = int(np.prod(shape))
        if name == "TaskIndex":
            i16[:, :, o] = np.where(flat[:, :, lay["AgentId"].offset] != 0, task_index, 0)
        else:
            i16[:, :, o:o + k] = flat[:, :, lay[name].offset:lay[name].offset + k].astype(np.int16)
    rows[:, :, abi.NATIVE_MASK_BYTES:] = i16.view(np.uint8).reshape(n, players, -1)
    m = lay["Market"]
    for e in range(n):  # the Market is the same for every agent in the realm: take the first
        alive = np.flatnonzero(flat[e, :, lay["AgentId"].offset])
        if len(alive):
            mk = flat[e, alive[0], m.offset:m.offset + 1024 * 16].astype(np.int16)
            out[e, players * abi.NATIVE_ROW_BYTES:] = mk.view(np.uint8)
    return out


def test_native_geometry():
    assert abi.NATIVE_ROW_BYTES == 9552 and abi.NATIVE_ROW_BYTES % 16 == 0
    offs = layout.native_offsets()
    assert offs["TaskIndex"][0] + 1 <= abi.NATIVE_I16
    n_masks = sum(size for _, size in layout.MASK_SEGMENTS)
    assert n_masks == 1586 <= abi.NATIVE_MASK_BYTES
    # ~10x fewer bytes per agent-step than pufferlib's float32 row
    per_agent = abi.native_env_bytes(128) / 128
    assert layout.obs_elems() * 4 / per_agent > 9.5


def test_unflatten_native_matches_flat():
    cfg = Config.preset("C4", MAP_N=4, early_stop_agent_num=8)
    task = (np.arange(2048) % 31 / 31.0).astype(np.float16)
    orc = OracleEnvs(cfg, 2, seed=4, task_embedding=task)
    orc.reset()
    for t in range(12):
        orc.step(orc.scripted_actions(t))
    flat = orc.obs
    nat = encode_native(flat, cfg.PLAYER_N, np.zeros((2, cfg.PLAYER_N), np.int16))
    table = task.astype(np.float32).reshape(1, -1)
    a = layout.unflatten(flat.reshape(2 * cfg.PLAYER_N, -1))
    b = layout.unflatten_native(nat, cfg.PLAYER_N, table)

    def walk(x, y, path=""):
        if isinstance(x, dict):
            assert set(x) == set(y), path
            for k in x:
                walk(x[k], y[k], path + "." + k)
        else:
            assert x.shape == y.shape, (path, x.shape, y.shape)
            assert np.array_equal(np.asarray(x, np.float32), np.asarray(y, np.float32)), path

    walk(a, b)
