"""TEST INFRASTRUCTURE ONLY — ctypes wrapper of the CPU oracle (oracle/nmmo_oracle.c).

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import this module.
Parity vs the real nmmo 2.1 is UNPINNED (see nmmo_oracle.c header and SPEC.md).
"""

from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

from nmmo_amd import abi

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, "build", "libnmmo_oracle.so")
_lib = None


def build(force: bool = False) -> str:
    if force or not os.path.exists(LIB_PATH):
        subprocess.check_call(["make", "-s", "-C", _HERE])
    return LIB_PATH


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            build()
        L = ctypes.CDLL(LIB_PATH)
        vp, i32, u64, sz = ctypes.c_void_p, ctypes.c_int, ctypes.c_uint64, ctypes.c_size_t
        L.oracle_create.restype = vp
        L.oracle_create.argtypes = [ctypes.POINTER(abi.NmmoConfig), i32, u64, vp]
        L.oracle_destroy.argtypes = [vp]
        L.oracle_reset.argtypes = [vp, vp, vp, vp]
        L.oracle_step.argtypes = [vp, vp, vp, vp, vp, vp, vp]
        L.oracle_step_range.argtypes = [vp, i32, i32, vp, vp, vp, vp, vp, vp]
        L.oracle_scripted_actions.argtypes = [vp, u64, vp]
        L.oracle_scripted_actions_range.argtypes = [vp, i32, i32, u64, vp]
        L.oracle_get_state.argtypes = [vp, vp, sz]
        L.oracle_set_state.argtypes = [vp, vp, sz]
        L.oracle_get_map_bank.argtypes = [vp, vp, sz]
        L.oracle_set_map_bank.argtypes = [vp, vp, sz]
        L.oracle_end_episodes.argtypes = [vp, vp]
        L.oracle_set_task_weights.argtypes = [vp, vp, i32]
        L.oracle_write_obs.argtypes = [vp, i32, vp]
        L.oracle_get_events.argtypes = [vp, i32, vp, i32, ctypes.POINTER(i32)]
        L.oracle_set_tasks.argtypes = [vp, vp, i32, vp, vp]
        L.oracle_obs_elems.argtypes = [i32]
        L.oracle_flat_offsets.argtypes = [i32, vp]
        L.oracle_state_bytes_per_env.restype = sz
        L.oracle_state_bytes_per_env.argtypes = [i32, i32]
        _lib = L
    return _lib


def _p(a):
    return None if a is None else a.ctypes.data_as(ctypes.c_void_p)


class OracleEnvs:
    """n_envs independent envs stepped serially on the host, same API shape as the HIP engine."""

    def __init__(self, config, n_envs: int, seed: int, task_embedding=None, env_index_base=0):
        self.config = config
        self.cfg = config.to_c(env_index_base)
        self.n_envs = n_envs
        self.P = config.PLAYER_N
        self.S = config.PLAYER_N + (config.NPC_N if "NPC" in config.systems else 0)
        self.obs_elems = lib().oracle_obs_elems(config.TASK_EMBED_DIM)
        self._task = None
        if task_embedding is not None:
            self._task = np.ascontiguousarray(np.asarray(task_embedding, dtype=np.float16)).view(np.uint16)
        self.h = lib().oracle_create(ctypes.byref(self.cfg), n_envs, seed, _p(self._task))
        if not self.h:
            raise ValueError("oracle_create failed")
        with_obs = config.obs_layout == abi.OBS_FLAT
        self.obs = np.zeros((n_envs, self.P, self.obs_elems), np.float32) if with_obs else None
        self.rew = np.zeros((n_envs, self.P), np.float32)
        self.term = np.zeros((n_envs, self.P), np.uint8)
        self.trunc = np.zeros((n_envs, self.P), np.uint8)
        self.mask = np.zeros((n_envs, self.P), np.uint8)

    def __del__(self):
        if getattr(self, "h", None):
            lib().oracle_destroy(self.h)
            self.h = None

    def reset(self, env_seeds=None):
        seeds = None if env_seeds is None else np.ascontiguousarray(env_seeds, dtype=np.uint64)
        lib().oracle_reset(self.h, _p(seeds), _p(self.obs), _p(self.mask))

    def step(self, actions):
        actions = np.ascontiguousarray(actions, dtype=np.int32)
        assert actions.shape == (self.n_envs, self.P, abi.N_ACTION_HEADS)
        lib().oracle_step(self.h, _p(actions), _p(self.obs), _p(self.rew), _p(self.term),
                          _p(self.trunc), _p(self.mask))

    def end_episodes(self, env_mask):
        m = np.ascontiguousarray(env_mask, dtype=np.uint8)
        assert m.shape == (self.n_envs,)
        lib().oracle_end_episodes(self.h, _p(m))

    def flat_obs(self, env: int) -> np.ndarray:
        """Flat obs [P, obs_elems] of one env from its current state (any obs layout config)."""
        out = np.zeros((self.P, self.obs_elems), np.float32)
        rc = lib().oracle_write_obs(self.h, env, _p(out))
        assert rc == 0, rc
        return out

    def step_range(self, lo, hi, actions):
        lib().oracle_step_range(self.h, lo, hi, _p(actions), _p(self.obs), _p(self.rew),
                                _p(self.term), _p(self.trunc), _p(self.mask))

    def scripted_actions(self, policy_seed: int, out=None):
        out = np.zeros((self.n_envs, self.P, abi.N_ACTION_HEADS), np.int32) if out is None else out
        lib().oracle_scripted_actions(self.h, policy_seed, _p(out))
        return out

    def get_state(self) -> np.ndarray:
        n = lib().oracle_state_bytes_per_env(self.S, self.P) * self.n_envs
        buf = np.zeros(n, np.uint8)
        rc = lib().oracle_get_state(self.h, _p(buf), n)
        assert rc == 0, rc
        return buf

    def set_state(self, buf: np.ndarray):
        buf = np.ascontiguousarray(buf, dtype=np.uint8)
        rc = lib().oracle_set_state(self.h, _p(buf), buf.nbytes)
        assert rc == 0, rc

    def set_tasks(self, tasks, embeddings=None, assign=None):
        """tasks: sequence of abi.NmmoTask; embeddings fp16 [n_tasks, dim] or None;
        assign int32 [n_envs, P] or None (SPEC §12, as nmmo_set_tasks)."""
        arr = (abi.NmmoTask * len(tasks))(*tasks)
        emb = None if embeddings is None else np.ascontiguousarray(embeddings, np.float16)
        asg = None if assign is None else np.ascontiguousarray(assign, np.int32)
        rc = lib().oracle_set_tasks(self.h, ctypes.cast(arr, ctypes.c_void_p), len(tasks),
                                    None if emb is None else emb.ctypes.data_as(ctypes.c_void_p), _p(asg))
        assert rc == 0, rc

    def set_task_weights(self, weights):
        """as nmmo_set_task_weights (SPEC §12); None = fixed assignment."""
        w = None if weights is None else np.ascontiguousarray(weights, np.float64)
        rc = lib().oracle_set_task_weights(self.h, _p(w), 0 if w is None else len(w))
        if rc != 0:
            raise ValueError(f"oracle_set_task_weights failed ({rc})")

    def set_curriculum(self, specs, sample=True, assign=None):
        """A list of nmmo_amd.tasks.TaskSpec, as NmmoEngine.set_curriculum."""
        emb = None
        if all(s.embedding is not None for s in specs):
            emb = np.stack([np.asarray(s.embedding, np.float16) for s in specs])
        self.set_tasks([s.program() for s in specs], emb, assign)
        if sample:
            self.set_task_weights([float(s.sampling_weight) for s in specs])

    def events(self, env: int, max_rows: int = 1 << 20) -> np.ndarray:
        """Retained event-log rows of `env`, oldest first: int32 [n, 9] (SPEC §11)."""
        cap = max(self.config.event_cap, 1)
        buf = np.zeros((min(max_rows, cap), abi.EVENT_COLS), np.int32)
        n = ctypes.c_int()
        rc = lib().oracle_get_events(self.h, env, _p(buf), buf.shape[0], ctypes.byref(n))
        assert rc == 0, rc
        return buf[:n.value].copy()

    def map_bank(self) -> np.ndarray:
        buf = np.zeros((self.config.MAP_N, abi.MAP_SIZE, abi.MAP_SIZE), np.uint8)
        rc = lib().oracle_get_map_bank(self.h, _p(buf), buf.nbytes)
        assert rc == 0, rc
        return buf

    def set_map_bank(self, bank: np.ndarray):
        buf = np.ascontiguousarray(bank, dtype=np.uint8)
        rc = lib().oracle_set_map_bank(self.h, _p(buf), buf.nbytes)
        if rc != 0:
            raise ValueError(f"oracle_set_map_bank failed ({rc})")


def split_state(buf: np.ndarray, n_envs: int, slots: int, players: int = 128) -> dict:
    """View a state blob as named arrays (env [n,NE] i32, ent [n,NF,S] i16, ring, mat,
    items [n,P,12,2] u32, iring [n,12P] i16, tasks [n,P] i32, tstate [n,P] NmmoTaskState)."""
    per = abi.state_bytes_per_env(slots, players)
    b = buf.reshape(n_envs, per)
    o = 0
    env = b[:, o:o + abi.NE * 4].copy().view(np.int32); o += abi.NE * 4
    ent = b[:, o:o + abi.NF * slots * 2].copy().view(np.int16).reshape(n_envs, abi.NF, slots)
    o += abi.NF * slots * 2
    ring = b[:, o:o + slots * 2].copy().view(np.int16); o += slots * 2
    mat = b[:, o:o + abi.MAP_TILES].reshape(n_envs, abi.MAP_SIZE, abi.MAP_SIZE); o += abi.MAP_TILES
    ni = players * abi.INV_SLOTS
    items = b[:, o:o + ni * 8].copy().view(np.uint32).reshape(n_envs, players, abi.INV_SLOTS, 2)
    o += ni * 8
    iring = b[:, o:o + ni * 2].copy().view(np.int16)
    o += ni * 2
    tasks = b[:, o:o + players * 4].copy().view(np.int32)
    o += players * 4
    tstate = b[:, o:o + players * abi.TASK_STATE_BYTES].copy().view(abi.task_state_dtype())
    return {"env": env, "ent": ent, "ring": ring, "mat": mat, "items": items, "iring": iring,
            "tasks": tasks, "tstate": tstate}


def join_state(d: dict) -> np.ndarray:
    """Inverse of split_state."""
    n = d["env"].shape[0]
    parts = []
    for e in range(n):
        parts += [np.ascontiguousarray(d["env"][e], np.int32).view(np.uint8),
                  np.ascontiguousarray(d["ent"][e], np.int16).reshape(-1).view(np.uint8),
                  np.ascontiguousarray(d["ring"][e], np.int16).view(np.uint8),
                  np.ascontiguousarray(d["mat"][e], np.uint8).reshape(-1),
                  np.ascontiguousarray(d["items"][e], np.uint32).reshape(-1).view(np.uint8),
                  np.ascontiguousarray(d["iring"][e], np.int16).view(np.uint8),
                  np.ascontiguousarray(d["tasks"][e], np.int32).view(np.uint8),
                  np.ascontiguousarray(d["tstate"][e]).view(np.uint8)]
    return np.concatenate(parts)
