"""NmmoEngine — a batch of envs stepped in lockstep on one GPU through libnmmo_hip.so.

This is the MI355X replacement for the reference's whole env stack below the trainer:
`nmmo.Env` x num_envs + `pufferlib.vectorization.*` (clean_pufferl.py:106-114). State lives in
HBM as SoA over (env x slot); I/O buffers are torch tensors on the same device, passed to the
C-ABI as raw device pointers, and every call is enqueued on torch's current stream.
"""

from __future__ import annotations

import ctypes

import numpy as np
import torch

from . import abi
from ._native import NativeError, check, layout, lib


class TickFault(NativeError):
    """A tick launch hit one of its loop bounds (nmmo_get_fault): that env's step is not the
    serial-order result, so nothing downstream (a learner, a bench line) may use it."""

    def __init__(self, word: int, where: str = ""):
        self.word = int(word)
        self.code, self.env = self.word & 0xFF, self.word >> 8
        what = abi.FAULT_NAMES.get(self.code, f"code {self.code}")
        super().__init__(f"{where + ': ' if where else ''}tick fault word {self.word:#x}: {what} "
                         f"(env / list position {self.env})")


class NmmoEngine:
    def __init__(self, config, n_envs: int, seed: int = 0, device=None, task_embedding=None,
                 env_index_base: int = 0):
        self.config = config
        self.n_envs = int(n_envs)
        self.device = torch.device("cuda", torch.cuda.current_device()) if device is None \
            else torch.device(device)
        if self.device.type != "cuda":
            raise ValueError("NmmoEngine runs on a HIP device only")
        self.cfg = config.to_c(env_index_base)
        self.layout = layout(self.cfg)
        self.P = config.PLAYER_N
        self.S = self.layout.slots
        self.obs_elems = self.layout.obs_elems
        task = None
        if task_embedding is not None:
            task = np.ascontiguousarray(np.asarray(task_embedding, dtype=np.float16)).view(np.uint16)
            if task.size != config.TASK_EMBED_DIM:
                raise ValueError("task embedding size != TASK_EMBED_DIM")
        self._task = task
        h = ctypes.c_void_p()
        with torch.cuda.device(self.device):
            check(lib().nmmo_create(ctypes.byref(self.cfg), self.n_envs, seed & (2**64 - 1),
                                    self.device.index,
                                    None if task is None else task.ctypes.data_as(ctypes.c_void_p),
                                    ctypes.byref(h)), "nmmo_create")
        self.h = h
        d = self.device
        n, P = self.n_envs, self.P
        self.actions = torch.zeros((n, P, abi.N_ACTION_HEADS), dtype=torch.int32, device=d)
        if config.obs_layout == abi.OBS_FLAT:  # 12.6 GB at 1,024 envs: chunk-mapped (devmem)
            from . import devmem

            self.obs = devmem.empty((n, P, self.obs_elems), torch.float32, d)
        elif config.obs_layout == abi.OBS_NATIVE:  # SPEC §8b: per env, P rows + the Market
            from . import devmem

            self.obs = devmem.empty((n, abi.native_env_bytes(P)), torch.uint8, d)
        elif config.obs_layout == abi.OBS_WIRE:  # SPEC §8c: header + records, sized for full windows
            from . import devmem, wire

            self.obs = devmem.empty((wire.max_bytes(n, P),), torch.uint8, d)
        else:
            self.obs = None
        if self.obs is not None and config.obs_layout in (abi.OBS_FLAT, abi.OBS_NATIVE):
            # the engine's own buffer: obs rows are written incrementally (nmmo_obs_bind)
            check(lib().nmmo_obs_bind(self.h, self._ptr(self.obs)), "nmmo_obs_bind")
        emb = np.zeros((1, config.TASK_EMBED_DIM), np.float32) if task is None else \
            task.view(np.float16).astype(np.float32).reshape(1, -1)
        self.task_table = emb  # Task obs per task index (native-layout decoding)
        self.rew = torch.zeros((n, P), dtype=torch.float32, device=d)
        self.term = torch.zeros((n, P), dtype=torch.uint8, device=d)
        self.trunc = torch.zeros((n, P), dtype=torch.uint8, device=d)
        self.mask = torch.zeros((n, P), dtype=torch.uint8, device=d)
        self.info = None
        from . import maps

        self.maps_source = maps.prepare(self)  # PATH_MAPS / MAP_FORCE_GENERATION (environment.py:33,41)

    def close(self):
        if getattr(self, "h", None) is not None and self.h.value:
            torch.cuda.synchronize(self.device)
            lib().nmmo_destroy(self.h)
            self.obs = None
            from . import devmem

            devmem.release_pending()  # the chunk-mapped buffers no tensor holds any more
        self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    @staticmethod
    def _ptr(t):
        return None if t is None else ctypes.c_void_p(t.data_ptr())

    def _stream(self):
        return ctypes.c_void_p(torch.cuda.current_stream(self.device).cuda_stream)

    def reset(self, env_seeds=None):
        seeds = None
        if env_seeds is not None:
            seeds = np.ascontiguousarray(env_seeds, dtype=np.uint64)
            assert seeds.shape == (self.n_envs,)
        with torch.cuda.device(self.device):
            check(lib().nmmo_reset(self.h, None if seeds is None else seeds.ctypes.data_as(ctypes.c_void_p),
                                   self._ptr(self.obs), self._ptr(self.mask), self._stream()),
                  "nmmo_reset")
        self.rew.zero_()
        self.term.zero_()
        self.trunc.zero_()
        return self.obs, self.mask

    def end_episodes(self, env_mask):
        """End the current episode of the envs where env_mask (bool/u8 [n_envs], host or device)
        is set: their next step resets them (nmmo_end_episodes, enqueued on the current stream;
        the per-env reset of an async pool)."""
        m = torch.as_tensor(np.asarray(env_mask, dtype=np.uint8) if not torch.is_tensor(env_mask) else env_mask)
        if tuple(m.shape) != (self.n_envs,):
            raise ValueError(f"env_mask must have shape ({self.n_envs},)")
        m = m.to(device=self.device, dtype=torch.uint8).contiguous()
        with torch.cuda.device(self.device):
            check(lib().nmmo_end_episodes(self.h, self._ptr(m), self._stream()), "nmmo_end_episodes")
        self._end_mask = m  # alive until the stream has read it

    def step(self, actions=None, write_obs: bool = True):
        """One tick of every env; `actions` int32 [n_envs, P, 12] on the device (default: the
        engine's own action buffer). Outputs are the engine's tensors (overwritten in place);
        write_obs=False skips the obs gather for this tick (obs keeps its previous contents)."""
        a = self.actions if actions is None else actions
        if a.dtype != torch.int32 or not a.is_contiguous() or a.device != self.device:
            a = a.to(device=self.device, dtype=torch.int32).contiguous()
        assert tuple(a.shape) == (self.n_envs, self.P, abi.N_ACTION_HEADS)
        with torch.cuda.device(self.device):
            check(lib().nmmo_step(self.h, self._ptr(a), self._ptr(self.obs if write_obs else None),
                                  self._ptr(self.rew),
                                  self._ptr(self.term), self._ptr(self.trunc), self._ptr(self.mask),
                                  self._stream()), "nmmo_step")
        return self.obs, self.rew, self.term, self.trunc, self.mask

    def step_envs(self, env_ids, actions=None, write_obs: bool = True):
        """One tick of the listed envs only (nmmo_step_envs): env_ids int32 on the device
        (distinct, in [0, n_envs)); actions and outputs keep the full [n_envs, ...] shape, and
        only the listed envs' rows are read / written (the async pool's send, vecenv.py)."""
        a = self.actions if actions is None else actions
        if a.dtype != torch.int32 or not a.is_contiguous() or a.device != self.device:
            a = a.to(device=self.device, dtype=torch.int32).contiguous()
        assert tuple(a.shape) == (self.n_envs, self.P, abi.N_ACTION_HEADS)
        ids = env_ids
        if ids.dtype != torch.int32 or ids.device != self.device or not ids.is_contiguous():
            raise ValueError("env_ids must be a contiguous int32 tensor on the engine's device")
        with torch.cuda.device(self.device):
            check(lib().nmmo_step_envs(self.h, self._ptr(ids), ids.numel(), self._ptr(a),
                                       self._ptr(self.obs if write_obs else None), self._ptr(self.rew),
                                       self._ptr(self.term), self._ptr(self.trunc), self._ptr(self.mask),
                                       self._stream()), "nmmo_step_envs")
        self._ids = ids  # alive until the stream has read it
        return self.obs, self.rew, self.term, self.trunc, self.mask

    def observe(self, out=None):
        """The obs gather alone over the current state into `out` (default: the engine's obs
        buffer): step(write_obs=False) + observe() == step() (nmmo_observe)."""
        out = self.obs if out is None else out
        with torch.cuda.device(self.device):
            check(lib().nmmo_observe(self.h, self._ptr(out), self._stream()), "nmmo_observe")
        return out

    def expand_obs(self, native=None, out=None):
        """Native obs (SPEC §8b; default: this engine's) -> pufferlib flat float32
        [n, P, obs_elems] on the device, bit-identical to the flat layout (nmmo_expand_obs)."""
        native = self.obs if native is None else native
        n = native.shape[0]
        out = torch.empty((n, self.P, self.obs_elems), dtype=torch.float32, device=self.device) \
            if out is None else out
        with torch.cuda.device(self.device):
            check(lib().nmmo_expand_obs(self.h, self._ptr(native), self._ptr(out), n, self._stream()),
                  "nmmo_expand_obs")
        return out

    def scripted_actions(self, policy_seed: int, out=None):
        out = self.actions if out is None else out
        with torch.cuda.device(self.device):
            check(lib().nmmo_scripted_actions(self.h, policy_seed & (2**64 - 1), self._ptr(out),
                                              self._stream()), "nmmo_scripted_actions")
        return out

    def set_wrapper(self, wc):
        """Turn the device wrapper layer on (abi.NmmoWrapperConfig, e.g. from
        nmmo_amd.wrappers.wrapper_config) or off (None). While on, rewards are shaped in place,
        obs masks edited, and `self.info` (agent_info_dtype records [n_envs, P] as raw bytes on
        the device) holds each agent's episode record on its final step (SPEC §13)."""
        if wc is None:
            check(lib().nmmo_set_wrapper(self.h, None, None), "nmmo_set_wrapper")
            self.info = None
            return
        rec = abi.agent_info_dtype().itemsize
        self.info = torch.zeros((self.n_envs, self.P, rec), dtype=torch.uint8, device=self.device)
        self.wrapper = wc
        check(lib().nmmo_set_wrapper(self.h, ctypes.byref(wc), self._ptr(self.info)), "nmmo_set_wrapper")

    def wrapper_dropped_events(self) -> int:
        """Event rows the wrapper missed (ring overwritten within one tick; nonzero = raise
        event_cap, the episode stats diverge from the reference's BaseStatWrapper)."""
        v = ctypes.c_int64()
        check(lib().nmmo_get_wrapper_dropped(self.h, ctypes.byref(v)), "nmmo_get_wrapper_dropped")
        return v.value

    def info_records(self) -> np.ndarray:
        """The device episode records as numpy agent_info_dtype [n_envs, P] (synchronous)."""
        return self.info.cpu().numpy().view(abi.agent_info_dtype()).reshape(self.n_envs, self.P)

    def wrapper_state(self):
        """(NmmoWrapState records [n_envs, P], experienced bitsets u32 [n_envs, P, 153])."""
        st = np.zeros((self.n_envs, self.P), abi.wrap_state_dtype())
        uq = np.zeros((self.n_envs, self.P, abi.UNIQ_WORDS), np.uint32)
        check(lib().nmmo_get_wrapper_state(self.h, st.ctypes.data_as(ctypes.c_void_p),
                                           uq.ctypes.data_as(ctypes.c_void_p)), "nmmo_get_wrapper_state")
        return st, uq

    def set_timing(self, enable: bool):
        check(lib().nmmo_set_timing(self.h, 1 if enable else 0), "nmmo_set_timing")

    def set_counters(self, counters):
        """Device u64 [3] (torch int64 tensor on this device) the kernels add into: agent-steps
        (sum of mask), finished episodes and event-log rows appended; None disables."""
        if counters is not None and (counters.numel() < 3 or counters.dtype != torch.int64
                                     or counters.device != self.device):
            raise ValueError("counters must be an int64 tensor of >= 3 elements on the engine's device")
        ptr = None if counters is None else ctypes.c_void_p(counters.data_ptr())
        self._counters = counters
        check(lib().nmmo_set_counters(self.h, ptr), "nmmo_set_counters")

    def set_obs_counter(self, counter):
        """Device u64 [n_envs, 2] (torch int64 tensor on this device) every obs gather adds
        into, per env: [e, 0] the rows it wrote (rows of agents in the realm + rows zeroed),
        [e, 1] the bytes it stored (nmmo_set_obs_counter); None disables."""
        if counter is not None and (counter.numel() < 2 * self.n_envs or counter.dtype != torch.int64
                                    or counter.device != self.device or not counter.is_contiguous()):
            raise ValueError("counter must be a contiguous int64 tensor of >= 2 * n_envs elements on the "
                             "engine's device")
        self._obs_counter = counter
        check(lib().nmmo_set_obs_counter(self.h, None if counter is None else ctypes.c_void_p(counter.data_ptr())),
              "nmmo_set_obs_counter")

    def set_step_records(self, records, fault=None):
        """uint8 [n_envs, P, 8] device tensor (or None = off) every following step() with wire obs
        fills, per agent, with reward f32 | term | trunc | mask | 0 (nmmo_set_step_records); read
        when a step is enqueued, so a captured step keeps the tensor it saw. fault: a device int32
        tensor the same launch stores a nonzero tick fault word into (fault_into()'s effect)."""
        if records is not None and (records.dtype != torch.uint8 or records.device != self.device
                                    or not records.is_contiguous() or records.numel() < 8 * self.n_envs * self.P):
            raise ValueError("records must be a contiguous uint8 tensor of >= 8 * n_envs * P bytes on the "
                             "engine's device")
        if fault is not None and (fault.dtype != torch.int32 or fault.device != self.device):
            raise ValueError("fault must be an int32 tensor on the engine's device")
        self._step_records = (records, fault)
        check(lib().nmmo_set_step_records(self.h, None if records is None else ctypes.c_void_p(records.data_ptr()),
                                          None if fault is None else ctypes.c_void_p(fault.data_ptr())),
              "nmmo_set_step_records")

    def obs_invalidate(self):
        """Forget what the obs rows hold (nmmo_obs_invalidate): call after writing into self.obs;
        the next gather writes every row in full."""
        check(lib().nmmo_obs_invalidate(self.h, self._stream()), "nmmo_obs_invalidate")

    def obs_invalidate_envs(self, env_ids):
        """Forget what the listed envs' obs rows hold (nmmo_obs_invalidate_envs; env_ids a
        contiguous int32 tensor on the device): their next gather writes those rows in full.
        Enqueued on the current stream."""
        if env_ids.dtype != torch.int32 or env_ids.device != self.device or not env_ids.is_contiguous():
            raise ValueError("env_ids must be a contiguous int32 tensor on the engine's device")
        with torch.cuda.device(self.device):
            check(lib().nmmo_obs_invalidate_envs(self.h, self._ptr(env_ids), env_ids.numel(), self._stream()),
                  "nmmo_obs_invalidate_envs")
        self._inv_ids = env_ids  # alive until the stream has read it

    def obs_invalidate_sections(self, sections: int, env_ids=None):
        """Forget only the given sections (abi.OBS_SEC_*) of the listed envs' obs rows
        (nmmo_obs_invalidate_sections; env_ids a contiguous int32 tensor on the device, None =
        every env): OBS_SEC_TILE alone makes the next gather rewrite those rows' Tile sections and
        stay incremental elsewhere. Enqueued on the current stream."""
        if env_ids is not None and (env_ids.dtype != torch.int32 or env_ids.device != self.device
                                    or not env_ids.is_contiguous()):
            raise ValueError("env_ids must be a contiguous int32 tensor on the engine's device")
        with torch.cuda.device(self.device):
            check(lib().nmmo_obs_invalidate_sections(self.h, None if env_ids is None else self._ptr(env_ids),
                                                     0 if env_ids is None else env_ids.numel(), int(sections),
                                                     self._stream()), "nmmo_obs_invalidate_sections")
        self._inv_ids = env_ids

    def get_fault(self) -> int:
        """The tick fault word (nmmo_get_fault: NMMO_FAULT_* | env << 8, 0 = none), then cleared."""
        f = ctypes.c_int32()
        check(lib().nmmo_get_fault(self.h, ctypes.byref(f)), "nmmo_get_fault")
        return f.value

    def check_fault(self, where: str = ""):
        """Raise TickFault when a launch since the last read hit a loop bound (reads and clears
        the word; synchronous). Called at every host sync of the product paths."""
        f = self.get_fault()
        if f:
            raise TickFault(f, where)

    def fault_into(self, dst):
        """Enqueue: dst (device int32 [1]) takes the fault word if it is non-zero and dst is 0
        (nmmo_fault_into; no sync, graph-capturable)."""
        with torch.cuda.device(self.device):
            check(lib().nmmo_fault_into(self.h, self._ptr(dst), self._stream()), "nmmo_fault_into")

    def inject_fault(self, word: int):
        """Test hook (nmmo_inject_fault): set the fault word."""
        check(lib().nmmo_inject_fault(self.h, int(word)), "nmmo_inject_fault")

    def read_timing(self):
        """(tick_ms_sum, obs_ms_sum, n_steps, wrapper_ms_sum) from HIP events on the launch stream."""
        ms = (ctypes.c_double * 3)()
        n = ctypes.c_int32()
        check(lib().nmmo_read_timing(self.h, ms, ctypes.byref(n)), "nmmo_read_timing")
        return ms[0], ms[1], n.value, ms[2]

    def get_state(self) -> np.ndarray:
        n = self.layout.state_bytes_per_env * self.n_envs
        buf = np.zeros(n, np.uint8)
        check(lib().nmmo_get_state(self.h, buf.ctypes.data_as(ctypes.c_void_p), n), "nmmo_get_state")
        return buf

    def set_state(self, buf: np.ndarray):
        buf = np.ascontiguousarray(buf, dtype=np.uint8)
        check(lib().nmmo_set_state(self.h, buf.ctypes.data_as(ctypes.c_void_p), buf.nbytes),
              "nmmo_set_state")

    def set_tasks(self, tasks, embeddings=None, assign=None):
        """Task table (sequence of abi.NmmoTask, e.g. from nmmo_amd.tasks), optional fp16
        embeddings [n_tasks, task_embed_dim] for the Task obs, and int32 assign [n_envs, P]
        (None = task 0 for everyone). SPEC §12; call before reset() for whole episodes."""
        arr = (abi.NmmoTask * len(tasks))(*tasks)
        emb = None if embeddings is None else np.ascontiguousarray(embeddings, np.float16)
        self.task_table = (np.repeat(self.task_table[:1], len(tasks), axis=0) if emb is None
                           else emb.astype(np.float32).reshape(len(tasks), -1))
        asg = None if assign is None else np.ascontiguousarray(assign, np.int32)
        self.task_names = None
        check(lib().nmmo_set_tasks(self.h, ctypes.cast(arr, ctypes.c_void_p), len(tasks),
                                   None if emb is None else emb.ctypes.data_as(ctypes.c_void_p),
                                   None if asg is None else asg.ctypes.data_as(ctypes.c_void_p)),
              "nmmo_set_tasks")

    def set_task_weights(self, weights):
        """Sample every player's task at each env reset with probability weight / sum (SPEC §12,
        nmmo_set_task_weights); None = keep the fixed assignment."""
        w = None if weights is None else np.ascontiguousarray(weights, np.float64)
        check(lib().nmmo_set_task_weights(self.h, None if w is None else w.ctypes.data_as(ctypes.c_void_p),
                                          0 if w is None else len(w)), "nmmo_set_task_weights")

    def set_curriculum(self, specs, sample: bool = True, assign=None):
        """The curriculum the reference's env samples from (nmmo.Env with CURRICULUM_FILE_PATH,
        environment.py:48-49): a list of nmmo_amd.tasks.TaskSpec. Their programs become the task
        table, their embeddings (when every spec has one) the Task obs, their names the
        facade's spec_name; with sample=True each reset draws every player's task by
        sampling_weight (call before reset())."""
        emb = None
        if all(s.embedding is not None for s in specs):
            emb = np.stack([np.asarray(s.embedding, np.float16) for s in specs])
        self.set_tasks([s.program() for s in specs], emb, assign)
        self.task_names = [s.name for s in specs]
        if sample:
            self.set_task_weights([float(s.sampling_weight) for s in specs])

    def events(self, env: int, max_rows: int | None = None) -> np.ndarray:
        """Retained event-log rows of `env`, oldest first: int32 [n, 9] (SPEC §11 columns
        id, ent_id, tick, event, type, level, number, gold, target_ent). Synchronous."""
        cap = self.config.event_cap
        m = cap if max_rows is None else min(max_rows, cap)
        buf = np.zeros((max(m, 1), abi.EVENT_COLS), np.int32)
        n = ctypes.c_int32()
        check(lib().nmmo_get_events(self.h, env, buf.ctypes.data_as(ctypes.c_void_p), m, ctypes.byref(n)),
              "nmmo_get_events")
        return buf[:n.value].copy()

    def map_bank(self) -> np.ndarray:
        buf = np.zeros((self.config.MAP_N, abi.MAP_SIZE, abi.MAP_SIZE), np.uint8)
        check(lib().nmmo_get_map_bank(self.h, buf.ctypes.data_as(ctypes.c_void_p), buf.nbytes),
              "nmmo_get_map_bank")
        return buf

    def set_map_bank(self, bank: np.ndarray):
        """Replace the generated bank (e.g. maps loaded from PATH_MAPS, nmmo_amd/maps.py); envs
        use it from their next reset."""
        buf = np.ascontiguousarray(bank, dtype=np.uint8)
        if buf.shape != (self.config.MAP_N, abi.MAP_SIZE, abi.MAP_SIZE):
            raise ValueError(f"map bank must be uint8 [{self.config.MAP_N}, {abi.MAP_SIZE}, {abi.MAP_SIZE}]")
        check(lib().nmmo_set_map_bank(self.h, buf.ctypes.data_as(ctypes.c_void_p), buf.nbytes),
              "nmmo_set_map_bank")
