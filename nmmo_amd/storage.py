"""DeviceExperience — the reference trainer's rollout storage kept in HBM.

The reference's `clean_pufferl` allocates its experience buffers as host tensors viewed as numpy
arrays (`reinforcement_learning/clean_pufferl.py:182-197`), copies every recv's observations,
values, actions, logprobs, rewards and dones into them through the host (`:318,:329-346`), sorts
the `(env_id, step)` keys on the host (`:414`), walks the advantage recurrence in a Python loop
(`:424-436`) and gathers the minibatch rows with numpy fancy indexing before the H2D copies
(`:439-458`). Here every one of those steps is a HIP kernel on device buffers
(`nmmo_amd/csrc/storage.hip`), reached through the C-ABI (`include/nmmo_hip.h`,
`nmmo_exp_*`); the observation rows go straight from the env's obs buffer (flat) or its native
layout (SPEC §8b, expanded on store) into their experience slot.

Names follow the reference: obs / actions / logprobs / rewards / dones / truncateds / values,
`ptr`, `batch_size`, `batch_rows`, `bptt_horizon`, b_idxs, advantages, returns.
"""

from __future__ import annotations

import ctypes

import torch

from . import abi
from ._native import check, lib


def _p(t):
    return None if t is None else ctypes.c_void_p(t.data_ptr())


class DeviceExperience:
    def __init__(self, batch_size: int, obs_elems: int, n_slots: int, device=None, record_arena_bytes: int = 0):
        """batch_size: rows trained on per update (the buffers hold batch_size + 1, :182);
        n_slots: the env_id range = num_envs x agents_per_env (:119). record_arena_bytes > 0:
        compact storage (nmmo_exp_store_records) — observations stay the wire records they came
        in as (~0.3 KB per row instead of 95,948 B), in an arena of that many bytes, and are
        expanded to flat rows per minibatch (gather_obs)."""
        self.device = torch.device("cuda", torch.cuda.current_device()) if device is None \
            else torch.device(device)
        self.batch_size = int(batch_size)
        self.capacity = cap = self.batch_size + 1
        self.obs_elems = int(obs_elems)
        self.n_slots = int(n_slots)
        d = self.device
        f32 = dict(dtype=torch.float32, device=d)
        i32 = dict(dtype=torch.int32, device=d)
        from . import devmem

        self.records = None
        if record_arena_bytes > 0:
            self.obs = None
            self.arena = devmem.empty((int(record_arena_bytes),), torch.uint8, d)
            self.arena_used = torch.zeros(1, dtype=torch.int64, device=d)
            self.row_buf = torch.zeros(cap, dtype=torch.int64, device=d)
            self.row_agent = torch.zeros(cap, **i32)
            self.records = abi.NmmoRecordStore(self.arena.data_ptr(), int(record_arena_bytes),
                                               self.arena_used.data_ptr(), self.row_buf.data_ptr(),
                                               self.row_agent.data_ptr())
        else:
            self.obs = devmem.empty((cap, self.obs_elems), torch.float32, d)  # chunk-mapped when large
            self.obs.zero_()
        self.actions = torch.zeros((cap, abi.N_ACTION_HEADS), dtype=torch.int64, device=d)
        self.logprobs = torch.zeros(cap, **f32)
        self.rewards = torch.zeros(cap, **f32)
        self.dones = torch.zeros(cap, **f32)
        self.truncateds = torch.zeros(cap, **f32)
        self.values = torch.zeros(cap, **f32)
        self.env_id = torch.zeros(cap, **i32)
        self.step = torch.zeros(cap, **i32)
        self.seq = torch.zeros(cap, **i32)
        self.slot_count = torch.zeros(self.n_slots, **i32)
        self.ptr_dev = torch.zeros(1, **i32)
        self.status_dev = torch.zeros(1, **i32)  # bit 0: a row with an out-of-range env_id was dropped
        self._scratch_rows = 0
        self.scratch = torch.zeros(0, **i32)
        self.x = abi.NmmoExperience(cap, self.obs_elems, self.n_slots, *[
            None if t is None else t.data_ptr() for t in (self.obs, self.actions, self.logprobs, self.rewards, self.dones,
                                   self.truncateds, self.values, self.env_id, self.step, self.seq,
                                   self.slot_count, self.ptr_dev, self.status_dev)])

    def _stream(self):
        return ctypes.c_void_p(torch.cuda.current_stream(self.device).cuda_stream)

    def _ensure_scratch(self, n_rows: int, n_inputs: int = 0, max_rows: int = 0):
        """n_rows: the rows of one store; n_inputs > 0: a store_many over n_inputs inputs of at most
        max_rows rows (nmmo_exp_scratch_ints_many)."""
        need = int(lib().nmmo_exp_scratch_ints(max(n_rows, 1), self.n_slots))
        if n_inputs:
            need = max(need, int(lib().nmmo_exp_scratch_ints_many(n_inputs, max(max_rows, 1), self.n_slots)))
        if self.scratch.numel() < need:
            self.scratch = torch.zeros(need, dtype=torch.int32, device=self.device)

    # -- evaluate side (clean_pufferl.py:200-346)
    def reset(self):
        """Start a new batch: ptr = 0 (:200) and empty sort keys (:415)."""
        self.ptr_dev.zero_()
        self.slot_count.zero_()
        if self.records is not None:
            self.arena_used.zero_()

    @property
    def status(self) -> int:
        """Device status word (nmmo_hip.h NmmoExperience.status); 0 = every selected row stored."""
        return int(self.status_dev.item())

    @property
    def ptr(self) -> int:
        return int(self.ptr_dev.item())

    def full(self) -> bool:
        """The evaluate loop's exit test `ptr == batch_size + 1` (:290)."""
        return self.ptr == self.capacity

    def store(self, o, r, d, mask, actions, logprob, value, step: int, env_id=None, env_id_base: int = 0,
              engine=None, validate: bool = False):
        """Append the learner-mask rows of one recv in row order, cut at the room left (:331-346).
        o: flat float32 [N, obs_elems] (or [n_envs, P, obs_elems]), the native uint8
        [n_envs, env_bytes] buffer of `engine` (an NmmoEngine with obs_layout NATIVE), expanded
        on store, or a uint8 wire buffer (SPEC §8c) of N / P envs with `engine` an NmmoEngine
        with obs_layout WIRE (its layout and task table), the kept rows decoded on store; r float32 [N]; d / mask uint8 or bool [N]; actions int [N, 12]; logprob /
        value float32 [N]; env_id int [N] distinct agent-slot ids (None = env_id_base + row)."""
        dev = self.device

        def cvt(t, dtype):
            t = torch.as_tensor(t)
            if t.dtype == torch.bool:
                t = t.to(torch.uint8)
            return t.to(device=dev, dtype=dtype).contiguous().view(-1)

        r_, d_, m_ = cvt(r, torch.float32), cvt(d, torch.uint8), cvt(mask, torch.uint8)
        lp, v = cvt(logprob, torch.float32), cvt(value, torch.float32)
        n = r_.numel()
        a = torch.as_tensor(actions).to(device=dev, dtype=torch.int32).contiguous().view(n, abi.N_ACTION_HEADS)
        eid = None if env_id is None else cvt(env_id, torch.int32)
        if validate and eid is not None:  # the ABI precondition (synchronising check)
            sel = eid[cvt(mask, torch.uint8) != 0]
            if sel.numel() and (int(sel.min()) < 0 or int(sel.max()) >= self.n_slots):
                raise ValueError("env_id outside [0, n_slots)")
            if torch.unique(sel).numel() != sel.numel():
                raise ValueError("env_id must be distinct within one store")
        native = engine is not None and engine.config.obs_layout == abi.OBS_NATIVE
        wired = engine is not None and engine.config.obs_layout == abi.OBS_WIRE
        if self.records is not None and not wired:
            raise ValueError("compact (record) storage stores wire buffers: pass the wire engine")
        obs_flat = obs_nat = obs_wire = None
        if native:
            if o.dtype != torch.uint8 or o.shape[0] * engine.P != n:
                raise ValueError("native obs must be the engine's uint8 [n_envs, env_bytes] buffer")
            obs_nat = o.contiguous()
        elif wired:  # a wire buffer of n / P envs (SPEC §8c): only the kept rows are decoded
            if o.dtype != torch.uint8 or o.dim() != 1 or n % engine.P:
                raise ValueError("wire obs must be a uint8 wire buffer of whole envs")
            obs_wire = o
        else:
            obs_flat = o.contiguous().view(n, self.obs_elems)
            if obs_flat.dtype != torch.float32:
                raise ValueError("flat obs must be float32")
        for t in (m_, d_, lp, v):
            if t.numel() != n:
                raise ValueError("per-row inputs must all have N rows")
        self._ensure_scratch(n)
        inp = abi.NmmoStoreInput(n, int(step), obs_flat.data_ptr() if obs_flat is not None else None,
                                 obs_nat.data_ptr() if obs_nat is not None else None, r_.data_ptr(),
                                 d_.data_ptr(), m_.data_ptr(), eid.data_ptr() if eid is not None else None,
                                 int(env_id_base), a.data_ptr(), lp.data_ptr(), v.data_ptr(),
                                 obs_wire.data_ptr() if obs_wire is not None else None)
        with torch.cuda.device(dev):
            if self.records is not None:
                self._engine = engine  # its task table decodes the records (gather_obs)
                check(lib().nmmo_exp_store_records(engine.h, ctypes.byref(self.x), ctypes.byref(self.records),
                                                   ctypes.byref(inp), _p(self.scratch), self._stream()),
                      "nmmo_exp_store_records")
            else:
                check(lib().nmmo_exp_store(engine.h if native or wired else None, ctypes.byref(self.x),
                                           ctypes.byref(inp), _p(self.scratch), self._stream()), "nmmo_exp_store")
        # keep the inputs alive until the kernels that read them have been enqueued
        self._inflight = (r_, d_, m_, lp, v, a, eid, obs_flat, obs_nat, obs_wire)

    def store_many(self, inputs, step: int, engine, field_stride: int = 0, expect=None, check_status=None,
                   checked=None):
        """Several wire buffers stored as one store, in input order (compact storage only;
        nmmo_exp_store_records_many: a fixed number of launches for up to 16 buffers, e.g. every
        rank's buffers of a step at the learner). inputs: (wire, rewards, dones, mask, actions,
        logprobs, values, env_id_base) per buffer, all device tensors already in their final
        dtype; field_stride > 0: rewards / dones / mask are byte views read field_stride bytes
        apart per row (the gather's packed 8-B per-agent smalls).

        check_status (device int32 [1]) fuses the received-buffer check into the store
        (nmmo_exp_store_records_checked): every input is validated as nmmo_wire_check_many does,
        its bits OR-ed into check_status, and an input that fails keeps no row. expect: per
        input a device int64 [1] announced total, or None; checked: per input whether to check it
        (default all; an unchecked input, e.g. the root's own buffer, counts as clean)."""
        if self.records is None:
            raise ValueError("store_many needs compact (record) storage")
        n = len(inputs)
        arr = (abi.NmmoStoreInput * n)()
        rows = 0
        keep = []
        for i, (w, r, d, m, a, lp, v, base) in enumerate(inputs):
            nr = a.shape[0]
            rows += nr
            arr[i] = abi.NmmoStoreInput(nr, int(step), None, None, r.data_ptr(), d.data_ptr(), m.data_ptr(), None,
                                        int(base), a.data_ptr(), lp.data_ptr(), v.data_ptr(), w.data_ptr())
            keep.append((w, r, d, m, a, lp, v))
        self._ensure_scratch(rows, n, max(a.shape[0] for _, _, _, _, a, _, _, _ in inputs))
        self._engine = engine
        with torch.cuda.device(self.device):
            if check_status is None:
                check(lib().nmmo_exp_store_records_many(engine.h, ctypes.byref(self.x), ctypes.byref(self.records), arr,
                                                        n, int(field_stride), _p(self.scratch), self._stream()),
                      "nmmo_exp_store_records_many")
            else:
                if check_status.dtype != torch.int32 or check_status.device != self.device:
                    raise ValueError("check_status must be a device int32 tensor on the store's device")
                ex = list(expect) if expect is not None else [None] * n
                if len(ex) != n or any(e is not None and (e.dtype != torch.int64 or e.device != self.device)
                                       for e in ex):
                    raise ValueError("expect: one device int64 [1] (or None) per input")
                exp_arr = (ctypes.c_void_p * n)(*[None if e is None else e.data_ptr() for e in ex])
                mask = sum(1 << i for i in range(n) if checked is None or checked[i])
                if getattr(self, "_ctl", None) is None:  # zero; every call leaves it zero
                    self._ctl = torch.zeros(abi.STORE_CTL_INTS, dtype=torch.int32, device=self.device)
                check(lib().nmmo_exp_store_records_checked(engine.h, ctypes.byref(self.x), ctypes.byref(self.records),
                                                           arr, n, int(field_stride), exp_arr, mask, _p(check_status),
                                                           _p(self._ctl), _p(self.scratch), self._stream()),
                      "nmmo_exp_store_records_checked")
                keep.append(ex)
        self._inflight = keep

    # -- train side (clean_pufferl.py:413-458)
    def sort(self) -> torch.Tensor:
        """idxs: the stored rows sorted by (env_id, step) (:414), device int32 [ptr]."""
        n = self.ptr
        idxs = torch.empty(n, dtype=torch.int32, device=self.device)
        self._ensure_scratch(1)
        with torch.cuda.device(self.device):
            check(lib().nmmo_exp_sort(ctypes.byref(self.x), _p(idxs), _p(self.scratch), self._stream()),
                  "nmmo_exp_sort")
        self.slot_count.zero_()  # data.sort_keys = [] (:415)
        return idxs

    def advantages(self, idxs: torch.Tensor, gamma: float, gae_lambda: float) -> torch.Tensor:
        """The reversed GAE loop over idxs (:424-436), float32, bit-identical to the reference."""
        if idxs.numel() != self.capacity:
            raise ValueError("advantages need a full batch (ptr == batch_size + 1)")
        adv = torch.zeros(self.batch_size, dtype=torch.float32, device=self.device)
        with torch.cuda.device(self.device):
            check(lib().nmmo_exp_gae(ctypes.byref(self.x), _p(idxs), self.batch_size, float(gamma),
                                     float(gae_lambda), _p(adv), self._stream()), "nmmo_exp_gae")
        return adv

    def batch(self, idxs: torch.Tensor, advantages: torch.Tensor, batch_rows: int, bptt_horizon: int) -> dict:
        """The flattened batch of :417-450: b_idxs [num_minibatches, batch_rows, bptt_horizon],
        b_advantages, b_values, b_returns in the same shapes (values/advantages gathered on
        the device; obs stay in place and are gathered per minibatch)."""
        num_mb = self.batch_size // bptt_horizon // batch_rows
        b_idxs = idxs[:-1].reshape(batch_rows, num_mb, bptt_horizon).transpose(0, 1)
        b_values = self.gather(self.values, b_idxs)
        b_adv = advantages.reshape(batch_rows, num_mb, bptt_horizon).transpose(0, 1)
        return {"b_idxs": b_idxs, "b_values": b_values, "b_advantages": b_adv, "b_returns": b_adv + b_values,
                "num_minibatches": num_mb}

    def minibatch(self, b_idxs: torch.Tensor, mb: int) -> dict:
        """Minibatch `mb` of the flattened batch (:456-462): obs [batch_rows, bptt, obs_elems],
        actions, logprobs, dones, values gathered straight from the experience rows."""
        idx = b_idxs[mb]
        return {"obs": self.gather_obs(idx), "actions": self.gather(self.actions, idx),
                "logprobs": self.gather(self.logprobs, idx), "dones": self.gather(self.dones, idx),
                "values": self.gather(self.values, idx)}

    def gather_obs(self, idx: torch.Tensor, engine=None) -> torch.Tensor:
        """Flat float32 obs rows of experience rows idx (any shape): a row gather, or with compact
        storage the records expanded on the device (nmmo_exp_gather_records; `engine` = the wire
        handle whose task table the records use, default the one the stores came from)."""
        if self.records is None:
            return self.gather(self.obs, idx)
        eng = engine or self._engine
        flat_idx = idx.reshape(-1).to(torch.int32).contiguous()
        out = torch.empty((flat_idx.numel(), self.obs_elems), dtype=torch.float32, device=self.device)
        with torch.cuda.device(self.device):
            check(lib().nmmo_exp_gather_records(eng.h, ctypes.byref(self.x), ctypes.byref(self.records), _p(flat_idx),
                                                flat_idx.numel(), _p(out), self._stream()), "nmmo_exp_gather_records")
        return out.view(tuple(idx.shape) + (self.obs_elems,))

    def gather(self, src: torch.Tensor, idx: torch.Tensor) -> torch.Tensor:
        """src[idx] on the device through nmmo_gather_rows (rows of src's trailing dims)."""
        flat_idx = idx.reshape(-1).to(torch.int32).contiguous()
        row_shape = tuple(src.shape[1:])
        out = torch.empty((flat_idx.numel(),) + row_shape, dtype=src.dtype, device=src.device)
        row_bytes = src[0].numel() * src.element_size()
        with torch.cuda.device(self.device):
            check(lib().nmmo_gather_rows(_p(src), row_bytes, _p(flat_idx), flat_idx.numel(), _p(out),
                                         self._stream()), "nmmo_gather_rows")
        return out.view(tuple(idx.shape) + row_shape)
