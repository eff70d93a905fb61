"""Drop-in vectorized env for the reference trainer (pufferlib 0.7.3 pool protocol) and a
PettingZoo-style single-env facade (nmmo.Env protocol), both backed by the HIP engine.

Protocol 2 — what `reinforcement_learning/clean_pufferl.py` consumes:
    pool = GpuVecEnv(env_creator, env_kwargs=..., num_envs=..., envs_per_worker=...,
                     envs_per_batch=..., env_pool=..., mask_agents=True)   # :106-114
    pool.single_observation_space.shape, pool.single_action_space.shape    # :116-117
    pool.agents_per_env, pool.envs_per_batch, pool.driver_env              # :118,134-136,151
    pool.async_reset(seed)                                                 # :175
    o, r, d, t, infos, env_id, mask = pool.recv()                          # :293
    pool.send(actions)                                                     # :357
    pool.close()                                                           # :563
The async env pool of the reference's default config (`num_envs: 15, envs_per_batch: 6,
env_pool: True`, config.yaml:35-38) is served with a fixed ready order (SPEC §14): envs become
ready in the order they were sent, i.e. a FIFO queue that `async_reset` fills with 0..num_envs-1;
`recv` pops the first `envs_per_batch` envs and returns their `envs_per_batch * 128` rows, with
`env_id` the agent slots `env * 128 + agent` of those envs (clean_pufferl.py:158,310-315,346);
`send` steps exactly those envs (nmmo_step_envs: one launch over the listed envs, the others keep
their state) and appends them to the queue. That is the order a pufferlib pool of equally fast
workers produces; with `envs_per_batch == num_envs` it is plain lockstep.
Differences by design: `recv` returns device tensors for the observations (the trainer's
`torch.as_tensor(o).to(device)` at :302,318 is then a no-op instead of an H2D copy); `mask` is a
host numpy bool array because the trainer combines it with host arrays (:306,334).

The obs contract at this boundary. `recv` hands out views of the engine's own obs buffer (a
batch of contiguous envs), which the engine writes incrementally (nmmo_obs_bind: a row stores only
what differs from what the buffer already holds). In the reference the trainer's `.to(device)`
copies the shared-memory rows, so a policy may edit its input in place -- the start-kit's
TileEncoder does (`tile[:, :, :2] -= ...; += 7`, baseline_policy.py:96-97, on
unpack_batched_obs views); the takeru and yaofeng policies only read theirs. `obs_writes` names
the sections a consumer writes into: before `send` steps the envs whose rows the last `recv`
handed out, their state for those sections is forgotten, so every `recv` returns the bytes of a
full write whatever the consumer did to the previous ones:
  - `{"Tile"}`: only the Tile sections are rewritten in full next step (nmmo_obs_invalidate_sections);
    every other section stays incremental;
  - `set()` (or `obs_readonly=True`): the consumer writes nothing; the rows stay incremental;
  - `"all"`: whole rows are rewritten (nmmo_obs_invalidate_envs; the full-write cost).
The default (`obs_writes=None`) is what the policy of the agent env_creator names writes
(`AGENT_OBS_WRITES`: the start-kit `{"Tile"}`, takeru / yaofeng nothing), and `"all"` when no agent
is named. A batch that wraps around the env range is returned as a copy and needs none of it.

Protocol 1 — `NmmoEnv` exposes `reset(seed)` / `step(actions)` with per-agent dict
observations (the unflattened layout) like `nmmo.Env`, for wrappers such as
`reinforcement_learning/stat_wrapper.py` (the realm facade is partial: see `NmmoEnv.realm`).
"""

from __future__ import annotations

import collections
import ctypes

import numpy as np
import torch

from . import abi, layout
from .config import Config
from .engine import NmmoEngine


class Box:
    """Minimal gym.spaces.Box stand-in (gymnasium is not installed in this image)."""

    def __init__(self, low, high, shape, dtype):
        self.low, self.high, self.shape, self.dtype = low, high, tuple(shape), np.dtype(dtype)

    def __repr__(self):
        return f"Box({self.shape}, {self.dtype})"


class MultiDiscrete:
    def __init__(self, nvec):
        self.nvec = np.asarray(nvec, dtype=np.int64)
        self.shape = self.nvec.shape
        self.dtype = np.dtype(np.int64)

    def sample(self, rng=None):
        rng = rng or np.random.default_rng()
        return (rng.random(self.shape) * self.nvec).astype(np.int64)

    def __repr__(self):
        return f"MultiDiscrete({self.nvec.tolist()})"


class DriverEnv:
    """The attributes the reference reads off `pool.driver_env` (clean_pufferl.py:134-136,
    baseline_policy.py:28): unflatten_context, obs_sz, possible_agents, spaces."""

    def __init__(self, config: Config, obs_elems: int):
        self.config = config
        self.obs_sz = obs_elems
        self.possible_agents = list(range(1, config.PLAYER_N + 1))
        self.unflatten_context = layout.flat_layout(config.TASK_EMBED_DIM)
        self.single_observation_space = Box(-2**20, 2**20, (obs_elems,), np.float32)
        self.single_action_space = MultiDiscrete(layout.ACTION_DIMS)

    def unflatten(self, flat):
        return layout.unflatten(flat, self.config.TASK_EMBED_DIM)


def reset_seeds(seed: int, env_index_base: int, n: int) -> np.ndarray:
    """Per-env reset seeds of pool.async_reset(seed) (clean_pufferl.py:175): env i of a shard
    whose first global env index is env_index_base gets seed + env_index_base + i, so the
    shards of a multi-GPU pool reset exactly the envs one pool of all envs would."""
    return (np.uint64(seed) + np.uint64(env_index_base) + np.arange(n, dtype=np.uint64)).astype(np.uint64)


def _config_from_kwargs(env_kwargs) -> Config:
    if isinstance(env_kwargs, Config):
        return env_kwargs
    if env_kwargs and "env" in env_kwargs:  # environment.py:57 passes kwargs["env"]
        return Config(env_kwargs["env"])
    return Config()


def _as_dict(ns) -> dict:
    """The reward_wrapper kwargs: a dict, or the pufferlib.namespace train.py builds (:105,209)."""
    if ns is None:
        return {}
    if isinstance(ns, dict):
        return dict(ns)
    return dict(vars(ns))


# What each reference agent's Policy writes into its observation input in place (agent_zoo/<agent>):
# the start-kit TileEncoder edits Tile[:, :, :2] (neurips23_start_kit/baseline_policy.py:96-97); the
# takeru (ReducedTileEncoder slices, policy.py:85-97) and yaofeng (policy.py:91-106) policies only read.
AGENT_OBS_WRITES = {"neurips23_start_kit": frozenset({"Tile"}), "takeru": frozenset(), "yaofeng": frozenset()}
OBS_SECTIONS = {"Tile": abi.OBS_SEC_TILE}


def resolve_obs_writes(agent, obs_writes=None, obs_readonly=False):
    """GpuVecEnv's obs_writes: frozenset of section names or "all" (module docstring)."""
    if obs_readonly:
        return frozenset()
    if obs_writes is None:
        return AGENT_OBS_WRITES.get(agent, "all")
    if obs_writes == "all":
        return "all"
    if isinstance(obs_writes, str):
        raise ValueError('obs_writes: a set of section names (e.g. {"Tile"}), "all" or None')
    names = frozenset(obs_writes)
    known = {k for k in layout.flat_layout() if k != "__total__"} | {"ActionTargets"}
    unknown = names - known
    if unknown:
        raise ValueError(f"obs_writes: unknown obs sections {sorted(unknown)}")
    return names


def agent_from_creator(env_creator):
    """The agent whose RewardWrapper `environment.make_env_creator(reward_wrapper_cls=...)`
    closed over (environment.py:50-58, train.py:226): `agent_zoo.<agent>.reward_wrapper` ->
    "<agent>" (None when env_creator is not such a closure). A Syllabus creator
    (syllabus_wrapper.make_syllabus_env_creator) is refused: curricula run on the device through
    NmmoEngine.set_curriculum instead."""
    cells = getattr(env_creator, "__closure__", None) or ()
    names = getattr(getattr(env_creator, "__code__", None), "co_freevars", ())
    agent = None
    for name, cell in zip(names, cells):
        try:
            v = cell.cell_contents
        except ValueError:
            continue
        if name == "syllabus" and v is not None:
            raise ValueError("a Syllabus env_creator: use NmmoEngine.set_curriculum on the pool's engine")
        mod = getattr(v, "__module__", "") or ""
        if isinstance(v, type) and mod.startswith("agent_zoo."):
            agent = mod.split(".")[1]
    return agent


class GpuVecEnv:
    """pufferlib-0.7.3 pool protocol over one NmmoEngine: lockstep (envs_per_batch == num_envs)
    or the async env pool (envs_per_batch < num_envs) with the FIFO ready order of SPEC §14."""

    def __init__(self, env_creator=None, env_kwargs=None, num_envs=1, envs_per_worker=1,
                 envs_per_batch=None, env_pool=False, mask_agents=True, *, config=None,
                 device=None, seed=0, task_embedding=None, env_index_base=0, agent=None,
                 obs_readonly=False, obs_writes=None):
        """obs_writes: the obs sections the consumer writes into in place (module docstring): a set
        of section names, "all", or None = what the named agent's policy writes (AGENT_OBS_WRITES;
        "all" without an agent). obs_readonly=True is obs_writes=set()."""
        del envs_per_worker  # the engine replaces workers
        self._views_out = False  # the last recv() handed out views of the engine's obs buffer
        self.config = config or _config_from_kwargs(env_kwargs)
        rw = _as_dict(env_kwargs.get("reward_wrapper")) if isinstance(env_kwargs, dict) else {}
        if config is None and "early_stop_agent_num" in rw:  # BaseStatWrapper's early stop (stat_wrapper.py:68-69)
            self.config.early_stop_agent_num = int(rw["early_stop_agent_num"])
        if agent is None:  # env_creator's RewardWrapper (environment.py:58), when it names one
            agent = agent_from_creator(env_creator)
        self.obs_writes = resolve_obs_writes(agent, obs_writes, obs_readonly)
        self.obs_readonly = self.obs_writes == frozenset()
        if self.config.obs_layout != abi.OBS_FLAT:
            raise ValueError("GpuVecEnv serves flat observations (obs_layout=OBS_FLAT)")
        self.num_envs = int(num_envs)
        epb = self.num_envs if envs_per_batch is None else int(envs_per_batch)
        if not 1 <= epb <= self.num_envs:
            raise ValueError(f"envs_per_batch must be in 1..num_envs ({self.num_envs}), got {envs_per_batch}")
        if not env_pool and self.num_envs % epb:
            # without the env pool, pufferlib steps fixed batches of envs_per_batch envs
            raise ValueError(f"num_envs ({self.num_envs}) must be a multiple of envs_per_batch ({epb}) "
                             f"unless env_pool=True")
        self.envs_per_batch = epb
        self.env_pool = bool(env_pool)
        self.mask_agents = mask_agents
        self.engine = NmmoEngine(self.config, self.num_envs, seed=seed, device=device,
                                 task_embedding=task_embedding, env_index_base=env_index_base)
        # env_creator's RewardWrapper (environment.py:58) with the YAML reward_wrapper kwargs,
        # run on the device (SPEC §13); agent=None keeps the bare env
        self.stat_prefix = rw.get("stat_prefix")
        if agent is not None:
            from .wrappers import wrapper_config

            self.engine.set_wrapper(wrapper_config(agent, **rw))
        self.agents_per_env = self.config.PLAYER_N
        self.driver_env = DriverEnv(self.config, self.engine.obs_elems)
        self.single_observation_space = self.driver_env.single_observation_space
        self.single_action_space = self.driver_env.single_action_space
        self._seed = seed
        self.env_index_base = int(env_index_base)
        self._ready: collections.deque | None = None  # envs whose outputs await recv, in ready order
        self._batch: list | None = None               # envs returned by the last recv, awaiting send
        P, d = self.agents_per_env, self.engine.device
        if epb < self.num_envs:  # batch-shaped outputs for batches that wrap around the env range
            self._obs_b = torch.empty((epb, P, self.engine.obs_elems), dtype=torch.float32, device=d)
            self._ids_host = torch.empty(epb, dtype=torch.int32).pin_memory()
            self._ids = torch.empty(epb, dtype=torch.int32, device=d)

    # -- protocol
    def _forget(self, ids=None):
        """Forget what the consumer may have written into the rows the last recv() handed out
        (ids: their envs on the device; None = every env), as obs_writes says."""
        e = self.engine
        if not self._views_out or self.obs_readonly:
            return
        if self.obs_writes == "all" or any(s not in OBS_SECTIONS for s in self.obs_writes):
            if ids is None:
                e.obs_invalidate()
            else:
                e.obs_invalidate_envs(ids)
        else:
            e.obs_invalidate_sections(sum(OBS_SECTIONS[s] for s in self.obs_writes), ids)

    def async_reset(self, seed=None):
        self._forget()  # the reset writes into the same rows
        self._views_out = False
        if seed is not None:
            self.engine.reset(reset_seeds(seed, self.env_index_base, self.num_envs))
        else:
            self.engine.reset()
        self._ready = collections.deque(range(self.num_envs))
        self._batch = None

    def recv(self):
        if self._ready is None:
            raise RuntimeError("recv() before async_reset()")
        if self._batch is not None:
            raise RuntimeError("recv() twice without send(): the batch it returned is still out")
        k, P, e = self.envs_per_batch, self.agents_per_env, self.engine
        batch = [self._ready.popleft() for _ in range(k)]
        self._batch = batch
        N = k * P
        lo = batch[0]
        if batch == list(range(lo, lo + k)):  # contiguous envs: views of the engine's buffers
            sl = slice(lo, lo + k)
            o = e.obs[sl].view(N, e.obs_elems)
            self._views_out = True
            r, d, t, m = (x[sl].reshape(N) for x in (e.rew, e.term, e.trunc, e.mask))
        else:  # the batch wraps around: gather its env rows (nmmo_gather_rows)
            idx = torch.as_tensor(batch, dtype=torch.int32).to(e.device)
            row_bytes = P * e.obs_elems * 4
            from ._native import check, lib

            with torch.cuda.device(e.device):
                check(lib().nmmo_gather_rows(ctypes.c_void_p(e.obs.data_ptr()), row_bytes,
                                             ctypes.c_void_p(idx.data_ptr()), k,
                                             ctypes.c_void_p(self._obs_b.data_ptr()),
                                             ctypes.c_void_p(torch.cuda.current_stream(e.device).cuda_stream)),
                      "nmmo_gather_rows")
            o = self._obs_b.view(N, e.obs_elems)
            self._views_out = False  # a copy: the engine's rows were not handed out
            il = idx.long()
            r, d, t, m = (x.index_select(0, il).reshape(N) for x in (e.rew, e.term, e.trunc, e.mask))
        mask = m.to(torch.bool).cpu().numpy()  # the host sync of this step
        e.check_fault("GpuVecEnv.recv")
        env_id = (np.asarray(batch, np.int64)[:, None] * P + np.arange(P)).reshape(-1)
        return o, r, d, t, self._infos(batch), env_id, mask

    def _infos(self, batch):
        """Per env of the batch {agent_id: info} of the agents whose episode ended this step
        (BaseStatWrapper's info dicts, stat_wrapper.py:128-185); empty dicts without the wrapper
        layer. Only the records of finished agents cross to the host."""
        e = self.engine
        if e.info is None:
            return [{} for _ in batch]
        from .wrappers import infos_from_records

        il = torch.as_tensor(batch, dtype=torch.long, device=e.device)
        done = (e.term.index_select(0, il) | e.trunc.index_select(0, il)).view(-1).nonzero().view(-1)
        recs = np.zeros((len(batch), self.agents_per_env), abi.agent_info_dtype())
        if done.numel():
            info = e.info.index_select(0, il)
            rows = info.view(-1, info.shape[-1]).index_select(0, done).cpu().numpy()
            idx = done.cpu().numpy()
            recs.reshape(-1)[idx] = rows.view(abi.agent_info_dtype()).reshape(-1)
        return infos_from_records(recs, stat_prefix=self.stat_prefix)

    def send(self, actions):
        if self._batch is None:
            raise RuntimeError("send() without a recv() batch to step")
        batch, k, P, e = self._batch, self.envs_per_batch, self.agents_per_env, self.engine
        a = torch.as_tensor(actions)
        a = a.to(device=e.device, dtype=torch.int32).reshape(k, P, abi.N_ACTION_HEADS)
        if k == self.num_envs:  # lockstep (every recv returns 0..num_envs-1 in order)
            self._forget()  # the consumer may have edited the rows recv handed out
            e.step(a)
        else:
            lo = batch[0]
            if batch == list(range(lo, lo + k)):
                e.actions[lo:lo + k].copy_(a)
            else:
                e.actions.index_copy_(0, torch.as_tensor(batch, dtype=torch.long, device=e.device), a)
            self._ids_host.copy_(torch.as_tensor(batch, dtype=torch.int32))
            self._ids.copy_(self._ids_host, non_blocking=True)
            self._forget(self._ids)
            e.step_envs(self._ids)
        self._views_out = False
        self._ready.extend(batch)
        self._batch = None

    def close(self):
        self.engine.close()

    # -- helpers
    def unflatten_obs(self):
        return self.driver_env.unflatten(self.engine.obs)


class NmmoEnv:
    """PettingZoo-ParallelEnv-shaped facade over a 1-env engine (nmmo.Env protocol).

    reset(seed) -> (obs, infos); step(actions: {agent_id: int[12] or dict}) ->
    (obs, rewards, terminated, truncated, infos); obs[agent] is the unflattened dict of numpy
    arrays (Tile, Entity, Inventory, Market, Task, AgentId, CurrentTick, ActionTargets)."""

    def __init__(self, config: Config | None = None, seed: int = 0, device=None, task_embedding=None):
        self.config = config or Config()
        self.config.obs_layout = abi.OBS_FLAT
        self.engine = NmmoEngine(self.config, 1, seed=seed, device=device,
                                 task_embedding=task_embedding)
        self.possible_agents = list(range(1, self.config.PLAYER_N + 1))
        self.agents: list[int] = []
        self._obs_space = Box(-2**20, 2**20, (self.engine.obs_elems,), np.float32)
        self._act_space = MultiDiscrete(layout.ACTION_DIMS)
        # state / realm / tasks of the current tick, read from the device once per tick
        # (BaseStatWrapper reads env.realm once per agent per step, stat_wrapper.py:122-123);
        # reset() and step() invalidate it
        self._tick_cache: dict = {}

    def observation_space(self, agent):
        return self._obs_space

    def action_space(self, agent):
        return self._act_space

    def _obs_dict(self, mask):
        flat = self.engine.obs[0].cpu().numpy()
        d = layout.unflatten(flat, self.config.TASK_EMBED_DIM)
        out = {}
        for i, a in enumerate(self.possible_agents):
            if mask[i]:
                out[a] = _index(d, i)
        return out

    def reset(self, seed=None, options=None):
        self._tick_cache = {}
        self.engine.reset(None if seed is None else np.array([seed], dtype=np.uint64))
        mask = self.engine.mask[0].cpu().numpy()
        self.agents = [a for i, a in enumerate(self.possible_agents) if mask[i]]
        return self._obs_dict(mask), {a: {} for a in self.agents}

    def step(self, actions):
        buf = np.zeros((1, self.config.PLAYER_N, abi.N_ACTION_HEADS), np.int32)
        buf[0, :, 1] = layout.PLAYER_N_OBS  # noop defaults
        buf[0, :, 8] = 4
        for a, act in actions.items():
            if isinstance(act, dict):
                act = flatten_action(act)
            buf[0, a - 1] = np.asarray(act, dtype=np.int32)
        self._tick_cache = {}
        self.engine.step(torch.from_numpy(buf).to(self.engine.device))
        e = self.engine
        mask = e.mask[0].cpu().numpy()
        rew, term, trunc = (x[0].cpu().numpy() for x in (e.rew, e.term, e.trunc))
        present = [a for i, a in enumerate(self.possible_agents) if mask[i]]
        obs = self._obs_dict(mask)
        rewards = {a: float(rew[a - 1]) for a in present}
        terms = {a: bool(term[a - 1]) for a in present}
        truncs = {a: bool(trunc[a - 1]) for a in present}
        self.agents = [a for a in present if not (terms[a] or truncs[a])]
        if getattr(self, "_replay", None) is not None:
            self._replay.update()
        return obs, rewards, terms, truncs, {a: {} for a in present}

    @property
    def realm(self):
        """Realm facade: `realm.tick`, `realm.players` (id -> entity, with `dead_this_tick`),
        `realm.npcs` and `realm.event_log` — the reads of stat_wrapper.py:122-185, 216-285 and
        train_helper.py:133-166."""
        if "realm" not in self._tick_cache:
            self._tick_cache["realm"] = _Realm(self.state(), self.engine.events(0), env=self)
        return self._tick_cache["realm"]

    @property
    def max_num_agents(self) -> int:
        return self.config.PLAYER_N

    @property
    def tasks(self) -> list:
        """One Task per agent in possible_agents order (nmmo.Env.tasks)."""
        if "tasks" not in self._tick_cache:
            names = getattr(self.engine, "task_names", None) or [default_spec_name(self.config)]
            self._tick_cache["tasks"] = tasks_from_state(self.state(), self.possible_agents, names,
                                                         self.engine.task_table)
        return self._tick_cache["tasks"]

    @property
    def agent_task_map(self) -> dict:
        """agent id -> [Task] (nmmo.Env.agent_task_map, read at stat_wrapper.py:155)."""
        if "task_map" not in self._tick_cache:
            self._tick_cache["task_map"] = {t.assignee[0]: [t] for t in self.tasks}
        return self._tick_cache["task_map"]

    def state(self) -> dict:
        """The env's parsed state blob (nmmo_get_state), read once per tick."""
        if "state" not in self._tick_cache:
            st = self.engine.get_state()
            self._tick_cache["state"] = parse_env_state(st, self.engine.S, self.config.PLAYER_N)
        return self._tick_cache["state"]

    def record_replay(self, helper):
        """realm.record_replay(replay_helper) (train_helper.py:134): the helper is updated after
        every step (nmmo_amd/replay.py)."""
        helper.set_env(self)
        self._replay = helper

    def close(self):
        self.engine.close()


def flatten_action(act: dict) -> np.ndarray:
    """{"Move": {"Direction": 2}, "Attack": {"Style": 0, "Target": 5}, ...} -> int[12] in the
    MultiDiscrete head order (takeru/policy.py:293-307); absent heads take their noop."""
    out = np.array([0, 100, 1024, 12, 12, 100, 0, 100, 4, 12, 0, 12], dtype=np.int32)
    for i, ((a, b), _) in enumerate(layout.ACTION_HEADS):
        if a in act and b in act[a]:
            out[i] = int(act[a][b])
    return out


def parse_env_state(blob: np.ndarray, S: int, P: int, env: int = 0) -> dict:
    """One env of an nmmo_get_state blob (include/nmmo_hip.h) as named arrays."""
    per = abi.state_bytes_per_env(S, P)
    b = blob[env * per:(env + 1) * per]
    o = 0
    E = b[o:o + abi.NE * 4].copy().view(np.int32); o += abi.NE * 4
    ent = b[o:o + abi.NF * S * 2].copy().view(np.int16).reshape(abi.NF, S); o += abi.NF * S * 2
    o += S * 2  # free datastore-row ring
    mat = b[o:o + abi.MAP_TILES].reshape(abi.MAP_SIZE, abi.MAP_SIZE).copy(); o += abi.MAP_TILES
    ni = P * abi.INV_SLOTS
    items = b[o:o + ni * 8].copy().view(np.uint32).reshape(P, abi.INV_SLOTS, 2); o += ni * 8
    o += ni * 2  # item-row ring
    assign = b[o:o + P * 4].copy().view(np.int32); o += P * 4
    tstate = b[o:o + P * abi.TASK_STATE_BYTES].copy().view(abi.task_state_dtype())
    return {"tick": int(E[abi.E["tick"]]), "env": E, "material": mat, "items": items,
            "assign": assign, "tstate": tstate,
            "entities": {n: ent[i].copy() for i, n in enumerate(abi.ENTITY_FIELDS)}}


def default_spec_name(config) -> str:
    from .tasks import spec_name

    return spec_name("TickGE", num_tick=config.task_num_tick)


def tasks_from_state(st: dict, possible_agents, names, embeddings=None) -> list:
    """Task facades of one env (parse_env_state) in possible_agents order."""
    out = []
    for i, a in enumerate(possible_agents):
        k = int(st["assign"][i])
        out.append(Task((a,), names[k] if k < len(names) else names[0], st["tstate"][i],
                        None if embeddings is None else embeddings[min(k, len(embeddings) - 1)]))
    return out


class Val(int):
    """An int entity attribute that also answers `.val` (nmmo's datastore-backed attributes are
    read as `agent.food.val` at stat_wrapper.py:146-175)."""

    @property
    def val(self) -> int:
        return int(self)


class _Entity:
    """One entity row: every entity-table field is a Val attribute (alive, health, food, ...),
    plus nmmo's derived `attack_level` (max melee/range/mage level, stat_wrapper.py:170) and a
    settable `name` (train_helper.py:147)."""

    def __init__(self, cols: dict, slot: int):
        for k, v in cols.items():
            setattr(self, k, Val(int(v[slot])))
        self.ent_id = int(self.id)
        self.name = f"{'Player' if self.ent_id > 0 else 'NPC'}_{self.ent_id}"

    @property
    def attack_level(self) -> int:
        return int(max(self.melee_level, self.range_level, self.mage_level))


class _Players(dict):
    """realm.players: id -> entity of live players, plus `dead_this_tick` (id -> entity of the
    players culled by the last tick, still readable: stat_wrapper.py:136)."""

    def __init__(self, live: dict, dead_this_tick: dict):
        super().__init__(live)
        self.dead_this_tick = dead_this_tick


class Task:
    """nmmo.task.task_api.Task facade over the engine's per-agent task state (SPEC §12): the
    fields stat_wrapper.py:155-163 and train_helper.py:201-225 read."""

    def __init__(self, assignee, spec_name: str, ts, embedding=None):
        self.assignee = tuple(assignee)
        self.spec_name = spec_name
        self._max_progress = float(ts["max_progress"])
        self.reward_signal_count = int(ts["signals"])
        self.completed = bool(ts["completed_tick"] > 0)
        self.embedding = embedding
        self.progress_info = {"max_progress": self._max_progress,
                              "completed_tick": int(ts["completed_tick"])}

    def __repr__(self):
        return f"Task({self.spec_name}, assignee={self.assignee}, max_progress={self._max_progress})"


class EventLog:
    """realm.event_log facade (nmmo.lib.event_log.EventLogger as read by stat_wrapper.py:123,
    218-219): get_data(agents=[...], tick=None|-1|t) and attr_to_col over the engine's ring."""

    def __init__(self, rows: np.ndarray, tick: int):
        self._rows = rows
        self._tick = tick
        self.attr_to_col = dict(abi.ATTR_TO_COL)

    def get_data(self, agents=None, event_code=None, tick=None) -> np.ndarray:
        r = self._rows
        if agents is not None:
            r = r[np.isin(r[:, abi.ATTR_TO_COL["ent_id"]], list(agents))]
        if event_code is not None:
            r = r[r[:, abi.ATTR_TO_COL["event"]] == event_code]
        if tick is not None:
            t = self._tick if tick == -1 else tick
            r = r[r[:, abi.ATTR_TO_COL["tick"]] == t]
        return r


class _Realm:
    def __init__(self, st: dict, events: np.ndarray | None = None, env=None):
        self._env = env
        self.tick = st["tick"]
        self.event_log = EventLog(np.zeros((0, abi.EVENT_COLS), np.int32) if events is None else events,
                                  self.tick)
        ent = st["entities"]
        ids, alive, died = ent["id"], ent["alive"], ent["died_tick"]
        live = {int(ids[s]): _Entity(ent, s) for s in range(len(ids)) if ids[s] > 0 and alive[s]}
        dead = {int(ids[s]): _Entity(ent, s) for s in range(len(ids))
                if ids[s] > 0 and not alive[s] and self.tick > 0 and died[s] == self.tick}
        self.players = _Players(live, dead)
        self.npcs = {int(ent["id"][s]): _Entity(ent, s) for s in range(len(ent["id"]))
                     if ent["id"][s] < 0 and ent["alive"][s]}

    def record_replay(self, helper):
        self._env.record_replay(helper)


def _index(d, i):
    if isinstance(d, dict):
        return {k: _index(v, i) for k, v in d.items()}
    return d[i]
