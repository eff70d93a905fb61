"""Env configuration, mirroring the reference's nmmo Config.

Reference: reinforcement_learning/environment.py:14-49 (the Config mixin of 10 systems and its 16
`.set(...)` overrides) fed from config.yaml `env:` (config.yaml:75-86). `Config(env_args)` takes
the same Namespace the reference builds (`num_agents`, `num_npcs`, `max_episode_length`,
`num_maps`, `task_size`, `spawn_immunity`, `resilient_population`, ...).
"""

from __future__ import annotations

import dataclasses
from argparse import Namespace

from . import abi

SYSTEM_BITS = {
    "Resource": abi.SYS_RESOURCE,
    "Combat": abi.SYS_COMBAT,
    "NPC": abi.SYS_NPC,
    "Progression": abi.SYS_PROGRESSION,
    "Item": abi.SYS_ITEM,
    "Equipment": abi.SYS_EQUIPMENT,
    "Profession": abi.SYS_PROFESSION,
    "Exchange": abi.SYS_EXCHANGE,
}

# BASELINE.json configs -> enabled systems
PRESETS = {
    "C2": ("Resource",),
    "C3": ("Resource", "Combat", "NPC", "Progression"),
    "C4": tuple(SYSTEM_BITS),
}


@dataclasses.dataclass
class Config:
    """nmmo Config subset used by the hot path (environment.py:31-49 names in comments)."""

    PLAYER_N: int = 128                  # env_args.num_agents
    NPC_N: int = 256                     # env_args.num_npcs
    HORIZON: int = 1024                  # env_args.max_episode_length
    MAP_N: int = 256                     # env_args.num_maps
    MAP_CENTER: int = 128                # env_args.map_size (fixed: 160x160 incl. border)
    TASK_EMBED_DIM: int = 2048           # env_args.task_size
    COMBAT_SPAWN_IMMUNITY: int = 20      # env_args.spawn_immunity
    RESOURCE_RESILIENT_POPULATION: float = 0.2  # env_args.resilient_population
    PROVIDE_ACTION_TARGETS: bool = True
    PROVIDE_NOOP_ACTION_TARGET: bool = True
    PLAYER_DEATH_FOG: int | None = None  # only None is supported
    systems: tuple = tuple(SYSTEM_BITS)
    early_stop_agent_num: int = 0        # BaseStatWrapper (stat_wrapper.py:68-69)
    task_num_tick: int = 1024            # default task TickGE(num_tick)
    event_cap: int = 4096                # event-log ring rows per env (SPEC §11), 0 = off
    obs_layout: int = abi.OBS_FLAT
    map_seed: int = 0
    PATH_MAPS: str | None = None         # f"{maps_path}/{map_size}/" (environment.py:41); None = in memory
    MAP_FORCE_GENERATION: bool = False   # env_args.map_force_generation (environment.py:33)

    def __init__(self, env_args: Namespace | None = None, **overrides):
        for f in dataclasses.fields(self):
            setattr(self, f.name, f.default)
        if env_args is not None:
            mapping = {
                "num_agents": "PLAYER_N", "num_npcs": "NPC_N",
                "max_episode_length": "HORIZON", "num_maps": "MAP_N",
                "map_size": "MAP_CENTER", "task_size": "TASK_EMBED_DIM",
                "spawn_immunity": "COMBAT_SPAWN_IMMUNITY",
                "resilient_population": "RESOURCE_RESILIENT_POPULATION",
                "death_fog_tick": "PLAYER_DEATH_FOG",
            }
            for k, v in vars(env_args).items():
                if k in mapping:
                    setattr(self, mapping[k], v)
            if getattr(env_args, "maps_path", None):
                self.PATH_MAPS = f"{env_args.maps_path}/{getattr(env_args, 'map_size', self.MAP_CENTER)}/"
            if hasattr(env_args, "map_force_generation"):
                self.MAP_FORCE_GENERATION = bool(env_args.map_force_generation)
        for k, v in overrides.items():
            if not hasattr(self, k):
                raise AttributeError(f"unknown config key {k}")
            setattr(self, k, v)
        self.validate()

    def set(self, key, value):
        """nmmo Config.set (environment.py:31-49 style)."""
        if not hasattr(self, key):
            raise AttributeError(f"unknown config key {key}")
        setattr(self, key, value)
        self.validate()

    @classmethod
    def preset(cls, name: str, **overrides):
        return cls(systems=PRESETS[name], **overrides)

    def validate(self):
        if self.MAP_CENTER != 128:
            raise ValueError("only MAP_CENTER=128 (160x160 maps) is supported")
        if not (0 < self.PLAYER_N <= 128):
            raise ValueError("PLAYER_N must be in 1..128")
        if not (0 <= self.NPC_N <= 256):
            raise ValueError("NPC_N must be in 0..256")
        if self.PLAYER_DEATH_FOG is not None:
            raise ValueError("PLAYER_DEATH_FOG is not supported (reference default: None)")
        for s in self.systems:
            if s not in SYSTEM_BITS:
                raise ValueError(f"unknown system {s}")

    @property
    def system_bits(self) -> int:
        bits = 0
        for s in self.systems:
            bits |= SYSTEM_BITS[s]
        return bits

    def to_c(self, env_index_base: int = 0) -> abi.NmmoConfig:
        c = abi.NmmoConfig()
        c.abi_version = abi.ABI_VERSION
        c.player_n = self.PLAYER_N
        c.npc_n = self.NPC_N
        c.horizon = self.HORIZON
        c.map_n = self.MAP_N
        c.spawn_immunity = self.COMBAT_SPAWN_IMMUNITY
        c.early_stop_agent_num = self.early_stop_agent_num
        c.resilient_u32 = min(int(self.RESOURCE_RESILIENT_POPULATION * 2**32), 2**32 - 1)
        c.systems = self.system_bits
        c.obs_layout = self.obs_layout
        c.task_embed_dim = self.TASK_EMBED_DIM
        c.task_num_tick = self.task_num_tick
        c.event_cap = self.event_cap
        c.map_seed = self.map_seed
        c.env_index_base = env_index_base
        return c
