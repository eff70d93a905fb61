"""On-disk map bank: nmmo's PATH_MAPS directory of generated maps.

The reference points nmmo at `PATH_MAPS = f"{maps_path}/{map_size}/"` with `MAP_N` maps and
`MAP_FORCE_GENERATION` (reinforcement_learning/environment.py:33,36,41; evaluate.py:64-77 uses
the pre-generated `maps/pve_eval/` and `maps/pvp_eval/` sets). nmmo keeps one directory per map,
`map{i}/map.npy` for i = 1..MAP_N, holding the 160x160 material-id grid **[recalled: nmmo 2.1
MapGenerator; not in the reference tree, maps are git-ignored]**. Map bank index m (0-based, as
drawn at reset, SPEC §4) is directory map{m+1}.

Loading accepts any integer dtype (nmmo writes the grid as a numpy int array) and never
unpickles (`allow_pickle=False`); saving writes uint8. Material ids are nmmo's 16 (SPEC §2).
"""

from __future__ import annotations

import os

import numpy as np

from . import abi


def map_file(path_maps: str, m: int) -> str:
    return os.path.join(path_maps, f"map{m + 1}", "map.npy")


def available(path_maps: str, map_n: int) -> bool:
    return all(os.path.exists(map_file(path_maps, m)) for m in range(map_n))


def load_map(path: str) -> np.ndarray:
    g = np.load(path, allow_pickle=False)
    if g.shape != (abi.MAP_SIZE, abi.MAP_SIZE):
        raise ValueError(f"{path}: map shape {g.shape} != ({abi.MAP_SIZE}, {abi.MAP_SIZE})")
    if not np.issubdtype(g.dtype, np.integer):
        raise ValueError(f"{path}: map dtype {g.dtype} is not an integer material grid")
    if g.min() < 0 or g.max() >= 16:
        raise ValueError(f"{path}: material ids outside 0..15")
    return g.astype(np.uint8)


def load_map_bank(path_maps: str, map_n: int) -> np.ndarray:
    """uint8 [map_n, 160, 160] from PATH_MAPS/map{1..map_n}/map.npy."""
    return np.stack([load_map(map_file(path_maps, m)) for m in range(map_n)])


def save_map_bank(bank: np.ndarray, path_maps: str) -> None:
    bank = np.asarray(bank)
    if bank.ndim != 3 or bank.shape[1:] != (abi.MAP_SIZE, abi.MAP_SIZE):
        raise ValueError("bank must be [map_n, 160, 160]")
    for m in range(bank.shape[0]):
        d = os.path.dirname(map_file(path_maps, m))
        os.makedirs(d, exist_ok=True)
        tmp = os.path.join(d, "map.tmp.npy")
        np.save(tmp, bank[m].astype(np.uint8), allow_pickle=False)
        os.replace(tmp, map_file(path_maps, m))


def prepare(engine) -> str:
    """nmmo's map preparation for `engine.config`: with PATH_MAPS set, load the bank from disk
    when every map file exists and MAP_FORCE_GENERATION is off; otherwise keep the generated
    bank and write it there. Returns "loaded", "generated" or "memory" (no PATH_MAPS)."""
    cfg = engine.config
    if not cfg.PATH_MAPS:
        return "memory"
    if not cfg.MAP_FORCE_GENERATION and available(cfg.PATH_MAPS, cfg.MAP_N):
        engine.set_map_bank(load_map_bank(cfg.PATH_MAPS, cfg.MAP_N))
        return "loaded"
    save_map_bank(engine.map_bank(), cfg.PATH_MAPS)
    return "generated"
