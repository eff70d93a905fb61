"""On-disk map bank (nmmo_amd/maps.py): PATH_MAPS/map{i}/map.npy round
trips, rejects malformed files without unpickling, and a bank loaded from disk drives the
CPU oracle exactly like the same bank in memory. CPU only."""

import os
from argparse import Namespace

import numpy as np
import pytest

from nmmo_amd import maps
from nmmo_amd.config import Config
from oracle.oracle import OracleEnvs


def test_config_path_maps_from_env_args():
    ns = Namespace(num_agents=128, num_maps=4, map_size=128, maps_path="maps/train/", map_force_generation=True)
    c = Config(ns)
    assert c.PATH_MAPS == "maps/train//128/"  # environment.py:41 f"{maps_path}/{map_size}/"
    assert c.MAP_FORCE_GENERATION is True
    assert Config().PATH_MAPS is None


def test_save_load_round_trip(tmp_path):
    o = OracleEnvs(Config.preset("C2", MAP_N=3), 1, seed=0)
    bank = o.map_bank()
    maps.save_map_bank(bank, str(tmp_path))
    assert sorted(os.listdir(tmp_path)) == ["map1", "map2", "map3"]
    assert maps.available(str(tmp_path), 3) and not maps.available(str(tmp_path), 4)
    assert np.array_equal(maps.load_map_bank(str(tmp_path), 3), bank)
    # nmmo writes an int64 grid: accepted, same materials
    np.save(maps.map_file(str(tmp_path), 1), bank[1].astype(np.int64))
    assert np.array_equal(maps.load_map_bank(str(tmp_path), 3), bank)


def test_malformed_maps_rejected(tmp_path):
    p = str(tmp_path / "m.npy")
    np.save(p, np.zeros((10, 10), np.uint8))
    with pytest.raises(ValueError, match="shape"):
        maps.load_map(p)
    np.save(p, np.full((160, 160), 16, np.uint8))
    with pytest.raises(ValueError, match="material"):
        maps.load_map(p)
    np.save(p, np.array([{"a": 1}], dtype=object), allow_pickle=True)
    with pytest.raises(ValueError):  # object arrays need pickle: refused
        maps.load_map(p)


def test_loaded_bank_drives_the_oracle(tmp_path):
    cfg = Config.preset("C4", MAP_N=2)
    src = OracleEnvs(cfg, 1, seed=4).map_bank()
    foreign = np.ascontiguousarray(src[:, ::-1, :].transpose(0, 2, 1))  # still valid nmmo maps
    maps.save_map_bank(foreign, str(tmp_path))
    a = OracleEnvs(cfg, 2, seed=4)
    a.set_map_bank(maps.load_map_bank(str(tmp_path), 2))
    b = OracleEnvs(cfg, 2, seed=4)
    b.set_map_bank(foreign)
    c = OracleEnvs(cfg, 2, seed=4)
    for o in (a, b, c):
        o.reset()
    for t in range(20):
        for o in (a, b, c):
            o.step(o.scripted_actions(t))
    assert np.array_equal(a.get_state(), b.get_state())
    assert not np.array_equal(a.get_state(), c.get_state())
    with pytest.raises(ValueError):
        a.set_map_bank(np.full((2, 160, 160), 200, np.uint8))
