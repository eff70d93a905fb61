"""Wire codec (SPEC.md §8c, csrc/wire.hip) on MI355X: nmmo_wire_pack's bytes equal the numpy
restatement's (oracle/wire.py, which derives every count from the native bytes) and
nmmo_wire_unpack restores the native obs bit-exactly, small and at C4 size (1,024 envs,
staggered episodes)."""

import numpy as np
import pytest
import torch

from tests.conftest import gpu_available

pytestmark = [pytest.mark.gpu, pytest.mark.skipif(not gpu_available(), reason="needs a GPU")]


def _engine(n, seed, map_n=4):
    from nmmo_amd import abi
    from nmmo_amd.config import Config
    from nmmo_amd.engine import NmmoEngine

    cfg = Config.preset("C4", MAP_N=map_n, early_stop_agent_num=8, obs_layout=abi.OBS_NATIVE)
    return NmmoEngine(cfg, n, seed=seed)


def test_wire_pack_matches_restatement():
    from nmmo_amd import wire
    from oracle import wire as owire

    eng = _engine(3, seed=21)
    eng.reset()
    for t in range(45):
        if t == 20:
            eng.end_episodes(np.array([0, 1, 0], bool))
        eng.scripted_actions(500 + t)
        eng.step()
        if t % 15 != 14:
            continue
        w = wire.pack(eng)
        total = wire.total_bytes(w)
        nat = eng.obs.cpu().numpy()
        ref = owire.pack(nat, eng.P)
        assert total == ref.nbytes, (t, total, ref.nbytes)
        assert np.array_equal(w[:total].cpu().numpy(), ref), f"wire bytes differ at tick {t}"
        back = wire.unpack(w, eng.n_envs, eng.P)
        assert torch.equal(back, eng.obs), f"unpack differs at tick {t}"
    eng.close()


def test_wire_roundtrip_fullsize():
    from nmmo_amd import wire

    n = 1024
    eng = _engine(n, seed=3, map_n=256)
    eng.reset()
    ids = np.arange(n)
    for k in range(24):  # staggered episode phases, as in the bench
        eng.end_episodes(ids % 24 == k)
        eng.scripted_actions(77 + k)
        eng.step()
    w = wire.pack(eng)
    back = wire.unpack(w, n, eng.P)
    assert torch.equal(back, eng.obs)
    total = wire.total_bytes(w)
    assert total * 4 < eng.obs.numel(), (total, eng.obs.numel())
    eng.close()
