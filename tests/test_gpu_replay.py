"""Replay recording through the nmmo.Env facade on the HIP engine (train_helper.py:132-134,
:171, :229-235): realm.record_replay(helper), reset, steps, save -> .replay.lzma whose packets
match the realm state after every step."""

import numpy as np
import pytest

from nmmo_amd.config import Config

pytestmark = pytest.mark.gpu


def test_record_replay_via_realm(tmp_path):
    from nmmo_amd.replay import FileReplayHelper, load_replay
    from nmmo_amd.vecenv import NmmoEnv

    env = NmmoEnv(Config.preset("C4", MAP_N=2), seed=3)
    obs, _ = env.reset(seed=5)
    helper = FileReplayHelper()
    env.realm.record_replay(helper)
    helper.reset()
    rng = np.random.default_rng(0)
    positions = []
    for t in range(10):
        acts = {a: {"Move": {"Direction": int(rng.integers(0, 5))}} for a in env.agents}
        env.step(acts)
        st = env.state()
        positions.append({int(st["entities"]["id"][s]): (int(st["entities"]["row"][s]), int(st["entities"]["col"][s]))
                          for s in range(len(st["entities"]["id"]))
                          if st["entities"]["id"][s] > 0 and st["entities"]["alive"][s]})
    rp = load_replay(helper.save(str(tmp_path / "replay_seed_1"), compress=True))
    assert len(rp["packets"]) == 11
    for pk, pos in zip(rp["packets"][1:], positions):
        got = {int(k): (v["base"]["r"], v["base"]["c"]) for k, v in pk["player"].items()}
        assert got == pos
    env.close()
