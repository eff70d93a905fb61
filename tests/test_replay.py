"""Replay files (nmmo_amd/replay.py): FileReplayHelper's reset/update/save
cycle (train_helper.py:132-134, :171, :229-235) over a stand-in env backed by the CPU oracle;
the saved .replay.lzma decodes to the realm it recorded, tick by tick. CPU only."""

import numpy as np

from nmmo_amd import abi
from nmmo_amd.config import Config
from nmmo_amd.replay import FileReplayHelper, load_replay
from oracle.oracle import OracleEnvs, split_state


class _OracleEnv:
    """The two calls the helper makes on the env: state() and engine.events(0)."""

    def __init__(self, cfg):
        self.o = OracleEnvs(cfg, 1, seed=11)
        self.engine = self
        self.o.reset()

    def events(self, env):
        return self.o.events(env)

    def state(self):
        d = split_state(self.o.get_state(), 1, self.o.S, self.o.P)
        return {"tick": int(d["env"][0, abi.E["tick"]]), "material": d["mat"][0].copy(),
                "entities": {n: d["ent"][0, i].copy() for i, n in enumerate(abi.ENTITY_FIELDS)}}

    def step(self, t):
        self.o.step(self.o.scripted_actions(t))


def test_replay_round_trip(tmp_path):
    env = _OracleEnv(Config.preset("C4", MAP_N=2))
    helper = FileReplayHelper()
    helper.set_env(env)
    helper.reset()
    states = [env.state()]
    for t in range(12):
        env.step(t)
        helper.update()
        states.append(env.state())
    path = helper.save(str(tmp_path / "replay_seed_1_x"), compress=True)
    assert path.endswith(".replay.lzma")
    rp = load_replay(path)
    assert np.array_equal(np.array(rp["map"]), states[0]["material"])
    assert len(rp["packets"]) == 13
    mat = states[0]["material"].copy()
    for pk, st in zip(rp["packets"], states):
        assert pk["tick"] == st["tick"]
        ent = st["entities"]
        live = {int(ent["id"][s]): s for s in range(len(ent["id"])) if ent["id"][s] != 0 and ent["alive"][s]}
        got = {int(k): v for k, v in {**pk["player"], **pk["npc"]}.items()}
        assert set(got) == set(live)
        for eid, s in live.items():
            assert (got[eid]["base"]["r"], got[eid]["base"]["c"]) == (int(ent["row"][s]), int(ent["col"][s]))
            assert got[eid]["resource"]["health"]["val"] == int(ent["health"][s])
        for r, c, m in pk["resource"]:  # material deltas rebuild the map of each tick
            mat[r, c] = m
        assert np.array_equal(mat, st["material"])
        assert all(row[abi.ATTR_TO_COL["tick"]] == st["tick"] for row in pk["event"])
    assert any(pk["event"] for pk in rp["packets"])
    js = helper.save(str(tmp_path / "plain"), compress=False)
    assert load_replay(js) == rp
