"""HIP path vs the CPU oracle, bit-exact (SPEC.md v1). Calls go through the C-ABI
(libnmmo_hip.so via nmmo_amd.engine); the oracle is only the checker."""

import numpy as np
import pytest

from nmmo_amd import abi
from nmmo_amd.config import Config
from oracle.oracle import OracleEnvs, split_state

pytestmark = pytest.mark.gpu


def _engine(cfg, n_envs, seed, task=None):
    import torch

    from nmmo_amd.engine import NmmoEngine

    assert torch.cuda.is_available()
    return NmmoEngine(cfg, n_envs, seed=seed, task_embedding=task)


def _cmp_state(ga, oa, n, S, where, P=128):
    g = split_state(ga, n, S, P)
    o = split_state(oa, n, S, P)
    for key in ("env", "ring", "mat", "items", "iring"):
        if not np.array_equal(g[key], o[key]):
            bad = np.argwhere(g[key] != o[key])[:5]
            raise AssertionError(f"{where}: {key} differs at {bad.tolist()}")
    if not np.array_equal(g["ent"], o["ent"]):
        bad = np.argwhere(g["ent"] != o["ent"])[:8]
        names = [(int(e), abi.ENTITY_FIELDS[f] if f < len(abi.ENTITY_FIELDS) else f, int(s),
                  int(g["ent"][e, f, s]), int(o["ent"][e, f, s])) for e, f, s in bad]
        raise AssertionError(f"{where}: entity fields differ (env, field, slot, gpu, oracle): {names}")


def test_map_bank_parity():
    cfg = Config.preset("C2", MAP_N=16, map_seed=123)
    eng = _engine(cfg, 1, seed=0)
    orc = OracleEnvs(cfg, 1, seed=0)
    assert np.array_equal(eng.map_bank(), orc.map_bank())


@pytest.mark.parametrize("preset", ["C2", "C3", "C4"])
def test_rollout_parity(preset):
    import torch

    n, steps = 6, 120
    task = (np.arange(2048) % 97 / 97.0 - 0.5).astype(np.float16)
    cfg = Config.preset(preset, MAP_N=8, early_stop_agent_num=8)
    eng = _engine(cfg, n, seed=11, task=task)
    orc = OracleEnvs(cfg, n, seed=11, task_embedding=task)
    eng.reset()
    orc.reset()
    torch.cuda.synchronize()
    _cmp_state(eng.get_state(), orc.get_state(), n, eng.S, "reset")
    if orc.obs is not None:
        assert np.array_equal(eng.obs.cpu().numpy(), orc.obs), "reset obs"
    assert np.array_equal(eng.mask.cpu().numpy(), orc.mask)
    for t in range(steps):
        acts = orc.scripted_actions(1000 + t)
        g_acts = eng.scripted_actions(1000 + t)
        assert np.array_equal(g_acts.cpu().numpy(), acts), f"policy differs at step {t}"
        orc.step(acts)
        eng.step(torch.from_numpy(acts).cuda())
        torch.cuda.synchronize()
        _cmp_state(eng.get_state(), orc.get_state(), n, eng.S, f"step {t}")
        for name in ("rew", "term", "trunc", "mask"):
            gv = getattr(eng, name).cpu().numpy()
            ov = getattr(orc, name)
            assert np.array_equal(gv, ov), f"{name} differs at step {t}"
        if orc.obs is not None and (t % 10 == 0 or t == steps - 1):
            go = eng.obs.cpu().numpy()
            if not np.array_equal(go, orc.obs):
                bad = np.argwhere(go != orc.obs)[:5]
                raise AssertionError(f"obs differs at step {t}: {bad.tolist()}")


def test_set_state_roundtrip():
    import torch

    cfg = Config.preset("C3", MAP_N=4)
    orc = OracleEnvs(cfg, 3, seed=5)
    orc.reset()
    for t in range(15):
        orc.step(orc.scripted_actions(t))
    eng = _engine(cfg, 3, seed=99)
    eng.set_state(orc.get_state())
    for t in range(15, 40):
        a = orc.scripted_actions(t)
        orc.step(a)
        eng.step(torch.from_numpy(a).cuda())
    torch.cuda.synchronize()
    _cmp_state(eng.get_state(), orc.get_state(), 3, eng.S, "after set_state")


class _EngineStepper:
    """HIP engine behind the golden-rollout driver (numpy in/out)."""

    def __init__(self, preset):
        from tests.golden.make_rollout_fixtures import config

        self.e = _engine(config(preset), 4, seed=2024)

    def reset(self):
        self.e.reset()

    def step(self, a):
        import torch

        self.e.step(torch.from_numpy(a).cuda())

    def scripted_actions(self, s):
        return self.e.scripted_actions(s).cpu().numpy()

    def get_state(self):
        import torch

        torch.cuda.synchronize()
        return self.e.get_state()

    def outputs(self):
        return tuple(getattr(self.e, n).cpu().numpy() for n in ("rew", "term", "trunc", "mask"))


@pytest.mark.parametrize("preset", ["C2", "C3"])
def test_golden_rollout_hashes_gpu(preset):
    import json

    from tests.golden.make_rollout_fixtures import rollout

    golden = json.load(open("tests/golden/rollout_hashes.json"))[preset]
    assert rollout(_EngineStepper(preset), preset) == golden
