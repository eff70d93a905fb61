"""Device wrapper layer (SPEC.md §13, libnmmo_hip.so wrap_kernel) vs the CPU restatement of the
reference's wrappers (oracle/wrapper.py: stat_wrapper.py + agent_zoo/*/reward_wrapper.py).
Shaped rewards and edited obs bit-exact; episode info dicts equal key for key."""

import numpy as np
import pytest

from nmmo_amd import abi
from nmmo_amd.config import Config
from nmmo_amd.wrappers import infos_from_records, wrapper_config
from oracle.oracle import OracleEnvs
from oracle.wrapper import OracleWrapper

pytestmark = pytest.mark.gpu

# the reference's YAML reward_wrapper sections (config.yaml:99-107) plus non-zero weights for
# every shaping term so each one is exercised
CASES = [
    ("neurips23_start_kit", "C4", dict(heal_bonus_weight=0.03, explore_bonus_weight=0.01)),
    ("neurips23_start_kit", "C2", dict(heal_bonus_weight=0.03, explore_bonus_weight=0.01, eval_mode=True)),
    ("takeru", "C4", dict(explore_bonus_weight=0.01)),
    ("yaofeng", "C4", dict(hp_bonus_weight=0.03, exp_bonus_weight=0.002, defense_bonus_weight=0.04,
                           attack_bonus_weight=0.001, gold_bonus_weight=0.001, custom_bonus_scale=0.5)),
    ("yaofeng", "C3", dict(hp_bonus_weight=0.03, exp_bonus_weight=0.002, use_custom_reward=False)),
    ("base", "C3", dict()),
]


def _eq_info(g, o, where):
    assert set(g) == set(o), f"{where}: agents {sorted(g)} vs {sorted(o)}"
    for a in g:
        gs, os_ = g[a]["stats"], o[a]["stats"]
        assert set(gs) == set(os_), f"{where} agent {a}: stat keys {sorted(set(gs) ^ set(os_))}"
        for k in gs:
            assert gs[k] == os_[k], f"{where} agent {a}: {k} gpu {gs[k]} oracle {os_[k]}"
        for k in ("length", "curriculum"):
            assert g[a][k] == o[a][k], f"{where} agent {a}: {k} gpu {g[a][k]} oracle {o[a][k]}"
        # return: the same double sum of float32 env rewards on both sides (SPEC §13)
        assert g[a]["return"] == o[a]["return"], f"{where} agent {a}: return"


@pytest.mark.parametrize("agent,preset,kw", CASES)
def test_wrapper_parity(agent, preset, kw):
    import torch

    from nmmo_amd.engine import NmmoEngine

    n, steps = 4, 90
    cfg = Config.preset(preset, MAP_N=8, early_stop_agent_num=8)
    eng = NmmoEngine(cfg, n, seed=21)
    orc = OracleEnvs(cfg, n, seed=21)
    eng.set_wrapper(wrapper_config(agent, **kw))
    ow = OracleWrapper(orc, agent, **kw)
    eng.reset()
    orc.reset()
    ow.after_reset()
    torch.cuda.synchronize()
    if orc.obs is not None:
        assert np.array_equal(eng.obs.cpu().numpy(), orc.obs), "reset obs"
    n_done = 0
    for t in range(steps):
        acts = orc.scripted_actions(500 + t)
        orc.step(acts)
        ow.after_step(acts)
        eng.step(torch.from_numpy(acts).cuda())
        torch.cuda.synchronize()
        gr, orw = eng.rew.cpu().numpy(), orc.rew
        if not np.array_equal(gr, orw):
            bad = np.argwhere(gr != orw)[:5]
            raise AssertionError(f"step {t}: shaped reward differs at {bad.tolist()}: "
                                 f"{[(float(gr[tuple(b)]), float(orw[tuple(b)])) for b in bad]}")
        g_inf = infos_from_records(eng.info_records())
        for e in range(n):
            _eq_info(g_inf[e], ow.infos[e], f"step {t} env {e}")
            n_done += len(ow.infos[e])
        st, _ = eng.wrapper_state()
        for e in range(n):
            for a in range(1, cfg.PLAYER_N + 1):
                assert st["curr_count"][e, a - 1] == ow.uniq[e][a]["curr_count"], f"step {t} env {e} agent {a}: unique count"
                assert st["cum_reward"][e, a - 1] == ow.cum[e][a], f"step {t} env {e} agent {a}: cum reward"
        if orc.obs is not None and (t % 7 == 0 or t == steps - 1):
            go = eng.obs.cpu().numpy()
            if not np.array_equal(go, orc.obs):
                bad = np.argwhere(go != orc.obs)[:5]
                raise AssertionError(f"obs differs at step {t}: {bad.tolist()}")
    assert n_done > 0, "no agent finished an episode: the info path was not exercised"
    assert eng.wrapper_dropped_events() == 0


def test_wrapper_reports_dropped_events():
    """A ring smaller than one tick's events: the overwritten rows are counted, not silently lost."""
    from nmmo_amd.engine import NmmoEngine

    eng = NmmoEngine(Config.preset("C2", MAP_N=2, event_cap=8), 2, seed=4)
    eng.set_wrapper(wrapper_config("base"))
    eng.reset()
    for t in range(6):
        eng.step(eng.scripted_actions(t))
    assert eng.wrapper_dropped_events() > 0


def test_wrapper_off_restores_raw_rewards():
    import torch

    from nmmo_amd.engine import NmmoEngine

    cfg = Config.preset("C2", MAP_N=4)
    a, b = NmmoEngine(cfg, 2, seed=3), NmmoEngine(cfg, 2, seed=3)
    a.set_wrapper(wrapper_config("neurips23_start_kit", heal_bonus_weight=0.5))
    a.set_wrapper(None)
    a.reset()
    b.reset()
    for t in range(20):
        act = b.scripted_actions(t)
        a.step(act)
        b.step(act)
    torch.cuda.synchronize()
    assert torch.equal(a.rew, b.rew)
    assert a.info is None


def test_wrapper_needs_event_log():
    from nmmo_amd._native import NativeError
    from nmmo_amd.engine import NmmoEngine

    eng = NmmoEngine(Config.preset("C2", MAP_N=2, event_cap=0), 1, seed=0)
    with pytest.raises(NativeError, match="event log"):
        eng.set_wrapper(wrapper_config("base"))
    assert abi.agent_info_dtype().itemsize == 104
