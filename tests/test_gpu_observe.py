"""nmmo_observe and env batches on MI355X: nmmo_step(obs = NULL) + nmmo_observe writes the same
bytes as nmmo_step(obs), flat and native; and a rollout split into batches (one handle each,
consecutive env_index_base, as bench.py --batches runs it) is the rollout of one handle over all
the envs, bit for bit (obs, rewards, flags)."""

import numpy as np
import pytest
import torch

from tests.conftest import gpu_available

pytestmark = [pytest.mark.gpu, pytest.mark.skipif(not gpu_available(), reason="needs a GPU")]


def _cfg(layout):
    from nmmo_amd.config import Config

    return Config.preset("C4", MAP_N=4, early_stop_agent_num=8, obs_layout=layout)


@pytest.mark.parametrize("layout", ["flat", "native"])
def test_observe_equals_step_obs(layout):
    from nmmo_amd import abi
    from nmmo_amd.engine import NmmoEngine

    cfg = _cfg(abi.OBS_FLAT if layout == "flat" else abi.OBS_NATIVE)
    a = NmmoEngine(cfg, 3, seed=5)
    b = NmmoEngine(cfg, 3, seed=5)
    a.reset()
    b.reset()
    for t in range(30):
        a.scripted_actions(900 + t)
        b.scripted_actions(900 + t)
        a.step()
        b.step(write_obs=False)
        b.observe()
        if t % 10 == 9:
            torch.cuda.synchronize()
            assert torch.equal(a.obs.view(torch.uint8), b.obs.view(torch.uint8)), f"tick {t}"
    a.close()
    b.close()


def test_observe_refused_without_obs_layout():
    from nmmo_amd import abi
    from nmmo_amd._native import NativeError
    from nmmo_amd.engine import NmmoEngine

    e = NmmoEngine(_cfg(abi.OBS_NONE), 1, seed=1)
    e.reset()
    with pytest.raises(NativeError):
        e.observe(out=torch.zeros(16, device=e.device))
    e.close()


def test_batches_equal_one_handle():
    from nmmo_amd import abi
    from nmmo_amd.engine import NmmoEngine

    cfg = _cfg(abi.OBS_NATIVE)
    n, parts = 4, 2
    whole = NmmoEngine(cfg, n, seed=3)
    halves = [NmmoEngine(cfg, n // parts, seed=3, env_index_base=i * (n // parts)) for i in range(parts)]
    whole.reset()
    for h in halves:
        h.reset()
    streams = [torch.cuda.Stream() for _ in halves]
    for t in range(40):
        if t == 12:
            m = np.array([1, 0, 0, 1], bool)
            whole.end_episodes(m)
            for i, h in enumerate(halves):
                h.end_episodes(m[i * 2:(i + 1) * 2])
        whole.scripted_actions(77)
        whole.step()
        torch.cuda.current_stream().synchronize()
        for h, st in zip(halves, streams):
            with torch.cuda.stream(st):
                h.scripted_actions(77)
                h.step(write_obs=False)
                h.observe()
        torch.cuda.synchronize()
        for name in ("rew", "term", "trunc", "mask"):
            got = torch.cat([getattr(h, name) for h in halves])
            assert torch.equal(getattr(whole, name), got), f"{name} tick {t}"
        got = torch.cat([h.obs.view(n // parts, -1) for h in halves])
        assert torch.equal(whole.obs.view(n, -1), got), f"obs tick {t}"
    whole.close()
    for h in halves:
        h.close()


@pytest.mark.parametrize("preset", ["C2", "C3", "C4"])
def test_counters_equal_the_outputs(preset):
    """The device counters the bench reads (nmmo_set_counters): agent-steps = the sum of every
    step's mask, event rows = the growth of the event count, over staggered episode ends and
    auto-resets (the tick adds them with one atomic per workgroup)."""
    from nmmo_amd import abi
    from nmmo_amd.config import Config
    from nmmo_amd.engine import NmmoEngine

    cfg = Config.preset(preset, MAP_N=4, early_stop_agent_num=8, obs_layout=abi.OBS_NONE)
    n = 12
    eng = NmmoEngine(cfg, n, seed=17)
    eng.reset()
    cnt = torch.zeros(3, dtype=torch.int64, device=eng.device)
    eng.set_counters(cnt)
    ids = np.arange(n)
    total = 0
    for t in range(40):
        eng.end_episodes(ids % 8 == t % 8)
        eng.scripted_actions(500 + t)
        eng.step(write_obs=False)
        total += int(eng.mask.sum().item())
    torch.cuda.synchronize()
    assert int(cnt[0].item()) == total
    assert int(cnt[1].item()) >= 0 and int(cnt[2].item()) > 0
    eng.close()
