"""Native obs layout on the GPU (SPEC.md §8b): the native obs_kernel variant, expanded by
nmmo_expand_obs, is bit-identical to the flat kernel's pufferlib row; the learner-side decoder
gives the same fields. Both engines step the same action stream through the C-ABI."""

import numpy as np
import pytest

from nmmo_amd import abi, layout
from nmmo_amd.config import Config

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("preset,wrapper", [("C4", None), ("C3", None), ("C4", "yaofeng"),
                                            ("C4", "neurips23_start_kit")])
def test_native_expands_to_flat(preset, wrapper):
    import torch

    from nmmo_amd.engine import NmmoEngine
    from nmmo_amd.wrappers import wrapper_config

    n, steps = 3, 60
    task = (np.arange(2048) % 53 / 53.0 - 0.25).astype(np.float16)
    flat = NmmoEngine(Config.preset(preset, MAP_N=4, early_stop_agent_num=8), n, seed=13, task_embedding=task)
    nat = NmmoEngine(Config.preset(preset, MAP_N=4, early_stop_agent_num=8, obs_layout=abi.OBS_NATIVE), n,
                     seed=13, task_embedding=task)
    assert nat.obs.dtype == torch.uint8 and nat.obs.shape == (n, abi.native_env_bytes(128))
    if wrapper:
        kw = dict(hp_bonus_weight=0.03) if wrapper == "yaofeng" else dict(heal_bonus_weight=0.03)
        flat.set_wrapper(wrapper_config(wrapper, **kw))
        nat.set_wrapper(wrapper_config(wrapper, **kw))
    flat.reset()
    nat.reset()
    for t in range(steps):
        if t:
            a = flat.scripted_actions(900 + t)
            flat.step(a)
            nat.step(a)
        ex = nat.expand_obs()
        torch.cuda.synchronize()
        if not torch.equal(ex, flat.obs):
            bad = (ex != flat.obs).nonzero()[:5].tolist()
            raise AssertionError(f"step {t}: expanded native obs differs from flat at {bad}")
        assert torch.equal(nat.rew, flat.rew) and torch.equal(nat.mask, flat.mask)
        if t % 20 == 0:
            a_ = layout.unflatten(flat.obs.view(n * 128, -1))
            b_ = layout.unflatten_native(nat.obs, 128, nat.task_table)
            for k in ("Entity", "Tile", "Inventory", "Market", "Task", "AgentId", "CurrentTick"):
                assert torch.equal(a_[k], b_[k]), f"step {t}: {k}"
            for h, d in a_["ActionTargets"].items():
                for k2, v in d.items():
                    assert torch.equal(v, b_["ActionTargets"][h][k2]), f"step {t}: {h}.{k2}"


def test_expand_subset_of_envs():
    """A learner expands any run of consecutive envs (e.g. one gathered shard)."""
    import torch

    from nmmo_amd.engine import NmmoEngine

    cfg = Config.preset("C4", MAP_N=4, obs_layout=abi.OBS_NATIVE)
    nat = NmmoEngine(cfg, 4, seed=2)
    nat.reset()
    for t in range(5):
        nat.step(nat.scripted_actions(t))
    full = nat.expand_obs()
    part = nat.expand_obs(nat.obs[2:4])
    torch.cuda.synchronize()
    assert torch.equal(full[2:4], part)
