"""The device evaluate/train loop (nmmo_amd/trainer.py) end to end on MI355X: recv -> policy ->
HBM store -> step until the batch is full, then sort, GAE, flatten and PPO minibatches. Every
store's inputs are replayed into the reference's host storage restated in oracle/storage.py
(clean_pufferl.py:182-197, 327-346, 414-446); the device experience, sort order, advantages and
flattened batch must equal it exactly."""

import numpy as np
import pytest
import torch

from tests.conftest import gpu_available

pytestmark = [pytest.mark.gpu, pytest.mark.skipif(not gpu_available(), reason="needs a GPU")]


def test_device_trainer_matches_reference_storage():
    from nmmo_amd.config import Config
    from nmmo_amd.engine import NmmoEngine
    from nmmo_amd.trainer import DeviceTrainer, MaskedLinearAgent, TrainConfig
    from oracle.storage import ReferenceStorage

    torch.manual_seed(0)
    cfg = Config.preset("C4", MAP_N=2, early_stop_agent_num=8)
    eng = NmmoEngine(cfg, 2, seed=5)
    eng.reset()
    agent = MaskedLinearAgent(cfg.TASK_EMBED_DIM).cuda()
    tc = TrainConfig(batch_size=1024, batch_rows=16, bptt_horizon=8, update_epochs=2, total_timesteps=4096)
    tr = DeviceTrainer(eng, agent, tc)
    ref = ReferenceStorage(tc.batch_size, eng.obs_elems)

    def on_store(o, r, d, mask, actions, logprob, value, env_id, step):
        ref.store(o.cpu().numpy(), r.cpu(), d.cpu(), mask.cpu().numpy(), actions.cpu().numpy(),
                  logprob.cpu().numpy(), value.cpu().numpy(), env_id.cpu().numpy(), step)

    stats = tr.evaluate(on_store=on_store)
    exp = tr.experience
    assert exp.ptr == tc.batch_size + 1 == ref.ptr
    assert stats["agent_steps"] >= tc.batch_size + 1 and stats["agent_SPS"] > 0
    assert torch.equal(exp.obs.cpu(), ref.obs)
    assert torch.equal(exp.actions.cpu(), ref.actions)
    for name in ("logprobs", "rewards", "dones", "values"):
        assert torch.equal(getattr(exp, name).cpu(), getattr(ref, name)), name

    before = [p.detach().clone() for p in agent.parameters()]
    losses = tr.train()
    idxs, adv, b = tr.last_batch
    ref_idxs = ref.sort()
    assert idxs.cpu().tolist() == ref_idxs
    ref_adv = ref.advantages(ref_idxs, tc.gamma, tc.gae_lambda)
    assert torch.equal(adv.cpu(), ref_adv)
    rb = ref.batch(ref_idxs, ref_adv, tc.batch_rows, tc.bptt_horizon)
    assert torch.equal(b["b_idxs"].cpu().long(), rb["b_idxs"])
    assert torch.equal(b["b_values"].cpu(), rb["b_values"])
    assert torch.equal(b["b_returns"].cpu(), rb["b_returns"])
    m = exp.minibatch(b["b_idxs"], 1)
    assert np.array_equal(m["obs"].cpu().numpy(), rb["b_obs"][1])
    assert np.array_equal(m["actions"].cpu().numpy(), rb["b_actions"][1])
    for k in ("policy_loss", "value_loss", "entropy", "approx_kl", "clipfrac"):
        assert np.isfinite(losses[k]), k
    assert any(not torch.equal(p0, p1.detach()) for p0, p1 in zip(before, agent.parameters()))
    # a second batch continues from where the first left the envs
    tr.evaluate()
    assert tr.experience.ptr == tc.batch_size + 1
    tr.train()
    assert tr.update == 2
    eng.close()
