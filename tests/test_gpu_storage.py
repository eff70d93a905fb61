"""GPU-resident experience storage against the reference's storage
restated on the CPU (oracle/storage.py): rollouts of the HIP engine are stored step by step on
the device (flat obs, native obs expanded on store, wire records decoded on store) and on the host checker with the same
learner masks, actions, logprobs and values; every buffer, the (env_id, step) order, the
advantages and the minibatch gathers must be bit-identical."""

import numpy as np
import pytest

from nmmo_amd import abi
from nmmo_amd.config import Config
from oracle.storage import ReferenceStorage

pytestmark = pytest.mark.gpu


def _roll(layout_kind, batch_size, n_envs, masked_policy, env_id_mode):
    import torch

    from nmmo_amd.engine import NmmoEngine
    from nmmo_amd.storage import DeviceExperience

    cfg = Config.preset("C4", MAP_N=4, early_stop_agent_num=8, obs_layout=layout_kind)
    eng = NmmoEngine(cfg, n_envs, seed=21)
    P = eng.P
    n = n_envs * P
    x = DeviceExperience(batch_size, eng.obs_elems, n + 7, device=eng.device)
    ref = ReferenceStorage(batch_size, eng.obs_elems)
    g = torch.Generator(device="cpu").manual_seed(5)
    perm = torch.randperm(n, generator=g).to(torch.int32) if env_id_mode == "perm" else None
    eng.reset()
    step = 0
    while ref.ptr < batch_size + 1:
        step += 1
        a = eng.scripted_actions(300 + step)
        eng.step(a)
        lp = torch.randn(n, generator=g)
        v = torch.randn(n, generator=g)
        pmask = (torch.rand(n, generator=g) < 0.8) if masked_policy else torch.ones(n, dtype=torch.bool)
        learner_mask = eng.mask.view(-1).cpu().bool() & pmask
        if layout_kind == abi.OBS_FLAT:
            flat = eng.obs.view(n, -1)
        elif layout_kind == abi.OBS_NATIVE:
            flat = eng.expand_obs().view(n, -1)
        else:  # wire records -> native -> flat: the checker's rows come the long way round
            from nmmo_amd import wire

            flat = eng.expand_obs(wire.unpack(eng.obs, n_envs, P)).view(n, -1)
        env_id = perm if perm is not None else torch.arange(n, dtype=torch.int32) + 3
        x.store(eng.obs, eng.rew.view(-1), eng.term.view(-1), learner_mask, a.view(n, 12), lp, v, step,
                env_id=env_id if perm is not None else None, env_id_base=3,
                engine=eng if layout_kind != abi.OBS_FLAT else None)
        ref.store(flat.cpu().numpy(), eng.rew.view(-1).cpu().numpy(), eng.term.view(-1).cpu().numpy(),
                  learner_mask.numpy(), a.view(n, 12).cpu().numpy(), lp.numpy(), v.numpy(), env_id.numpy(), step)
        assert x.ptr == ref.ptr, f"step {step}: ptr {x.ptr} != {ref.ptr}"
        assert step < 400
    eng.close()
    return x, ref


def _same(a, b, what):
    import torch

    a = a.cpu()
    b = torch.as_tensor(b)
    assert a.shape == b.shape, (what, a.shape, b.shape)
    if a.dtype == torch.float32:
        a, b = a.view(torch.int32), b.view(torch.int32)
    assert torch.equal(a, b), f"{what} differs at {(a != b).nonzero()[:5].tolist()}"


@pytest.mark.parametrize("layout_kind,masked_policy,env_id_mode", [
    (abi.OBS_FLAT, False, "base"), (abi.OBS_NATIVE, True, "base"), (abi.OBS_FLAT, True, "perm"),
    (abi.OBS_WIRE, True, "perm")])
def test_storage_matches_reference(layout_kind, masked_policy, env_id_mode):
    import torch

    B, rows, bptt = 1024, 16, 8
    x, ref = _roll(layout_kind, B, 3, masked_policy, env_id_mode)
    for name in ("obs", "actions", "logprobs", "rewards", "dones", "truncateds", "values"):
        _same(getattr(x, name), getattr(ref, name), name)
    idxs = x.sort()
    ridx = ref.sort()
    _same(idxs.long(), torch.tensor(ridx), "sorted idxs")
    adv = x.advantages(idxs, 0.99, 0.95)
    radv = ref.advantages(ridx, 0.99, 0.95)
    _same(adv, radv, "advantages")
    b = x.batch(idxs, adv, rows, bptt)
    rb = ref.batch(ridx, radv, rows, bptt)
    _same(b["b_idxs"].long(), rb["b_idxs"], "b_idxs")
    for k in ("b_values", "b_advantages", "b_returns"):
        _same(b[k].contiguous(), rb[k].contiguous(), k)
    for mb in range(b["num_minibatches"]):
        m = x.minibatch(b["b_idxs"], mb)
        _same(m["obs"], rb["b_obs"][mb], f"mb {mb} obs")
        _same(m["actions"], rb["b_actions"][mb], f"mb {mb} actions")
        _same(m["logprobs"], rb["b_logprobs"][mb], f"mb {mb} logprobs")
        _same(m["dones"], rb["b_dones"][mb], f"mb {mb} dones")


def test_store_respects_capacity_in_one_recv():
    """A recv with more alive rows than room left: only the first ones in row order are kept."""
    import torch

    from nmmo_amd.storage import DeviceExperience

    n, elems = 1000, 9
    x = DeviceExperience(99, elems, n)
    o = torch.arange(n * elems, dtype=torch.float32).view(n, elems).cuda()
    mask = (torch.arange(n) % 3 != 0).to(torch.uint8).cuda()
    z = torch.zeros(n, device="cuda")
    x.store(o, z, z.to(torch.uint8), mask, torch.zeros(n, 12, dtype=torch.int32), z, z, 1)
    assert x.ptr == 100
    keep = torch.nonzero(mask.cpu()).view(-1)[:100]
    assert torch.equal(x.obs.cpu(), o.cpu()[keep])
    assert torch.equal(x.env_id.cpu().long(), keep)
    x.store(o, z, z.to(torch.uint8), mask, torch.zeros(n, 12, dtype=torch.int32), z, z, 2)
    assert x.ptr == 100  # full: nothing more is stored


def test_store_drops_out_of_range_env_ids():
    """A selected row whose env_id is outside [0, n_slots) is dropped without writing out of range
    and raises status bit 0 (nmmo_hip.h NmmoExperience.status); the other rows store normally."""
    import torch

    from nmmo_amd.storage import DeviceExperience

    n, elems, slots = 64, 5, 64
    x = DeviceExperience(200, elems, slots)
    o = torch.arange(n * elems, dtype=torch.float32).view(n, elems).cuda()
    mask = torch.ones(n, dtype=torch.uint8).cuda()
    eid = torch.arange(n, dtype=torch.int32)
    eid[5], eid[9] = slots + 1000, -3
    z = torch.zeros(n, device="cuda")
    x.store(o, z, z.to(torch.uint8), mask, torch.zeros(n, 12, dtype=torch.int32), z, z, 1, env_id=eid)
    assert x.status == 1
    assert x.ptr == n - 2
    keep = [r for r in range(n) if r not in (5, 9)]
    assert torch.equal(x.obs[:n - 2].cpu(), o.cpu()[keep])
    assert torch.equal(x.slot_count.cpu(), torch.tensor([0 if r in (5, 9) else 1 for r in range(slots)],
                                                         dtype=torch.int32))
    with pytest.raises(ValueError):
        x.store(o, z, z.to(torch.uint8), mask, torch.zeros(n, 12, dtype=torch.int32), z, z, 2, env_id=eid,
                validate=True)
