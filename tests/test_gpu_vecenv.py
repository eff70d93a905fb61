"""The pufferlib-shaped pool and the PettingZoo-shaped facade driven the way the reference
drives them (clean_pufferl.py:106-118,175,293,357; stat_wrapper.py:51,64), on the GPU."""

import numpy as np
import pytest

from nmmo_amd import layout
from nmmo_amd.config import Config

pytestmark = pytest.mark.gpu


def test_pool_protocol_matches_engine_and_oracle():
    import torch

    from nmmo_amd.vecenv import GpuVecEnv
    from oracle.oracle import OracleEnvs

    cfg = Config.preset("C4", MAP_N=4, early_stop_agent_num=8)
    pool = GpuVecEnv(None, env_kwargs=None, num_envs=3, envs_per_worker=1, envs_per_batch=3,
                     env_pool=True, mask_agents=True, config=cfg, seed=5)
    assert pool.single_observation_space.shape == (23987,)
    assert pool.single_action_space.shape == (12,)
    assert pool.agents_per_env == 128 and pool.driver_env.obs_sz == 23987
    ref = OracleEnvs(cfg, 3, seed=5)
    pool.async_reset(1)
    ref.reset(env_seeds=np.array([1, 2, 3], dtype=np.uint64))
    rng = np.random.default_rng(0)
    for t in range(10):
        o, r, d, tr, infos, env_id, mask = pool.recv()
        assert o.shape == (3 * 128, 23987) and o.is_cuda and mask.dtype == np.bool_
        assert np.array_equal(o.cpu().numpy(), ref.obs.reshape(3 * 128, -1))
        assert np.array_equal(mask, ref.mask.reshape(-1).astype(bool))
        # a policy-like action sampler over the masks (baseline_policy.py:228-264)
        d_ = layout.unflatten(o.cpu().numpy())
        acts = np.zeros((3 * 128, 12), np.int64)
        for h, ((a, b), n) in enumerate(layout.ACTION_HEADS):
            m = d_["ActionTargets"][a][b].astype(bool)
            for i in range(3 * 128):
                ok = np.flatnonzero(m[i])
                acts[i, h] = rng.choice(ok) if len(ok) else 0
        pool.send(acts)
        ref.step(acts.reshape(3, 128, 12).astype(np.int32))
    o, r, d, tr, infos, env_id, mask = pool.recv()
    torch.cuda.synchronize()
    assert np.array_equal(r.cpu().numpy(), ref.rew.reshape(-1))
    assert np.array_equal(pool.engine.get_state(), ref.get_state())
    pool.close()


def test_pettingzoo_facade():
    from nmmo_amd.vecenv import NmmoEnv

    env = NmmoEnv(Config.preset("C3", MAP_N=2), seed=3)
    obs, info = env.reset(seed=7)
    assert len(obs) == 128 and set(obs[1]) >= {"Tile", "Entity", "Task", "AgentId", "ActionTargets"}
    assert obs[5]["AgentId"][0] == 5 and obs[5]["Tile"].shape == (225, 3)
    total = 0
    for t in range(30):
        acts = {a: {"Move": {"Direction": t % 4}} for a in env.agents}
        obs, rew, term, trunc, info = env.step(acts)
        total += len(rew)
        assert all(abs(v - 1 / 1024) < 1e-9 or v == -1.0 for v in rew.values())
    realm = env.realm
    assert realm.tick == 30 and all(p.alive for p in realm.players.values())
    assert total > 0
    env.close()


def test_pool_with_reward_wrapper_returns_stat_infos():
    """env_creator's RewardWrapper on the device: recv() hands the trainer the same shaped
    rewards and per-env info dicts the CPU restatement of stat_wrapper.py produces."""
    import torch

    from nmmo_amd.vecenv import GpuVecEnv
    from oracle.oracle import OracleEnvs
    from oracle.wrapper import OracleWrapper

    cfg = Config.preset("C4", MAP_N=4, early_stop_agent_num=8, HORIZON=40)
    rw = {"eval_mode": False, "early_stop_agent_num": 8, "use_custom_reward": True,
          "heal_bonus_weight": 0.03, "explore_bonus_weight": 0.01}  # config.yaml:99-107
    pool = GpuVecEnv(None, env_kwargs={"reward_wrapper": rw}, num_envs=2, config=cfg, seed=8,
                     agent="neurips23_start_kit")
    ref = OracleEnvs(cfg, 2, seed=8)
    ow = OracleWrapper(ref, "neurips23_start_kit", **rw)
    pool.async_reset()
    ref.reset()
    ow.after_reset()
    finished = 0
    for t in range(50):
        o, r, d, tr, infos, env_id, mask = pool.recv()
        assert np.array_equal(o.cpu().numpy(), ref.obs.reshape(2 * 128, -1)), f"obs step {t}"
        assert np.array_equal(r.cpu().numpy(), ref.rew.reshape(-1)), f"reward step {t}"
        assert len(infos) == 2
        for e in range(2):
            assert set(infos[e]) == set(ow.infos[e]), f"step {t} env {e}"
            for a, info in infos[e].items():
                assert info["stats"] == ow.infos[e][a]["stats"]
                assert info["length"] == ow.infos[e][a]["length"]
                finished += 1
        acts = ref.scripted_actions(77 + t)
        pool.send(torch.from_numpy(acts.reshape(-1, 12)))
        ref.step(acts)
        ow.after_step(acts)
    assert finished > 0
    pool.close()


def test_facade_serves_stat_wrapper_reads():
    """NmmoEnv over the HIP engine answers every read of stat_wrapper.py:122-185 (dead_this_tick,
    .val attributes, attack_level, agent_task_map task fields) with the values the oracle's state
    gives, on a sampled heldout curriculum."""
    from nmmo_amd import tasks
    from nmmo_amd.vecenv import NmmoEnv, _Realm, parse_env_state, tasks_from_state
    from oracle.oracle import OracleEnvs
    from tests.test_facade import walk_stat_wrapper_reads

    cfg = Config.preset("C4", MAP_N=2, early_stop_agent_num=0)
    env = NmmoEnv(cfg, seed=17)
    ref = OracleEnvs(cfg, 1, seed=17)
    specs = tasks.heldout_curriculum()
    env.engine.set_curriculum(specs)
    ref.set_curriculum(specs)
    env.reset()
    ref.reset()
    names = [s.name for s in specs]
    walked = 0
    for t in range(90):
        a = ref.scripted_actions(40 + t)
        ref.step(a)
        _, rew, term, trunc, _ = env.step({p: a[0, p - 1] for p in env.possible_agents})
        realm, tmap = env.realm, env.agent_task_map
        st = parse_env_state(ref.get_state(), ref.S, ref.P)
        oreal = _Realm(st, ref.events(0))
        otmap = {tk.assignee[0]: [tk] for tk in tasks_from_state(st, env.possible_agents, names)}
        assert realm.tick == oreal.tick
        assert sorted(realm.players.dead_this_tick) == sorted(oreal.players.dead_this_tick)
        for p, dead in term.items():
            if dead or trunc[p]:
                assert walk_stat_wrapper_reads(realm, tmap, p, dead) == walk_stat_wrapper_reads(oreal, otmap, p, dead)
                walked += 1
    assert walked > 0
    env.close()


def test_realm_read_once_per_tick():
    """BaseStatWrapper reads env.realm once per agent per step (stat_wrapper.py:122-123): over
    the reads of a whole step for all 128 agents the facade copies the device state once."""
    from nmmo_amd.vecenv import NmmoEnv
    from tests.test_facade import walk_stat_wrapper_reads

    env = NmmoEnv(Config.preset("C4", MAP_N=2, early_stop_agent_num=0), seed=3)
    calls = []
    orig = env.engine.get_state
    env.engine.get_state = lambda: (calls.append(1), orig())[1]
    env.reset()
    for t in range(3):
        calls.clear()
        env.step({})
        realm = env.realm
        present = [a for a in env.possible_agents
                   if realm.players.get(a) is not None or a in realm.players.dead_this_tick]
        assert len(present) == 128
        for a in present:
            walk_stat_wrapper_reads(env.realm, env.agent_task_map, a, terminated=False)
        assert len(calls) == 1, f"tick {t}: {len(calls)} state copies"
    env.close()


def test_async_pool_15_6_clean_pufferl_loop_matches_oracle_per_env():
    """The reference's default pool (config.yaml:35-38: num_envs 15, envs_per_batch 6,
    env_pool True) driven in clean_pufferl.evaluate's order (recv -> per-slot state indexed by
    env_id -> policy -> store -> send, clean_pufferl.py:287-357): the FIFO ready order of SPEC §14,
    env_id = the batch envs' agent slots, and every env's trajectory bit-equal to the oracle
    stepping that env alone on the same action stream (auto-resets included)."""
    import collections

    import torch

    from nmmo_amd.vecenv import GpuVecEnv, reset_seeds
    from oracle.oracle import OracleEnvs

    n, k, P = 15, 6, 128
    cfg = Config.preset("C4", MAP_N=4, early_stop_agent_num=8, HORIZON=12)
    pool = GpuVecEnv(None, env_kwargs=None, num_envs=n, envs_per_worker=1, envs_per_batch=k,
                     env_pool=True, mask_agents=True, config=cfg, seed=5)
    assert pool.envs_per_batch == k and pool.agents_per_env == P
    ref = OracleEnvs(cfg, n, seed=5)
    pool.async_reset(1)
    ref.reset(env_seeds=reset_seeds(1, 0, n))
    order = collections.deque(range(n))
    lstm = np.zeros(n * P, np.int64)  # per-slot recurrent state, indexed by env_id (:310-315)
    stored = collections.Counter()     # sort keys (env_id, step) of stored rows (:346)
    full = np.zeros((n, P, 12), np.int32)
    steps = np.zeros(n, np.int64)
    for step in range(1, 46):
        o, r, d, t, infos, env_id, mask = pool.recv()
        batch = [order.popleft() for _ in range(k)]
        assert np.array_equal(env_id, (np.array(batch)[:, None] * P + np.arange(P)).reshape(-1))
        assert o.shape == (k * P, 23987) and len(infos) == k and mask.shape == (k * P,)
        assert np.array_equal(o.cpu().numpy(), ref.obs[batch].reshape(k * P, -1)), f"obs @ recv {step}"
        for name, x in (("rew", r), ("term", d), ("trunc", t)):
            assert np.array_equal(x.cpu().numpy(), getattr(ref, name)[batch].reshape(-1)), f"{name} @ {step}"
        assert np.array_equal(mask, ref.mask[batch].reshape(-1).astype(bool))
        lstm[env_id] += 1
        for i in np.flatnonzero(mask):
            stored[(int(env_id[i]), step)] += 1
        acts = ref.scripted_actions(300 + step)[batch]          # the policy's sample for this batch
        pool.send(acts.reshape(-1, 12).astype(np.int64))        # clean_pufferl sends int64 numpy
        for j, e in enumerate(batch):
            full[e] = acts[j]
            ref.step_range(e, e + 1, full)
        order.extend(batch)
        steps[batch] += 1
    torch.cuda.synchronize()
    assert np.array_equal(pool.engine.get_state(), ref.get_state())
    assert np.array_equal(lstm.reshape(n, P), np.repeat(steps[:, None], P, axis=1))
    assert max(s for _, s in stored) == 45 and len(stored) > 1000
    eps = ref.get_state().reshape(n, -1)[:, :64].copy().view(np.int32)[:, 3]  # E_EPISODE
    assert (eps >= 1).all()  # every env auto-reset at least once (HORIZON 12, 18 steps each)
    assert pool.engine.get_fault() == 0
    pool.close()


def test_pool_fault_word_raises_at_recv():
    """A tick fault (nmmo_get_fault) surfaces at recv's host sync instead of feeding a learner."""
    from nmmo_amd.engine import TickFault
    from nmmo_amd.vecenv import GpuVecEnv

    cfg = Config.preset("C3", MAP_N=2)
    cfg.obs_layout = 1
    pool = GpuVecEnv(None, num_envs=4, envs_per_batch=2, env_pool=True, config=cfg, seed=1)
    pool.async_reset(3)
    o, r, d, t, infos, env_id, mask = pool.recv()
    pool.send(np.zeros((2 * 128, 12), np.int64))
    pool.engine.inject_fault(1 | 3 << 8)
    with pytest.raises(TickFault, match="attack rounds"):
        pool.recv()
    pool.close()


def test_step_envs_drops_bad_ids_and_records_them():
    """nmmo_step_envs with an id outside the handle: that id is dropped (no out-of-range access),
    the listed valid env steps, and the fault word names the list position."""
    import torch

    from nmmo_amd.engine import NmmoEngine

    cfg = Config.preset("C2", MAP_N=2)
    eng = NmmoEngine(cfg, 3, seed=4)
    eng.reset()
    before = eng.get_state().reshape(3, -1)[:, :4].copy().view(np.int32)[:, 0]
    ids = torch.tensor([2, 7], dtype=torch.int32, device=eng.device)
    eng.step_envs(ids)
    torch.cuda.synchronize()
    after = eng.get_state().reshape(3, -1)[:, :4].copy().view(np.int32)[:, 0]
    assert before.tolist() == [0, 0, 0] and after.tolist() == [0, 0, 1]
    assert eng.get_fault() == 5 | 1 << 8
    eng.close()
