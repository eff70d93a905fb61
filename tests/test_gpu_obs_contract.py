"""The obs contract at the pool boundary (nmmo_amd.vecenv module docstring, nmmo_hip.h
nmmo_obs_invalidate_envs / nmmo_obs_invalidate_sections). recv() hands out views of the engine's
incrementally written obs buffer; the reference's start-kit policy edits its input in place (the
TileEncoder, agent_zoo/neurips23_start_kit/baseline_policy.py:96-97, on unpack_batched_obs views).
Under the pool's obs_writes contract every recv() must still equal the oracle's full-write obs
whatever the consumer did to the previous ones: here a consumer edits every recv() output in place
-- the start-kit's Tile edit (idempotent) or a non-idempotent one that touches every region the
incremental gather skips (Entity and Market zero tails, Buy entries, Task, rows of agents out of
the realm) -- in the reference's default 15/6 async pool and in lockstep, over deaths and
auto-resets. obs_writes="all" rewrites whole rows; obs_writes={"Tile"} rewrites only the Tile
sections and is exact for the start-kit edit; an edit outside the declared sections, or any edit
under obs_readonly=True, diverges (the declaration is what keeps it exact)."""

import collections

import numpy as np
import pytest

from nmmo_amd import layout
from nmmo_amd.config import Config

pytestmark = pytest.mark.gpu


def start_kit_tile_edit(o):
    """baseline_policy.py:96-97 restated on this layout's views."""
    tile = layout.unflatten(o)["Tile"]
    tile[:, :, :2] -= tile[:, 112:113, :2].clone()
    tile[:, :, :2] += 7


def non_idempotent_edit(o):
    """Every region an incremental row leaves alone, edited so that applying it twice differs."""
    d = layout.unflatten(o)
    d["Entity"] /= 2
    d["Market"] += 1
    d["Task"] *= 3
    d["ActionTargets"]["Buy"]["MarketItem"] += 2
    d["Tile"][:, :, 2] -= 1


EDITS = {"start_kit_tile": start_kit_tile_edit, "non_idempotent": non_idempotent_edit}


def _run_pool(n, k, edit, readonly, steps, seed=5, writes=None, reset_at=None):
    """Drive GpuVecEnv like clean_pufferl.evaluate (recv -> policy -> send) against the oracle
    stepping each env on the same action stream; returns the recv() indices whose obs differed."""
    import torch

    from nmmo_amd.vecenv import GpuVecEnv, reset_seeds
    from oracle.oracle import OracleEnvs

    P = 128
    # deaths from tick ~22, early-stop resets from ~30 (oracle rollout of these seeds)
    cfg = Config.preset("C4", MAP_N=4, early_stop_agent_num=8)
    pool = GpuVecEnv(None, env_kwargs=None, num_envs=n, envs_per_batch=k, env_pool=k < n, config=cfg,
                     seed=seed, obs_readonly=readonly, obs_writes=writes)
    ref = OracleEnvs(cfg, n, seed=seed)
    pool.async_reset(1)
    ref.reset(env_seeds=reset_seeds(1, 0, n))
    order = collections.deque(range(n))
    full = np.zeros((n, P, 12), np.int32)
    bad, dead_rows = [], 0
    for step in range(steps):
        o, r, d, t, infos, env_id, mask = pool.recv()
        batch = [order.popleft() for _ in range(k)]
        want = ref.obs[batch].reshape(k * P, -1)
        if not np.array_equal(o.cpu().numpy(), want):
            bad.append(step)
        dead_rows += int((~mask).sum())
        EDITS[edit](o)  # the consumer's in-place edit of what recv handed out
        if step == reset_at:  # the pool resets right after a recv whose rows the consumer edited
            pool.async_reset(2)
            ref.reset(env_seeds=reset_seeds(2, 0, n))
            order = collections.deque(range(n))
            continue
        acts = ref.scripted_actions(500 + step)[batch]
        pool.send(acts.reshape(-1, 12).astype(np.int64))
        for j, e in enumerate(batch):
            full[e] = acts[j]
            ref.step_range(e, e + 1, full)
        order.extend(batch)
    torch.cuda.synchronize()
    assert np.array_equal(pool.engine.get_state(), ref.get_state())
    if reset_at is None:
        eps = ref.get_state().reshape(n, -1)[:, :64].copy().view(np.int32)[:, 3]  # E_EPISODE
        assert (eps >= 1).all(), "every env auto-reset at least once"
    assert dead_rows > 0, "no agent out of the realm in the window"
    assert pool.engine.get_fault() == 0
    pool.close()
    return bad


@pytest.mark.parametrize("edit", sorted(EDITS))
@pytest.mark.parametrize("shape", [(15, 6), (4, 4)], ids=["pool15x6", "lockstep4"])
def test_mutating_consumer_gets_full_write_obs(edit, shape):
    n, k = shape
    bad = _run_pool(n, k, edit, readonly=False, steps=130 if k < n else 45)
    assert not bad, f"recv() obs differ from the oracle at steps {bad}"


@pytest.mark.parametrize("shape", [(15, 6), (4, 4)], ids=["pool15x6", "lockstep4"])
def test_start_kit_edit_under_tile_writes_stays_exact(shape):
    """obs_writes={"Tile"} (the start-kit agent's default): only the handed-out rows' Tile sections
    are rewritten next step (nmmo_obs_invalidate_sections), including the Tile of rows out of the
    realm the edit made nonzero, and every recv() equals the oracle."""
    n, k = shape
    bad = _run_pool(n, k, "start_kit_tile", readonly=False, steps=130 if k < n else 45, writes={"Tile"})
    assert not bad, f"recv() obs differ from the oracle at steps {bad}"


def test_edit_outside_the_declared_sections_diverges():
    """The declaration is what keeps it exact: an edit of sections other than Tile under
    obs_writes={"Tile"} leaves stale bytes in later recv() outputs."""
    bad = _run_pool(4, 4, "non_idempotent", readonly=False, steps=45, writes={"Tile"})
    assert bad, "an undeclared edit should leave stale bytes"


@pytest.mark.parametrize("writes", [None, {"Tile"}], ids=["all", "tile"])
def test_reset_after_an_edited_recv(writes):
    """async_reset after a recv() whose rows the consumer edited: the reset's gather forgets what
    the consumer may have written (the rows of every env), and the recv() after it equals the
    oracle's reset obs."""
    edit = "non_idempotent" if writes is None else "start_kit_tile"
    bad = _run_pool(4, 4, edit, readonly=False, steps=60, writes=writes, reset_at=35)
    assert not bad, f"recv() obs differ from the oracle at steps {bad}"


def test_readonly_mode_is_what_the_flag_says():
    """obs_readonly=True keeps the rows incremental, so a consumer that writes into them breaks
    later recv() outputs: the default mode above is what makes in-place edits safe."""
    bad = _run_pool(4, 4, "non_idempotent", readonly=True, steps=45)
    assert bad, "a writing consumer under obs_readonly=True should leave stale bytes"


def test_invalidate_envs_forgets_only_the_listed_envs():
    """nmmo_obs_invalidate_envs: a write into the skipped part of two envs' rows survives the next
    gather for the env not listed and is rewritten for the listed one (ids outside the handle are
    ignored)."""
    import torch

    from nmmo_amd.engine import NmmoEngine

    cfg = Config.preset("C4", MAP_N=4, early_stop_agent_num=8)
    eng = NmmoEngine(cfg, 3, seed=9)
    eng.reset()
    for t in range(4):
        eng.scripted_actions(70 + t)
        eng.step()
    task = layout.flat_layout()["Task"].offset
    eng.obs[0, :, task:task + 8].fill_(5.0)  # Task sections are not rewritten while the task holds
    eng.obs[2, :, task:task + 8].fill_(5.0)
    before = eng.obs[2, :, task:task + 8].clone()
    eng.obs_invalidate_envs(torch.tensor([2, 99], dtype=torch.int32, device=eng.device))
    eng.observe()
    torch.cuda.synchronize()
    assert bool((eng.obs[0, :, task:task + 8] == 5.0).all()), "env 0 was not listed"
    assert not torch.equal(eng.obs[2, :, task:task + 8], before), "env 2 was listed"
    assert eng.get_fault() == 0
    eng.close()
