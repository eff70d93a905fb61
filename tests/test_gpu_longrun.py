"""The incremental flat rows' row state (flat_obs.hip, DESIGN.md §3.2d: zero rows, zero thresholds,
the Task index, the tracked mask chunks, the Tile position and the item words per row) at the
headline's full size over a long horizon: 1,024 envs, 300 ticks, episode phases staggered over 64
ticks, the reference's manual curriculum (curriculum_generation/manual_curriculum.py:53-314: a
task drawn per player at every reset, so Task sections change at every reset), market listings
from the scripted policy, both kernel variants (flat_obs_kernel<false> bare, <true> under the
start-kit RewardWrapper, baseline_policy.py's agent). Checked:
  - every 16 ticks the tracked buffer is byte-equal to a handle that rewrites every row
    (NMMO_OBS_REZERO=1) -- so no row-state transition (death, respawn, reset, task change,
    listings appearing and expiring, inventory changes) ever left a stale byte;
  - at ticks 64, 128, 256 and 300, 32 sampled envs (the first and the last 16 global envs) equal
    the CPU oracle's flat rows (bare env; the oracle steps those envs on the GPU's actions)."""

import numpy as np
import pytest

from nmmo_amd import abi
from nmmo_amd.config import Config
from tests.conftest import gpu_available

pytestmark = [pytest.mark.gpu, pytest.mark.skipif(not gpu_available(), reason="needs a GPU")]

N, TICKS, STAGGER, CHECK_EVERY = 1024, 300, 64, 16
ORACLE_TICKS = (64, 128, 256, 300)
BLOCKS = ((0, 16), (N - 16, 16))  # (first global env, envs) stepped by the oracle


def _specs():
    """The manual curriculum with a distinct synthetic fp16 embedding per spec (the Task obs then
    changes with every task change)."""
    from nmmo_amd import tasks

    specs = tasks.manual_curriculum()
    rng = np.random.default_rng(5)
    for s in specs:
        s.embedding = rng.standard_normal(2048).astype(np.float16)
    return specs


@pytest.mark.parametrize("wrapper", [None, "neurips23_start_kit"], ids=["bare", "start_kit"])
def test_tracked_rows_full_size_long_horizon(wrapper, monkeypatch):
    import torch

    from nmmo_amd.engine import NmmoEngine
    from nmmo_amd.wrappers import wrapper_config
    from oracle.oracle import OracleEnvs

    specs = _specs()
    cfg = Config.preset("C4", early_stop_agent_num=8, obs_layout=abi.OBS_FLAT)
    assert cfg.MAP_N == 256
    a = NmmoEngine(cfg, N, seed=31)
    monkeypatch.setenv("NMMO_OBS_REZERO", "1")
    b = NmmoEngine(cfg, N, seed=31)
    monkeypatch.delenv("NMMO_OBS_REZERO")
    rows = torch.zeros((N, 2), dtype=torch.int64, device=a.device)
    a.set_obs_counter(rows)
    for e in (a, b):
        e.set_curriculum(specs)
        if wrapper:
            e.set_wrapper(wrapper_config(wrapper, heal_bonus_weight=0.03, explore_bonus_weight=0.01))
        e.reset()
    orcs = []
    if wrapper is None:
        ocfg = Config.preset("C4", early_stop_agent_num=8, obs_layout=abi.OBS_NONE)
        for lo, n in BLOCKS:
            o = OracleEnvs(ocfg, n, seed=31, env_index_base=lo)
            o.set_curriculum(specs)
            o.reset()
            orcs.append((lo, n, o))
    ids = np.arange(N)
    checked = 0
    listed = False
    from nmmo_amd import layout

    mk = layout.flat_layout()["Market"]
    mk_lo = mk.offset
    for t in range(TICKS):
        if t < STAGGER:
            m = ids % STAGGER == t
            a.end_episodes(m)
            b.end_episodes(m)
            for lo, n, o in orcs:
                o.end_episodes(m[lo:lo + n])
        acts = a.scripted_actions(9000 + t)
        b.step(acts.clone())
        a.step(acts)
        if orcs:
            host = acts.cpu().numpy()
            for lo, n, o in orcs:
                o.step(np.ascontiguousarray(host[lo:lo + n]))
        tick = t + 1
        if tick % CHECK_EVERY == 0 or tick == TICKS:
            torch.cuda.synchronize()
            assert torch.equal(a.obs.view(torch.int32), b.obs.view(torch.int32)), f"tracked != full write at tick {tick}"
            checked += 1
            listed = listed or bool((a.obs[:, 0, mk_lo:mk_lo + 16] != 0).any())
        if orcs and tick in ORACLE_TICKS:
            for lo, n, o in orcs:
                for k in range(n):
                    g = a.obs[lo + k].cpu().numpy()
                    want = o.flat_obs(k)
                    if not np.array_equal(g, want):
                        bad = np.argwhere(g != want)[:5]
                        raise AssertionError(f"tick {tick} env {lo + k}: obs differ at {bad.tolist()}")
    assert checked >= TICKS // CHECK_EVERY
    assert listed, "no market listing appeared in the window"
    st = a.get_state().reshape(N, -1)[:, :abi.NE * 4].copy().view(np.int32)
    eps = st[:, abi.ENV_FIELDS.index("episode")]
    assert int(eps.min()) >= 1, "every env reset inside the window"
    assert int(eps.sum()) > N + N // 4, "episodes ended on their own after the staggered ends"
    assert a.get_fault() == 0 and b.get_fault() == 0
    # incremental: far fewer bytes stored than full rows
    stored = int(rows[:, 1].sum().item())
    assert 0 < stored < TICKS * N * a.P * a.obs_elems * 4 // 8, stored
    a.close()
    b.close()
