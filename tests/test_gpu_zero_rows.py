"""The obs gather's zero-row skip on MI355X (nmmo_hip.h nmmo_obs_invalidate): rows of agents out
of the realm are zeroed once per buffer and then left alone. Over deaths, early-stop resets and
staggered episode ends, the tracked buffer's bytes after every step equal a handle that rewrites
every zero row (NMMO_OBS_REZERO=1), flat and native; the row counter says rows were skipped; a
caller's write into a skipped row survives until nmmo_obs_invalidate, after which the row is
zero again; an untracked buffer (torch's allocator) gets every row."""

import os

import numpy as np
import pytest
import torch

from tests.conftest import gpu_available

pytestmark = [pytest.mark.gpu, pytest.mark.skipif(not gpu_available(), reason="needs a GPU")]


def _engines(layout, n, seed):
    from nmmo_amd import abi
    from nmmo_amd.config import Config
    from nmmo_amd.engine import NmmoEngine

    cfg = Config.preset("C4", MAP_N=4, early_stop_agent_num=64,
                        obs_layout=abi.OBS_FLAT if layout == "flat" else abi.OBS_NATIVE)
    a = NmmoEngine(cfg, n, seed=seed)
    os.environ["NMMO_OBS_REZERO"] = "1"
    try:
        b = NmmoEngine(cfg, n, seed=seed)
    finally:
        del os.environ["NMMO_OBS_REZERO"]
    return a, b


def _rows(eng):
    n, P = eng.n_envs, eng.P
    return eng.obs.view(n, P, -1) if eng.obs.dim() == 3 else \
        eng.obs[:, :P * 9552].reshape(n, P, 9552)


@pytest.mark.parametrize("layout", ["flat", "native"])
def test_zero_row_skip_equals_full_write(layout):
    n = 4
    a, b = _engines(layout, n, seed=21)
    ca = torch.zeros((n, 2), dtype=torch.int64, device=a.device)
    cb = torch.zeros((n, 2), dtype=torch.int64, device=b.device)
    a.set_obs_counter(ca)
    b.set_obs_counter(cb)
    a.reset()
    b.reset()
    ids = np.arange(n)
    launches = 1
    for t in range(160):
        if t % 40 == 39:
            m = ids == (t // 40) % n
            a.end_episodes(m)
            b.end_episodes(m)
        a.scripted_actions(4100 + t)
        b.scripted_actions(4100 + t)
        a.step()
        b.step()
        launches += 1
        if t % 8 == 7:
            torch.cuda.synchronize()
            assert torch.equal(a.obs.view(torch.uint8), b.obs.view(torch.uint8)), f"tick {t}"
    torch.cuda.synchronize()
    assert torch.equal(a.obs.view(torch.uint8), b.obs.view(torch.uint8))
    ca, cb = ca.sum(0), cb.sum(0)
    total = launches * n * a.P
    assert int(cb[0].item()) == total  # every row, every launch
    assert int(ca[0].item()) < total, "no zero row was skipped (buffer not tracked?)"
    if layout == "flat":  # the zero runs, unchanged Task sections and dead rows were not stored
        assert int(ca[1].item()) < int(cb[1].item()) // 4, (int(ca[1].item()), int(cb[1].item()))
    assert int(cb[1].item()) == total * (a.obs_elems * 4 if layout == "flat" else 9552)
    zero = (_rows(a) == 0).all(-1)
    assert bool(zero.any()), "no agent left the realm in the window"

    # a caller's write into a skipped row survives the next gather ...
    e, ag = [int(x) for x in torch.nonzero(zero)[0]]
    _rows(a)[e, ag].fill_(7)
    a.observe()
    torch.cuda.synchronize()
    assert bool((_rows(a)[e, ag] == 7).all())
    # ... until the handle forgets its zero rows
    a.obs_invalidate()
    a.observe()
    b.observe()
    torch.cuda.synchronize()
    assert torch.equal(a.obs.view(torch.uint8), b.obs.view(torch.uint8))

    # an untracked buffer gets every row, zero rows included
    out = torch.full_like(a.obs, 0x5A if layout == "native" else float("nan"))
    a.observe(out=out)
    torch.cuda.synchronize()
    assert torch.equal(out.view(torch.uint8), a.obs.view(torch.uint8))
    a.close()
    b.close()
