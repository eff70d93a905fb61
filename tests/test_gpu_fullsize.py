"""HIP path vs the CPU oracle at the benchmark configs' real sizes (BASELINE.json configs[1..3]):
C2 = 256 envs, C3 = 1024 envs, C4 = 1024 envs with the flat obs buffer (1024 x 128 x 23,987
float32 = 3.1 G elements, past 2^31), all over the full 256-map bank, so env indices >= 256,
map ids across the whole bank and 1024-workgroup grids at 2-3 workgroups per CU are compared
with the oracle, not only the 1-6-env cases of test_gpu_parity.py. Episode phases are staggered
with nmmo_end_episodes (as bench.py does), so culls and in-kernel auto-resets happen inside the
compared window. Bit-exact on every integer state field, output, event row and obs element.

The oracle (test infrastructure only) steps env ranges on host threads (the GIL is released
inside its C calls)."""

import os
from concurrent.futures import ThreadPoolExecutor

import numpy as np
import pytest

from nmmo_amd import abi
from nmmo_amd.config import Config
from oracle.oracle import OracleEnvs
from oracle.oracle import lib as olib
from tests.test_gpu_parity import _cmp_events, _cmp_state

pytestmark = pytest.mark.gpu

THREADS = max(1, min(16, len(os.sched_getaffinity(0))))


class _ThreadedOracle:
    def __init__(self, cfg, n, seed, task):
        self.o = OracleEnvs(cfg, n, seed=seed, task_embedding=task)
        self.n = n
        self.pool = ThreadPoolExecutor(THREADS)
        k = -(-n // THREADS)
        self.ranges = [(lo, min(n, lo + k)) for lo in range(0, n, k)]

    def actions(self, pseed):
        a = np.zeros((self.n, self.o.P, abi.N_ACTION_HEADS), np.int32)
        list(self.pool.map(lambda r: olib().oracle_scripted_actions_range(self.o.h, r[0], r[1], pseed,
                                                                           a.ctypes.data), self.ranges))
        return a

    def step(self, a):
        list(self.pool.map(lambda r: self.o.step_range(r[0], r[1], a), self.ranges))


def _run(preset, n_envs, ticks, stagger, obs_envs=(), check_every=8):
    import torch

    from nmmo_amd.engine import NmmoEngine

    layout = abi.OBS_FLAT if obs_envs else abi.OBS_NONE
    cfg = Config.preset(preset, early_stop_agent_num=8, obs_layout=layout)
    assert cfg.MAP_N == 256
    ocfg = Config.preset(preset, early_stop_agent_num=8, obs_layout=abi.OBS_NONE)
    task = (np.arange(2048) % 89 / 89.0 - 0.5).astype(np.float16)
    eng = NmmoEngine(cfg, n_envs, seed=21, task_embedding=task)
    orc = _ThreadedOracle(ocfg, n_envs, 21, task)
    eng.reset()
    orc.o.reset()
    ids = np.arange(n_envs)
    episodes_seen = 0
    for t in range(ticks):
        if t < stagger:
            m = ids % stagger == t
            eng.end_episodes(m)
            orc.o.end_episodes(m)
        pseed = 5000 + t
        ga = eng.scripted_actions(pseed)
        oa = orc.actions(pseed)
        if not np.array_equal(ga.cpu().numpy(), oa):
            bad = np.argwhere(ga.cpu().numpy() != oa)[:5]
            raise AssertionError(f"{preset} tick {t}: scripted actions differ at {bad.tolist()}")
        eng.step(ga)
        orc.step(oa)
        torch.cuda.synchronize()
        for name in ("rew", "term", "trunc", "mask"):
            gv = getattr(eng, name).cpu().numpy()
            ov = getattr(orc.o, name)
            if not np.array_equal(gv, ov):
                bad = np.argwhere(gv != ov)[:5]
                raise AssertionError(f"{preset} tick {t}: {name} differs at {bad.tolist()}")
        if t % check_every == check_every - 1 or t == ticks - 1:
            gs, os_ = eng.get_state(), orc.o.get_state()
            _cmp_state(gs, os_, n_envs, eng.S, f"{preset} tick {t}")
            env = gs.reshape(n_envs, -1)[:, :abi.NE * 4].copy().view(np.int32)
            episodes_seen = int(env[:, abi.ENV_FIELDS.index("episode")].sum())
            if cfg.event_cap > 0:
                _cmp_events(eng, orc.o, n_envs, f"{preset} tick {t}")
            for e in obs_envs:
                g = eng.obs[e].cpu().numpy()
                o = orc.o.flat_obs(e)
                if not np.array_equal(g, o):
                    bad = np.argwhere(g != o)[:5]
                    raise AssertionError(f"{preset} tick {t}: env {e} obs differs at {bad.tolist()}")
    eng.close()
    return episodes_seen


def test_c2_full_size():
    ep = _run("C2", 256, ticks=128, stagger=32)
    assert ep > 256  # every env ended at least one episode inside the window


def test_c3_full_size():
    ep = _run("C3", 1024, ticks=96, stagger=32)
    assert ep > 1024


def test_c4_full_size_flat_obs():
    import torch

    free, _ = torch.cuda.mem_get_info()
    need = 1024 * 128 * 23987 * 4
    assert free > need * 1.2, "C4 flat obs needs ~12.6 GB of HBM"
    _run("C4", 1024, ticks=32, stagger=16, obs_envs=(0, 1, 255, 256, 511, 777, 1022, 1023), check_every=4)


def test_run_to_run_determinism():
    """The same seeds and action stream twice on two engines: identical state, outputs and obs
    (no dependence on scheduling: LDS atomics, wave order, graph replay)."""
    import hashlib

    import torch

    from nmmo_amd.engine import NmmoEngine

    cfg = Config.preset("C4", early_stop_agent_num=8, obs_layout=abi.OBS_NATIVE)
    digests = []
    for run in range(2):
        eng = NmmoEngine(cfg, 1024, seed=77)
        eng.reset()
        h = hashlib.sha256()
        for t in range(40):
            if t < 16:
                eng.end_episodes(np.arange(1024) % 16 == t)
            eng.scripted_actions(900 + t)
            eng.step()
            if t % 8 == 7:
                torch.cuda.synchronize()
                for x in (eng.obs, eng.rew, eng.term, eng.trunc, eng.mask):
                    h.update(x.cpu().numpy().tobytes())
                h.update(eng.get_state().tobytes())
        digests.append(h.hexdigest())
        eng.close()
    assert digests[0] == digests[1]


def test_long_rollout_rounds_finish():
    """600 ticks of the bench's C4 scenario (1,024 envs, staggered): every round loop of every
    tick ends by its serial-order bound (fault word 0). With one round-key array a wave still
    checking round r could see round r + 1's bids and miss its turn; repeated, a launch never
    finished (hung on MI355X at tick 184 of this scenario before the keys were double-buffered)."""
    import torch

    from nmmo_amd.engine import NmmoEngine

    cfg = Config.preset("C4", early_stop_agent_num=8, obs_layout=abi.OBS_NONE)
    eng = NmmoEngine(cfg, 1024, seed=1)
    eng.reset()
    assert eng.get_fault() == 0
    for t in range(600):
        if t < 64:
            eng.end_episodes(np.arange(1024) % 64 == t)
        eng.scripted_actions(1_000_003)
        eng.step()
        if t % 50 == 49:
            torch.cuda.synchronize()
            assert eng.get_fault() == 0, f"tick {t}: fault word {eng.get_fault():#x}"
    eng.close()
