"""A map bank loaded from PATH_MAPS drives the HIP engine bit-exactly like
the CPU oracle given the same bank; NmmoEngine follows nmmo's PATH_MAPS / MAP_FORCE_GENERATION
preparation (generate + save when absent or forced, load otherwise)."""

import numpy as np
import pytest

from nmmo_amd import maps
from nmmo_amd.config import Config

pytestmark = pytest.mark.gpu


def test_foreign_bank_parity(tmp_path):
    import torch

    from nmmo_amd.engine import NmmoEngine
    from oracle.oracle import OracleEnvs

    cfg = Config.preset("C4", MAP_N=3, early_stop_agent_num=8)
    src = OracleEnvs(cfg, 1, seed=9).map_bank()
    foreign = np.ascontiguousarray(src[:, :, ::-1].transpose(0, 2, 1))
    maps.save_map_bank(foreign, str(tmp_path))
    cfg_disk = Config.preset("C4", MAP_N=3, early_stop_agent_num=8, PATH_MAPS=str(tmp_path))
    eng = NmmoEngine(cfg_disk, 3, seed=9)
    assert eng.maps_source == "loaded"
    assert np.array_equal(eng.map_bank(), foreign)
    orc = OracleEnvs(cfg, 3, seed=9)
    orc.set_map_bank(foreign)
    eng.reset()
    orc.reset()
    for t in range(40):
        a = orc.scripted_actions(t)
        orc.step(a)
        eng.step(torch.from_numpy(a).cuda())
    torch.cuda.synchronize()
    assert np.array_equal(eng.get_state(), orc.get_state())
    assert np.array_equal(eng.obs.cpu().numpy(), orc.obs)
    eng.close()


def test_prepare_generates_then_loads(tmp_path):
    from nmmo_amd.engine import NmmoEngine

    d = str(tmp_path / "maps" / "128")
    e1 = NmmoEngine(Config.preset("C2", MAP_N=2, PATH_MAPS=d, map_seed=5), 1)
    assert e1.maps_source == "generated" and maps.available(d, 2)
    gen = e1.map_bank()
    e2 = NmmoEngine(Config.preset("C2", MAP_N=2, PATH_MAPS=d, map_seed=6), 1)
    assert e2.maps_source == "loaded" and np.array_equal(e2.map_bank(), gen)
    e3 = NmmoEngine(Config.preset("C2", MAP_N=2, PATH_MAPS=d, map_seed=6, MAP_FORCE_GENERATION=True), 1)
    assert e3.maps_source == "generated" and not np.array_equal(e3.map_bank(), gen)
    for e in (e1, e2, e3):
        e.close()
