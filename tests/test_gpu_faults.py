"""The tick fault word (nmmo_get_fault: a launch hit one of its loop bounds, so its env's tick is
not the serial-order result) stops every product path at its existing host sync instead of
feeding a learner or a bench line. The test-only hook nmmo_inject_fault sets the word; the pool's
recv() check is in tests/test_gpu_vecenv.py."""

import os
import subprocess
import sys

import pytest
import torch

from nmmo_amd.config import Config
from tests.conftest import gpu_available

pytestmark = [pytest.mark.gpu, pytest.mark.skipif(not gpu_available(), reason="needs a GPU")]

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_bench_exits_nonzero_without_a_line_on_a_fault():
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    out = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--config", "C2", "--envs", "8",
                          "--steps", "3", "--warmup", "1", "--stagger", "2", "--batches", "1",
                          "--no-cpu-baseline", "--inject-fault"],
                         capture_output=True, text=True, timeout=300, env=env)
    assert out.returncode != 0
    assert out.stdout.strip() == ""
    assert "tick fault word" in out.stderr


def test_wire_gather_raises_at_the_payload_of_a_faulted_step():
    from nmmo_amd import abi
    from nmmo_amd.distributed import WireGather
    from nmmo_amd.engine import NmmoEngine, TickFault

    cfg = Config.preset("C4", MAP_N=2, early_stop_agent_num=8, obs_layout=abi.OBS_WIRE)
    engs = [NmmoEngine(cfg, 2, seed=3, env_index_base=2 * i) for i in range(2)]
    for e in engs:
        e.reset()
    g = WireGather(engs, 11, graphs=True)
    for _ in range(3):
        g.step()
    torch.cuda.synchronize()
    engs[1].inject_fault(2 | 1 << 8)
    g.step()  # step 3 ships the word with its sizes
    with pytest.raises(TickFault, match="Buy rounds"):
        g.step()  # posts step 3's payload
    g.close()
    for e in engs:
        e.close()


def test_device_trainer_raises_at_the_batch_boundary():
    from nmmo_amd.engine import NmmoEngine, TickFault
    from nmmo_amd.trainer import DeviceTrainer, MaskedLinearAgent, TrainConfig

    cfg = Config.preset("C4", MAP_N=2, early_stop_agent_num=8)
    eng = NmmoEngine(cfg, 1, seed=5)
    eng.reset()
    agent = MaskedLinearAgent(cfg.TASK_EMBED_DIM).cuda()
    tr = DeviceTrainer(eng, agent, TrainConfig(batch_size=128, batch_rows=16, bptt_horizon=8,
                                               total_timesteps=1024))
    tr.evaluate()
    eng.inject_fault(4)
    with pytest.raises(TickFault, match="position-hash"):
        tr.evaluate()
    eng.close()
