"""The bench's multi-rank path on the one GPU a test box has: `bench.py --gpus 2` starts two ranks
(torch.distributed.run, 127.0.0.1) that share cuda:0 over gloo (NMMO_BENCH_BACKEND=gloo), shard
the envs by env_index_base, time with barriers and reduce max/sum over ranks; C5 adds the learner
gather (wire pack, point-to-point sends, root decode). Small env counts: this checks the path
runs end to end and reports the whole job, not its speed."""

import json
import os
import subprocess
import sys

import pytest

from tests.conftest import gpu_available

pytestmark = [pytest.mark.gpu, pytest.mark.skipif(not gpu_available(), reason="needs a GPU")]
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run(*args):
    env = dict(os.environ, NMMO_BENCH_BACKEND="gloo")
    out = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--steps", "6",
                          "--warmup", "2", "--stagger", "4", "--no-cpu-baseline", *args],
                         capture_output=True, text=True, timeout=110, env=env)
    assert out.returncode == 0, out.stderr[-2000:]
    return json.loads(out.stdout.strip().splitlines()[-1])


def test_two_ranks_c4():
    d = _run("--config", "C4", "--envs", "16")
    assert d["n_gpus"] == 2 and d["config"]["parallelism"] == "env-shard x2"
    assert d["config"]["envs_per_gpu"] == 16
    # alive agent-steps of both ranks per step: at most every slot of 2 x 16 envs x 128 agents
    # (1% for ms_per_step's rounding)
    assert 0 < d["value"] * d["ms_per_step"] / 1e3 <= 2 * 16 * 128 * 1.01
    assert d["slot_steps_per_sec"] * d["ms_per_step"] / 1e3 == pytest.approx(2 * 16 * 128, rel=0.01)


def test_two_ranks_c5_gather():
    d = _run("--config", "C5", "--envs", "8")
    assert d["n_gpus"] == 2
    assert d["gather"] and "B/step" in d["gather"]
