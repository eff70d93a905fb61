"""The multi-rank paths on the one GPU a test box has: ranks started by torch.distributed.run
(127.0.0.1) share cuda:0 over gloo.

- `bench.py --gpus 2` shards the envs by env_index_base, times with barriers and reduces
  max/sum over ranks (C4), and runs the C5 learner gather (delivered and decoded passes).
- The C5 content check (tests/_c5_worker.py): what rank 0 receives and decodes every step —
  native obs, reward / term / trunc / mask of every env of both ranks — and the experience rows
  it stores straight from the wire records equal one engine stepping all envs alone, bit for
  bit, over 18 ticks with staggered episode ends.
Small env counts: these check the paths end to end, not their speed."""

import json
import os
import socket
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


def test_two_ranks_c5_is_the_default_multi_gpu_line():
    d = _run("--envs", "8")  # no --config: N > 1 measures C5
    assert d["n_gpus"] == 2 and d["config"]["workload"].startswith("C5")
    assert d["value_kind"] == "delivered" and d["decoded"]["value"] > 0 and d["stored"]["value"] > 0
    # the root stored every row in the realm of both ranks: the rows/s equal the alive agent-steps/s
    # of the stored pass (env side), within timing rounding
    assert d["stored"]["rows_stored_per_sec"] == pytest.approx(d["stored"]["value"], rel=0.02)
    assert d["gather_bytes_per_step"] > 0 and "B/step" in d["gather"]
    assert 0 < d["value"] * d["ms_per_step"] / 1e3 <= 2 * 8 * 128 * 1.01


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _reference(world, mode="eager"):
    """One NATIVE-obs engine over all world x envs envs, the worker's schedule."""
    import numpy as np
    import torch

    from nmmo_amd import abi
    from nmmo_amd.config import Config
    from nmmo_amd.engine import NmmoEngine
    from nmmo_amd.storage import DeviceExperience
    from tests import _c5_worker as w

    N = world * w.N_PER_BATCH * w.BATCHES  # the same 12 global envs for every split
    cfg = Config.preset("C4", MAP_N=w.MAP_N, early_stop_agent_num=8, obs_layout=abi.OBS_NATIVE,
                        HORIZON=w.horizon(mode))
    eng = NmmoEngine(cfg, N, seed=w.SEED)
    P = eng.P
    eng.reset()
    ids = np.arange(N)
    for k in range(w.PREROLL):
        eng.end_episodes(w.preroll_mask(ids, k))
        eng.scripted_actions(w.PSEED)
        eng.step(write_obs=False)
    x = DeviceExperience(w.TICKS * N * P, eng.obs_elems, N * P, device=eng.device)
    xs = DeviceExperience(N * P, eng.obs_elems, N * P, device=eng.device)  # one step's rows
    rec = {"native": {}, "small": {}, "stored": {}}
    z = torch.zeros(N * P, device=eng.device)
    cnt = torch.zeros(3, dtype=torch.int64, device=eng.device)
    eng.set_counters(cnt)
    for t in range(w.TICKS):
        if mode == "eager":
            eng.end_episodes(w.end_mask(ids, t))
        eng.scripted_actions(w.PSEED)
        eng.step()
        small = torch.cat([eng.rew.view(torch.uint8).view(N, P, 4), eng.term[..., None], eng.trunc[..., None],
                           eng.mask[..., None]], -1)
        for i in range(N):
            rec["native"][f"{t}:{i}"] = w.digest(eng.obs[i])
            rec["small"][f"{t}:{i}"] = w.digest(small[i])
        x.store(eng.obs, eng.rew.view(-1), eng.term.view(-1), eng.mask.view(-1),
                torch.zeros((N * P, 12), dtype=torch.int32), z, z, step=t + 1, engine=eng)
        xs.reset()
        xs.store(eng.obs, eng.rew.view(-1), eng.term.view(-1), eng.mask.view(-1),
                 torch.zeros((N * P, 12), dtype=torch.int32), z, z, step=t + 1, engine=eng)
        k = xs.ptr
        rec["stored"][str(t)] = {"ptr": k, "obs": w.digest(xs.obs[:k]), "rewards": w.digest(xs.rewards[:k]),
                                 "dones": w.digest(xs.dones[:k]), "env_id": w.digest(xs.env_id[:k])}
    torch.cuda.synchronize()
    k = x.ptr
    rec["exp"] = {"ptr": k, "obs": w.digest(x.obs[:k]), "rewards": w.digest(x.rewards[:k]),
                  "dones": w.digest(x.dones[:k]), "env_id": w.digest(x.env_id[:k]), "step": w.digest(x.step[:k])}
    rec["episodes"] = int(cnt[1].item())
    eng.close()
    return rec


@pytest.mark.parametrize("mode,split,store", [("eager", "even", ""), ("graphs", "even", ""),
                                              ("eager", "uneven", "store"), ("graphs", "uneven", "store"),
                                              ("graphs", "uneven", "store-noplan")])
def test_c5_gather_content_matches_one_rank(tmp_path, mode, split, store):
    """eager: per-step episode ends, WireGather(graphs=False). graphs: the mode bench.py times —
    every (batch, ring slot) replayed from its hipGraph, ring slots reused every 3 steps behind
    cross-stream done events — with episodes ended by a horizon inside the checked window.
    uneven: the learner's smaller share (rank 0 1 env per batch, rank 1 5). store: rank 0's
    gather also keeps every step's rows in its compact record store (the fused checked store, the
    peer received straight into its arena slot; store-noplan: received into the exchange's buffers
    and copied), and each step's stored rows equal one engine's rows of that step."""
    out = tmp_path / "c5.json"
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()),
           os.path.join(ROOT, "tests", "_c5_worker.py"), str(out), mode, split, store]
    env = dict(os.environ, OMP_NUM_THREADS="1")
    p = subprocess.run(cmd, capture_output=True, text=True, timeout=110, env=env)
    assert p.returncode == 0, p.stderr[-3000:]
    got = json.loads(out.read_text())
    ref = _reference(2, mode)
    assert got["status"] == 0
    assert ref["episodes"] > 0  # episodes ended (and auto-reset) inside the checked window
    assert set(got["native"]) == set(ref["native"]) and len(ref["native"]) == 18 * 12
    bad = [k for k in ref["native"] if got["native"][k] != ref["native"][k]]
    assert not bad, f"decoded obs differ at (tick:env) {bad[:8]}"
    bad = [k for k in ref["small"] if got["small"][k] != ref["small"][k]]
    assert not bad, f"reward/dones/mask differ at (tick:env) {bad[:8]}"
    assert got["exp"] == ref["exp"]
    assert got["payload_bytes"] > 0
    if store:
        assert got["store_status"] == 0
        assert set(got["stored"]) == set(ref["stored"])
        bad = [k for k in ref["stored"] if got["stored"][k] != ref["stored"][k]]
        assert not bad, f"the gather's stored rows differ at steps {bad[:8]}"
