"""bench.py's multi-rank launcher (CPU only, no GPU call): `--gpus N` without WORLD_SIZE starts
N ranks under torch.distributed.run with RANK/WORLD_SIZE set; under torchrun a WORLD_SIZE that
differs from --gpus is refused."""

import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _env(**kw):
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    env.update(kw)
    return env


def test_gpus_n_spawns_n_ranks():
    out = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--dry-launch"],
                         capture_output=True, text=True, timeout=180, env=_env())
    assert out.returncode == 0, out.stderr
    lines = [json.loads(s) for s in out.stdout.splitlines() if s.startswith("{")]
    assert sorted(d["rank"] for d in lines) == [0, 1]
    assert {d["world_size"] for d in lines} == {2}
    assert sorted(d["local_rank"] for d in lines) == [0, 1]


def test_world_size_mismatch_is_refused():
    out = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "4"],
                         capture_output=True, text=True, timeout=120,
                         env=_env(WORLD_SIZE="2", RANK="0", LOCAL_RANK="0"))
    assert out.returncode == 2
    assert "WORLD_SIZE=2" in out.stderr


def test_single_rank_dry_launch():
    out = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--dry-launch"],
                         capture_output=True, text=True, timeout=120, env=_env())
    assert out.returncode == 0
    assert json.loads(out.stdout.strip()) == {"rank": 0, "world_size": 1, "local_rank": 0}


def test_cpu_info_counts_usable_cores():
    sys.path.insert(0, ROOT)
    import bench

    info = bench.cpu_info()
    assert 1 <= info["usable"] <= info["affinity"]
    assert info["usable"] == len(os.sched_getaffinity(0)) or info["cgroup_quota_cpus"]
