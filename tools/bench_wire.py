"""Wire codec (SPEC §8c) at C4 size on one GPU: bytes per agent in steady state (staggered
episodes) and the pack / unpack kernel times (HIP events on the launch stream).

Usage (GPU box): python tools/bench_wire.py [envs] [stagger]
"""

import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402
import torch  # noqa: E402

from nmmo_amd import abi, wire  # noqa: E402
from nmmo_amd.config import Config  # noqa: E402
from nmmo_amd.engine import NmmoEngine  # noqa: E402


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 1024
    L = int(sys.argv[2]) if len(sys.argv) > 2 else 64
    cfg = Config.preset("C4", early_stop_agent_num=8, obs_layout=abi.OBS_NATIVE)
    eng = NmmoEngine(cfg, n, seed=1)
    eng.reset()
    ids = np.arange(n)
    for k in range(L):
        eng.end_episodes(ids % L == k)
        eng.scripted_actions(1_000_003 + k)
        eng.step()
    for k in range(20):  # steady-state ticks after the pre-roll
        eng.scripted_actions(7 + k)
        eng.step()
    w = wire.pack(eng)
    native = torch.empty_like(eng.obs)
    t0, t1, t2 = (torch.cuda.Event(enable_timing=True) for _ in range(3))
    reps = 20
    t0.record()
    for _ in range(reps):
        wire.pack(eng, out=w)
    t1.record()
    for _ in range(reps):
        wire.unpack(w, n, eng.P, out=native)
    t2.record()
    torch.cuda.synchronize()
    assert torch.equal(native, eng.obs)
    total = wire.total_bytes(w)
    alive = int(eng.mask.sum())
    nat_bytes = eng.obs.numel()
    pack_ms, unpack_ms = t0.elapsed_time(t1) / reps, t1.elapsed_time(t2) / reps
    print(json.dumps({
        "workload": f"C4 native, {n} envs x 128 agents, {L}-tick staggered pre-roll + 20 ticks",
        "native_bytes": nat_bytes, "wire_bytes": total, "ratio": round(nat_bytes / total, 2),
        "agents_in_realm": alive, "wire_bytes_per_agent_in_realm": round(total / max(alive, 1), 1),
        "wire_bytes_per_slot": round(total / (n * eng.P), 1),
        "pack_ms": round(pack_ms, 4), "unpack_ms": round(unpack_ms, 4),
        "unpack_write_gbs": round(nat_bytes / (unpack_ms * 1e-3) / 1e9, 1),
    }))
    eng.close()


if __name__ == "__main__":
    main()
