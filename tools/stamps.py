"""Phase attribution of the tick kernel from in-kernel s_memtime stamps (diagnostic build).

Usage (GPU box): python tools/stamps.py [C3] [envs] [warmup]
Builds nothing on the box: run `python -c "from nmmo_amd import build; build.build(stamps=True)"`
here first (the .so travels with the snapshot). Prints median / p90 cycles per phase.
"""

import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
os.environ["NMMO_LIB"] = os.path.join(ROOT, "nmmo_amd", "lib", "libnmmo_hip_stamps.so")

import numpy as np  # noqa: E402
import torch  # noqa: E402

from nmmo_amd import _native, abi  # noqa: E402
from nmmo_amd.config import Config  # noqa: E402
from nmmo_amd.engine import NmmoEngine  # noqa: E402

PHASES = ["load", "rowslot", "decode+npc_decide", "update+harvest", "professions+items",
          "attack rounds+loot", "move", "cull+compact", "respawn", "npc_spawn", "rewards", "store"]


def main():
    preset = sys.argv[1] if len(sys.argv) > 1 else "C3"
    envs = int(sys.argv[2]) if len(sys.argv) > 2 else 1024
    warm = int(sys.argv[3]) if len(sys.argv) > 3 else 40
    cfg = Config.preset(preset, early_stop_agent_num=8,
                        obs_layout=abi.OBS_FLAT if preset == "C4" else abi.OBS_NONE)
    eng = NmmoEngine(cfg, envs, seed=1)
    eng.reset()
    stagger = int(os.environ.get("STAMPS_STAGGER", "0"))  # bench.py's staggered pre-roll
    for k in range(stagger):
        eng.end_episodes(np.arange(envs) % stagger == k)
        eng.scripted_actions(1_000_003)
        eng.step(write_obs=False)
    totals = []
    L = _native.lib()
    L.nmmo_debug_read_stamps.argtypes = [ctypes.c_void_p, ctypes.c_int]
    rows, subs = [], []
    for t in range(warm + 10):
        eng.scripted_actions(1000 + t)
        eng.step()
        torch.cuda.synchronize()
        if t >= warm:
            buf = np.zeros(4096 * 32, np.uint64)
            assert L.nmmo_debug_read_stamps(buf.ctypes.data_as(ctypes.c_void_p), buf.size) == 0
            st = buf.reshape(4096, 32)[:min(envs, 4096), :12].astype(np.int64)
            fin = st[:, 11] > st[:, 0]
            totals.append(np.stack([st[fin, 11] - st[fin, 0], (st[fin, 2] > 0).astype(np.int64)], 1))
            ok = (st[:, 2] > 0) & (st[:, 11] > st[:, 0])  # stepped (not reset) envs
            d = np.diff(st[ok], axis=1)
            rows.append(d)
            full = buf.reshape(4096, 32)[:min(envs, 4096)].astype(np.int64)[ok]
            subs.append(np.stack([full[:, 12] - full[:, 1], full[:, 2] - full[:, 12],
                                  full[:, 13] - full[:, 1], full[:, 15] - full[:, 3],
                                  full[:, 14] - full[:, 15], full[:, 4] - full[:, 14],
                                  full[:, 16] - full[:, 7], full[:, 17] - full[:, 16], full[:, 18] - full[:, 17],
                                  full[:, 19] - full[:, 18], full[:, 8] - full[:, 19],
                                  full[:, 20] - full[:, 0]], 1))
    d = np.concatenate(rows)
    tot = np.median(d.sum(1))
    print(f"{preset} envs={envs}: median total {tot:.0f} cycles over {len(d)} env-ticks")
    for i in range(11):
        med, p90 = np.median(d[:, i]), np.percentile(d[:, i], 90)
        print(f"  {PHASES[i+1]:22s} median {med:9.0f}  p90 {p90:9.0f}  ({100*med/tot:5.1f}%)")
    sub = np.concatenate(subs)
    print(f"  of which player decode  median {np.median(sub[:, 0]):9.0f} (visibility bitmap "
          f"{np.median(sub[:, 2]):9.0f}); npc decide median {np.median(sub[:, 1]):9.0f}")
    print(f"  update+harvest = resource {np.median(d[:, 2]):9.0f} + professions "
          f"{np.median(sub[:, 3]):9.0f}; item actions (Use..Destroy) {np.median(sub[:, 4]):9.0f}; "
          f"attack init {np.median(sub[:, 5]):9.0f}")
    print(f"  respawn = count {np.median(sub[:, 6]):9.0f} + prefix {np.median(sub[:, 7]):9.0f} + list "
          f"{np.median(sub[:, 8]):9.0f} + draws {np.median(sub[:, 9]):9.0f} + expiry/tick {np.median(sub[:, 10]):9.0f}; "
          f"groups n/a")
    print(f"  rowslot phase: state load {np.median(sub[:, 11]):9.0f}")
    tt = np.concatenate(totals)
    for name, sel in (("stepped", tt[:, 1] == 1), ("reset", tt[:, 1] == 0)):
        x = tt[sel, 0]
        if len(x):
            print(f"  {name:8s} env-ticks {len(x):6d}: total median {np.median(x):9.0f} p99 "
                  f"{np.percentile(x, 99):9.0f} max {x.max():9.0f}")


if __name__ == "__main__":
    main()
