"""Line-granular read model of the tick kernel's material-map accesses (CPU; oracle-driven).

The tick reads each in-realm slot's tile neighbourhood from the env's mutable 160x160 material
map (tick.hip `tick_env`: the two dwords of row r holding columns c-1..c+1 and the dwords of rows
r-1 / r+1 holding column c; slots not in the realm read the map centre). Those are 4-16 byte
loads, but HBM is read in 128-B lines (on MI355X 90+% of the tick's TCC_EA0 read requests are
128-B requests, profiles/r02/tick_reqs.json), so the bytes that reach HBM are the distinct
lines touched per env, not the bytes used. This replays the bench's C2/C3 scenario on the oracle
(staggered episode phases, masked-uniform scripted actions) and counts them.

  python tools/tick_lines.py [C2|C3|C4] [envs] [stagger] [ticks] [--bank]

(--bank: count the bank lines without professions too, as the tick read them before round 2
skipped that read.)
"""

import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from nmmo_amd import abi  # noqa: E402
from nmmo_amd.config import Config  # noqa: E402
from oracle.oracle import OracleEnvs, split_state  # noqa: E402

LINE = 128
K = abi.MAP_SIZE


def lines_touched(ent, slots):
    """Distinct 128-B lines of one env's material map read by the neighbourhood loads."""
    alive = ent[abi.F["alive"], :slots] != 0
    r = np.where(alive, ent[abi.F["row"], :slots], K // 2).astype(np.int64)
    c = np.where(alive, ent[abi.F["col"], :slots], K // 2).astype(np.int64)
    mcw = (c - 1) >> 2
    offs = np.concatenate([r * K + 4 * mcw, r * K + 4 * (mcw + 1),
                           (r - 1) * K + 4 * (c >> 2), (r + 1) * K + 4 * (c >> 2)])
    return np.unique(offs // LINE).size


def main():
    preset = sys.argv[1] if len(sys.argv) > 1 else "C2"
    envs = int(sys.argv[2]) if len(sys.argv) > 2 else 32
    stagger = int(sys.argv[3]) if len(sys.argv) > 3 else 64
    ticks = int(sys.argv[4]) if len(sys.argv) > 4 else 20
    cfg = Config.preset(preset, early_stop_agent_num=8, obs_layout=abi.OBS_NONE)
    o = OracleEnvs(cfg, envs, seed=1)
    o.reset()
    for k in range(stagger):  # bench.py's staggered pre-roll
        o.end_episodes(np.arange(envs) % stagger == k)
        o.step(o.scripted_actions(1_000_003))
    slots = o.S
    bank = o.map_bank().reshape(-1, K * K)
    n, nb = [], []
    for t in range(ticks):
        st = split_state(o.get_state(), envs, slots)
        n += [lines_touched(st["ent"][e], slots) for e in range(envs)]
        # respawn: one bank dword per 4-tile group holding a depleted tile (mat != bank); without
        # professions the tick no longer reads the bank (every depletion is eaten Foilage)
        for e in range(envs if "Profession" in cfg.systems or "--bank" in sys.argv else 0):
            dep = np.flatnonzero(st["mat"][e].reshape(-1) != bank[st["env"][e, abi.E["map_id"]]])
            nb.append(np.unique(dep // LINE).size)
        o.step(o.scripted_actions(1000 + t))
    n, nb = np.asarray(n), np.asarray(nb if nb else [0])
    print(f"{preset}: {envs} envs x {ticks} ticks, per env-tick: material-map lines read by the "
          f"neighbourhood loads mean {n.mean():.1f} ({n.mean() * LINE / 1024:.1f} KiB of the "
          f"{K * K / 1024:.1f} KiB map; min {n.min()} max {n.max()}); map-bank lines read by the "
          f"respawn draws mean {nb.mean():.1f} ({nb.mean() * LINE / 1024:.1f} KiB); "
          f"total {(n.mean() + nb.mean()) * LINE / 1024:.1f} KiB")


if __name__ == "__main__":
    main()
