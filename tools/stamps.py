"""Phase attribution of the tick kernel from in-kernel s_memtime stamps (diagnostic build).

Usage (GPU box): python tools/stamps.py [C2|C3|C4] [envs] [warmup]
Builds nothing on the box: run `python -c "from nmmo_amd import build; build.build(stamps=True)"`
here first (the .so travels with the snapshot). Prints median / p90 cycles per phase of the
stepped (not reset) env-ticks. Thread 0 stamps after each phase; a launch clears its stamps
first, so a phase its system set compiles out reads as absent (0 cycles), and phases without a
block barrier before their stamp (respawn sub-phases) time wave 0 only.
"""

import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
os.environ.setdefault("NMMO_LIB", os.path.join(ROOT, "nmmo_amd", "lib", "libnmmo_hip_stamps.so"))

import numpy as np  # noqa: E402
import torch  # noqa: E402

from nmmo_amd import _native, abi  # noqa: E402
from nmmo_amd.config import Config  # noqa: E402
from nmmo_amd.engine import NmmoEngine  # noqa: E402

# stamp ids in execution order (tick.hip NMMO_STAMP) and the phase that ENDS at each
STAMPS = [(0, None), (20, "state load"), (1, "prep: rowslot, positions, listings"),
          (13, "visibility bitmap"), (12, "action decode"), (2, "npc decide + hunt BFS"),
          (3, "update: resources, tile hash"), (15, "harvest: foilage, professions"),
          (21, "harvest events"), (22, "Use"), (28, "Buy: count"), (29, "Buy: order, eligibility"),
          (30, "Buy: rounds"), (23, "Buy: events, freed rows"), (24, "Give, GiveGold (serial)"),
          (14, "Destroy"), (4, "attack init"), (25, "attack rounds"), (26, "attack events"),
          (27, "parallel shots"), (5, "serial shots, loot"), (6, "move (+ Sell)"), (7, "cull, NPC compaction"),
          (16, "respawn scan (wave 0)"), (18, "respawn list (wave 0)"), (19, "respawn draws, expiry (wave 0)"),
          (8, "tick++ barrier"), (9, "npc spawn"), (10, "tasks, rewards, dones"), (11, "store")]


def phases(st: np.ndarray) -> np.ndarray:
    """st: [n, 32] raw stamps of stepped env-ticks -> [n, len(STAMPS)-1] cycles per phase
    (absent stamps take the previous present one's time: 0 cycles)."""
    ids = [k for k, _ in STAMPS]
    t = st[:, ids].astype(np.int64)
    for j in range(1, t.shape[1]):
        t[:, j] = np.where(t[:, j] == 0, t[:, j - 1], t[:, j])
    return np.diff(t, axis=1)


def main():
    preset = sys.argv[1] if len(sys.argv) > 1 else "C3"
    envs = int(sys.argv[2]) if len(sys.argv) > 2 else 1024
    warm = int(sys.argv[3]) if len(sys.argv) > 3 else 40
    cfg = Config.preset(preset, early_stop_agent_num=8,
                        obs_layout=abi.OBS_FLAT if preset == "C4" else abi.OBS_NONE)
    eng = NmmoEngine(cfg, envs, seed=1)
    cur = os.environ.get("STAMPS_CURRICULUM")  # e.g. manual / heldout: nmmo_amd.tasks' curricula
    if cur:
        from nmmo_amd import tasks

        eng.set_curriculum(getattr(tasks, cur + "_curriculum")())
    eng.reset()
    stagger = int(os.environ.get("STAMPS_STAGGER", "0"))  # bench.py's staggered pre-roll
    for k in range(stagger):
        eng.end_episodes(np.arange(envs) % stagger == k)
        eng.scripted_actions(1_000_003)
        eng.step(write_obs=False)
    L = _native.lib()
    L.nmmo_debug_read_stamps.argtypes = [ctypes.c_void_p, ctypes.c_int]
    rows, totals = [], []
    for t in range(warm + 10):
        eng.scripted_actions(1000 + t)
        eng.step(write_obs=False)
        torch.cuda.synchronize()
        if t >= warm:
            buf = np.zeros(4096 * 32, np.uint64)
            assert L.nmmo_debug_read_stamps(buf.ctypes.data_as(ctypes.c_void_p), buf.size) == 0
            st = buf.reshape(4096, 32)[:min(envs, 4096)].astype(np.int64)
            stepped = (st[:, 2] > 0) & (st[:, 11] > st[:, 0])  # the decode ran: not a reset
            rows.append(phases(st[stepped]))
            done = st[:, 11] > st[:, 0]
            totals.append(np.stack([st[done, 11] - st[done, 0], stepped[done].astype(np.int64)], 1))
    d = np.concatenate(rows)
    tot = np.median(d.sum(1))
    print(f"{preset} envs={envs}: median total {tot:.0f} cycles over {len(d)} stepped env-ticks")
    for i, (_, name) in enumerate(STAMPS[1:]):
        med, p90 = np.median(d[:, i]), np.percentile(d[:, i], 90)
        print(f"  {name:42s} median {med:9.0f}  p90 {p90:9.0f}  ({100 * med / tot:5.1f}%)")
    # the tail: a launch lasts as long as its slowest env, so what makes the slowest env-ticks
    # slow matters more than the median. Per phase: p99, and the mean over the slowest 5% of
    # env-ticks (by total) against the mean over all of them.
    tot_each = d.sum(1)
    slow = tot_each >= np.percentile(tot_each, 95)
    print(f"  tail: slowest 5% of stepped env-ticks ({int(slow.sum())}): total mean {tot_each[slow].mean():.0f} "
          f"vs {tot_each.mean():.0f} overall, p99 {np.percentile(tot_each, 99):.0f}, max {tot_each.max():.0f}")
    excess = d[slow].mean(0) - d.mean(0)
    for i in np.argsort(-excess)[:10]:
        print(f"    {STAMPS[i + 1][1]:42s} slow-5% mean {d[slow, i].mean():9.0f}  all mean {d[:, i].mean():9.0f}  "
              f"p99 {np.percentile(d[:, i], 99):9.0f}  excess {excess[i]:8.0f}")
    tt = np.concatenate(totals)
    for name, sel in (("stepped", tt[:, 1] == 1), ("reset", tt[:, 1] == 0)):
        x = tt[sel, 0]
        if len(x):
            print(f"  {name:8s} env-ticks {len(x):6d}: total median {np.median(x):9.0f} p99 "
                  f"{np.percentile(x, 99):9.0f} max {x.max():9.0f}")


if __name__ == "__main__":
    main()
