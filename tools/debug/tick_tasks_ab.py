"""Diagnostic: C4 tick time under a task curriculum (default the manual curriculum, whose
CanSeeTile / CanSeeAgent / skill tasks the bench's single TickGE task never evaluates): one
512-env batch, staggered, HIP events around each tick (nmmo_set_timing). Prints ms per tick.

  NMMO_LIB=<lib> NMMO_ALLOW_STALE=1 python tools/debug/tick_tasks_ab.py [manual|heldout|cansee]
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)


def main():
    import torch

    import bench
    from nmmo_amd import abi, tasks
    from nmmo_amd.config import Config
    from nmmo_amd.engine import NmmoEngine

    which = sys.argv[1] if len(sys.argv) > 1 else "manual"
    specs = {"manual": tasks.manual_curriculum, "heldout": tasks.heldout_curriculum}.get(which)
    specs = specs() if specs else [tasks.TaskSpec("CanSeeTile", {"tile_type": m}) for m in tasks.HARVESTABLE]
    dev = torch.device("cuda:0")
    cfg = Config.preset("C4", early_stop_agent_num=8, obs_layout=abi.OBS_FLAT)
    eng = NmmoEngine(cfg, 512, seed=1, device=dev)
    eng.set_curriculum(specs)
    eng.reset()
    pseed = 1_000_003
    bench._stagger([eng], 64, 512, 0, pseed)
    for _ in range(20):
        eng.scripted_actions(pseed)
        eng.step(write_obs=False)
    torch.cuda.synchronize()
    eng.set_timing(True)
    for _ in range(60):
        eng.scripted_actions(pseed)
        eng.step(write_obs=False)
    torch.cuda.synchronize()
    tick_ms, _, n, _ = eng.read_timing()
    print(f"{which}: {len(specs)} task specs, tick {tick_ms / max(n, 1) * 1e3:.1f} us per 512-env launch over {n} ticks")
    eng.check_fault("tick_tasks_ab")
    eng.close()


if __name__ == "__main__":
    main()
