"""Diagnostic: market listings per env (rows of the flat obs' Market section) in the C4 bench
workload, after the staggered pre-roll: how often an env has more than the flat kernel's 256
staged listings (the rest are read from HBM inside the row loop)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)


def main():
    import torch

    import bench
    from nmmo_amd import abi
    from nmmo_amd.config import Config
    from nmmo_amd.engine import NmmoEngine

    dev = torch.device("cuda:0")
    cfg = Config.preset("C4", early_stop_agent_num=8, obs_layout=abi.OBS_FLAT)
    eng = NmmoEngine(cfg, 512, seed=1, device=dev, task_embedding=bench._task_embedding())
    eng.reset()
    bench._stagger([eng], 64, 512, 0, 1_000_003)
    lay = eng.layout
    off = lay.off_market
    for t in range(90):
        eng.scripted_actions(1_000_003)
        eng.step()
        if t % 30 == 29:
            o = eng.obs.view(512, eng.P, -1)
            m = o[:, :8, off:off + abi.MARKET_ROWS * 16].reshape(512, 8, abi.MARKET_ROWS, 16)
            nm = (m[..., 1] != 0).sum(2).max(1).values.float()
            q = torch.quantile(nm, torch.tensor([0.5, 0.9, 0.99, 1.0], device=dev))
            print(f"tick {t}: listings per env median {q[0]:.0f} p90 {q[1]:.0f} p99 {q[2]:.0f} max {q[3]:.0f}; "
                  f"envs over 256: {(nm > 256).float().mean().item():.3f}")
    eng.close()


if __name__ == "__main__":
    main()
