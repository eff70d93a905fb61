"""End-to-end rate of the device evaluate/train loop (nmmo_amd/trainer.py) on one GPU: the
reference trainer's agent_SPS (clean_pufferl.py:364-376) with the HIP stepper, HBM storage and the
small stand-in policy, plus the train side (sort, GAE, PPO epochs) per update.

Usage (GPU box): python tools/bench_trainer.py [envs] [batch_size] [updates]
"""

import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

from nmmo_amd.config import Config  # noqa: E402
from nmmo_amd.engine import NmmoEngine  # noqa: E402
from nmmo_amd.trainer import DeviceTrainer, MaskedLinearAgent, TrainConfig  # noqa: E402


def main():
    envs = int(sys.argv[1]) if len(sys.argv) > 1 else 64
    batch = int(sys.argv[2]) if len(sys.argv) > 2 else 32768
    updates = int(sys.argv[3]) if len(sys.argv) > 3 else 3
    torch.manual_seed(1)
    cfg = Config.preset("C4", early_stop_agent_num=8)
    eng = NmmoEngine(cfg, envs, seed=1)
    eng.reset()
    agent = MaskedLinearAgent(cfg.TASK_EMBED_DIM).cuda()
    tc = TrainConfig(batch_size=batch, total_timesteps=batch * (updates + 1))
    tr = DeviceTrainer(eng, agent, tc)
    tr.evaluate()  # warm-up (allocator, kernels)
    tr.train()
    ev, trn = [], []
    for _ in range(updates):
        ev.append(tr.evaluate())
        trn.append(tr.train())
    out = {
        "workload": f"C4 {envs} envs x 128 agents, flat obs, batch_size {batch}, MaskedLinearAgent",
        "agent_SPS": round(sum(e["agent_SPS"] for e in ev) / len(ev)),
        "SPS": round(sum(e["SPS"] for e in ev) / len(ev)),
        "eval_time_s": round(sum(e["eval_time"] for e in ev) / len(ev), 4),
        "train_time_s": round(sum(t["train_time"] for t in trn) / len(trn), 4),
        "train_sps": round(sum(t["train_sps"] for t in trn) / len(trn)),
        "losses": {k: trn[-1][k] for k in ("policy_loss", "value_loss", "entropy", "approx_kl")},
    }
    print(json.dumps(out))
    eng.close()


if __name__ == "__main__":
    main()
