"""Device-resident evaluate/train loop around the HIP stepper and the HBM experience storage.

The reference trainer (`reinforcement_learning/clean_pufferl.py`) runs `evaluate(data)` — recv,
policy forward, copy the learner-mask rows into host storage, send (`:287-357`) — and then
`train(data)` — sort the (env_id, step) keys, the reversed GAE loop, flatten the batch and run
`update_epochs` of PPO minibatches (`:390-540`). `DeviceTrainer` keeps that control flow and
those names, but nothing leaves the GPU: recv is the engine's obs/reward/done/mask tensors in
HBM (`NmmoEngine`, the HIP tick + obs kernels), the stores, sort, advantages and minibatch
gathers are the `nmmo_exp_*` kernels (`DeviceExperience`, `csrc/storage.hip`), and send is
`nmmo_step` on the sampled actions. The PPO loss and optimizer step are the reference's
expressions (`:476-523`) on whatever agent the caller passes.

The policy networks themselves are out of scope (consumers of the path);
`MaskedLinearAgent` is a minimal stand-in with the reference policies' call convention —
`agent(obs, action=None) -> (action, logprob, entropy, value)` with every head's logits masked
by the obs ActionTargets (baseline_policy.py:245-262) — so the loop can be exercised and timed.
"""

from __future__ import annotations

import dataclasses
import math
import time

import numpy as np
import torch
from torch import nn

from . import layout
from .storage import DeviceExperience


@dataclasses.dataclass
class TrainConfig:
    """The `train:` section of the reference's config.yaml (names and defaults)."""

    seed: int = 1
    total_timesteps: int = 10_000_000
    learning_rate: float = 1.5e-4
    anneal_lr: bool = True
    gamma: float = 0.99
    gae_lambda: float = 0.95
    update_epochs: int = 3
    norm_adv: bool = True
    clip_coef: float = 0.1
    clip_vloss: bool = True
    ent_coef: float = 0.01
    vf_coef: float = 0.5
    max_grad_norm: float = 0.5
    target_kl: float | None = None
    batch_size: int = 32768
    batch_rows: int = 128
    bptt_horizon: int = 8
    vf_clip_coef: float = 0.1

    def validate(self):
        if self.batch_size % (self.bptt_horizon * self.batch_rows):
            raise ValueError("batch_size must be a multiple of bptt_horizon * batch_rows (clean_pufferl.py:412)")


class MaskedLinearAgent(nn.Module):
    """A small stand-in policy: the 15x15 Tile materials and the agent's own tick through one
    hidden layer, a linear head per action with illegal entries masked out by the obs's
    ActionTargets, and a value head."""

    def __init__(self, task_dim: int = 2048, hidden: int = 64):
        super().__init__()
        lay = layout.flat_layout(task_dim)
        self.o_tile = lay["Tile"].offset
        self.o_tick = lay["CurrentTick"].offset
        self.dims = list(layout.ACTION_DIMS)
        self.mask_off = np.cumsum([0] + self.dims).tolist()
        self.encoder = nn.Sequential(nn.Linear(layout.TILE_ROWS + 1, hidden), nn.ReLU())
        self.actor = nn.Linear(hidden, sum(self.dims))
        self.value = nn.Linear(hidden, 1)

    def forward(self, obs: torch.Tensor, action: torch.Tensor | None = None):
        mat = obs[:, self.o_tile + 2:self.o_tile + 3 * layout.TILE_ROWS:3] / 16.0
        tick = obs[:, self.o_tick:self.o_tick + 1] / 1024.0
        h = self.encoder(torch.cat([mat, tick], 1))
        logits = self.actor(h)
        masks = obs[:, :self.mask_off[-1]] > 0
        acts, logp, ent = [], 0.0, 0.0
        for k, n in enumerate(self.dims):
            lo, hi = self.mask_off[k], self.mask_off[k + 1]
            lg = logits[:, lo:hi].masked_fill(~masks[:, lo:hi], -1e9)
            dist = torch.distributions.Categorical(logits=lg)
            a = dist.sample() if action is None else action[:, k]
            acts.append(a)
            logp = logp + dist.log_prob(a)
            ent = ent + dist.entropy()
        return torch.stack(acts, 1), logp, ent, self.value(h)


class DeviceTrainer:
    """clean_pufferl's evaluate()/train() over one NmmoEngine (flat obs) and DeviceExperience."""

    def __init__(self, engine, agent: nn.Module, config: TrainConfig, env_id_base: int = 0):
        config.validate()
        self.engine = engine
        self.agent = agent
        self.config = config
        self.device = engine.device
        self.n_rows = engine.n_envs * engine.P
        self.env_id_base = int(env_id_base)
        self.experience = DeviceExperience(config.batch_size, engine.obs_elems, self.n_rows, device=self.device)
        self.optimizer = torch.optim.Adam(agent.parameters(), lr=config.learning_rate, eps=1e-5)
        self.total_updates = max(1, config.total_timesteps // config.batch_size)
        self.update = 0
        self.global_step = 0
        self.agent_step = 0
        self.last_batch = None
        self.stats = {}

    def evaluate(self, on_store=None) -> dict:
        """One batch of experience (clean_pufferl.py:287-357): recv -> forward -> store -> send
        until ptr == batch_size + 1. Returns the reference's SPS counters. `on_store(o, r, d,
        mask, actions, logprob, value, env_id, step)` (optional, for checkers) sees each store's
        inputs before the step overwrites them."""
        eng, exp = self.engine, self.experience
        exp.reset()
        N = self.n_rows
        agent_steps = torch.zeros((), dtype=torch.int64, device=self.device)
        padded = step = 0
        torch.cuda.synchronize(self.device)
        t0 = time.perf_counter()
        while not exp.full():
            step += 1
            o = eng.obs.view(N, eng.obs_elems)
            r, d, mask = eng.rew.view(N), eng.term.view(N), eng.mask.view(N)
            with torch.no_grad():
                actions, logprob, _, value = self.agent(o)
            agent_steps += mask.sum()
            padded += N
            exp.store(o, r, d, mask, actions, logprob, value.flatten(), step, env_id_base=self.env_id_base)
            if on_store is not None:
                on_store(o, r, d, mask, actions, logprob, value.flatten(),
                         self.env_id_base + torch.arange(N, device=self.device), step)
            eng.step(actions.to(torch.int32).view(eng.n_envs, eng.P, -1))
        torch.cuda.synchronize(self.device)
        elapsed = time.perf_counter() - t0
        eng.check_fault("DeviceTrainer.evaluate")  # the batch boundary: no faulted tick reaches train()
        agent_steps = int(agent_steps.item())
        self.agent_step += agent_steps
        self.global_step += padded
        self.stats = {"SPS": int(padded / elapsed), "agent_SPS": int(agent_steps / elapsed),
                      "agent_steps": agent_steps, "padded_steps": padded, "eval_time": elapsed,
                      "reward": float(exp.rewards[:exp.batch_size].mean())}
        return self.stats

    def train(self) -> dict:
        """One update (clean_pufferl.py:390-540): sort, GAE, flatten, PPO epochs."""
        cfg, exp, agent = self.config, self.experience, self.agent
        if cfg.anneal_lr:
            # clean_pufferl.py:409 with data.update counted from 0 and incremented after train()
            # (:140, :557): the first update's frac is 1 + 1/total_updates, as in the reference
            frac = 1.0 - (self.update - 1.0) / self.total_updates
            self.optimizer.param_groups[0]["lr"] = frac * cfg.learning_rate
        t0 = time.perf_counter()
        idxs = exp.sort()
        advantages = exp.advantages(idxs, cfg.gamma, cfg.gae_lambda)
        b = exp.batch(idxs, advantages, cfg.batch_rows, cfg.bptt_horizon)
        self.last_batch = (idxs, advantages, b)
        b_returns, b_values, b_adv = b["b_returns"], b["b_values"], b["b_advantages"]
        pg_losses, entropy_losses, v_losses, clipfracs, old_kls, kls = [], [], [], [], [], []
        approx_kl = None
        for _ in range(cfg.update_epochs):
            for mb in range(b["num_minibatches"]):
                m = exp.minibatch(b["b_idxs"], mb)
                mb_obs = m["obs"].reshape(-1, exp.obs_elems)
                mb_actions = m["actions"].reshape(-1, m["actions"].shape[-1])
                mb_values = b_values[mb].reshape(-1)
                mb_advantages = b_adv[mb].reshape(-1)
                mb_returns = b_returns[mb].reshape(-1)
                _, newlogprob, entropy, newvalue = agent(mb_obs, action=mb_actions)
                logratio = newlogprob - m["logprobs"].reshape(-1)
                ratio = logratio.exp()
                with torch.no_grad():
                    old_kls.append((-logratio).mean())
                    approx_kl = ((ratio - 1) - logratio).mean()
                    kls.append(approx_kl)
                    clipfracs.append(((ratio - 1.0).abs() > cfg.clip_coef).float().mean())
                if cfg.norm_adv:
                    mb_advantages = (mb_advantages - mb_advantages.mean()) / (mb_advantages.std() + 1e-8)
                pg_loss1 = -mb_advantages * ratio
                pg_loss2 = -mb_advantages * torch.clamp(ratio, 1 - cfg.clip_coef, 1 + cfg.clip_coef)
                pg_loss = torch.max(pg_loss1, pg_loss2).mean()
                newvalue = newvalue.view(-1)
                if cfg.clip_vloss:
                    v_loss_unclipped = (newvalue - mb_returns) ** 2
                    v_clipped = mb_values + torch.clamp(newvalue - mb_values, -cfg.vf_clip_coef, cfg.vf_clip_coef)
                    v_loss_clipped = (v_clipped - mb_returns) ** 2
                    v_loss = 0.5 * torch.max(v_loss_unclipped, v_loss_clipped).mean()
                else:
                    v_loss = 0.5 * ((newvalue - mb_returns) ** 2).mean()
                entropy_loss = entropy.mean()
                loss = pg_loss - cfg.ent_coef * entropy_loss + v_loss * cfg.vf_coef
                self.optimizer.zero_grad()
                loss.backward()
                nn.utils.clip_grad_norm_(agent.parameters(), cfg.max_grad_norm)
                self.optimizer.step()
                pg_losses.append(pg_loss.detach())
                v_losses.append(v_loss.detach())
                entropy_losses.append(entropy_loss.detach())
            if cfg.target_kl is not None and approx_kl is not None and approx_kl > cfg.target_kl:
                break
        y_pred, y_true = b_values.reshape(-1), b_returns.reshape(-1)
        var_y = torch.var(y_true, unbiased=False)
        explained_var = float("nan") if float(var_y) == 0 else float(1 - torch.var(y_true - y_pred, unbiased=False) / var_y)
        mean = lambda xs: float(torch.stack(xs).mean()) if xs else math.nan  # noqa: E731
        losses = {"policy_loss": mean(pg_losses), "value_loss": mean(v_losses), "entropy": mean(entropy_losses),
                  "old_approx_kl": mean(old_kls), "approx_kl": mean(kls), "clipfrac": mean(clipfracs),
                  "explained_variance": explained_var}
        torch.cuda.synchronize(self.device)
        self.update += 1
        losses["train_time"] = time.perf_counter() - t0
        losses["train_sps"] = int(cfg.batch_size / losses["train_time"])
        return losses
