"""CPU restatement of the reference trainer's rollout storage — TEST INFRASTRUCTURE ONLY.

Checker for nmmo_amd/storage.py (the HIP experience storage). It keeps
the reference's own data structures and arithmetic: host float32 tensors of batch_size + 1 rows
(reinforcement_learning/clean_pufferl.py:182-188), the learner-mask row selection cut at the room
left (:331-336), a Python list of (env_id, step) sort keys sorted with `sorted` (:345, :414),
the reversed advantage loop on 0-dim float32 CPU tensors one op at a time (:424-436), and fancy
indexing for the batch (:417-421, :439-446). Parity is pinned by construction to the
reference's torch CPU semantics: the same expressions on the same dtypes (pufferlib, which the
reference's evaluate loop also needs, is absent, so the loop itself cannot be imported).
Never imported by the product path.
"""

from __future__ import annotations

import numpy as np
import torch


class ReferenceStorage:
    def __init__(self, batch_size: int, obs_elems: int):
        self.batch_size = batch_size
        cap = batch_size + 1
        self.obs = torch.zeros(cap, obs_elems)                       # :182
        self.actions = torch.zeros(cap, 12, dtype=int)               # :183
        self.logprobs = torch.zeros(cap)
        self.rewards = torch.zeros(cap)
        self.dones = torch.zeros(cap)
        self.truncateds = torch.zeros(cap)
        self.values = torch.zeros(cap)
        self.sort_keys = []
        self.ptr = 0

    def store(self, o, r, d, mask, actions, logprob, value, env_id, step):
        """One evaluate iteration's stores (:327-346); every argument host numpy [N, ...]."""
        learner_mask = torch.Tensor(np.asarray(mask, dtype=np.float32))
        indices = torch.where(learner_mask)[0][: self.batch_size - self.ptr + 1].numpy()
        end = self.ptr + len(indices)
        self.obs.numpy()[self.ptr:end] = np.asarray(o, dtype=np.float32)[indices]
        self.values.numpy()[self.ptr:end] = np.asarray(value, dtype=np.float32)[indices]
        self.actions.numpy()[self.ptr:end] = np.asarray(actions)[indices]
        self.logprobs.numpy()[self.ptr:end] = np.asarray(logprob, dtype=np.float32)[indices]
        self.rewards.numpy()[self.ptr:end] = torch.as_tensor(r).float().view(-1).numpy()[indices]
        self.dones.numpy()[self.ptr:end] = torch.as_tensor(d).float().view(-1).numpy()[indices]
        self.sort_keys.extend([(int(env_id[i]), step) for i in indices])
        self.ptr += len(indices)
        return len(indices)

    def sort(self):
        idxs = sorted(range(len(self.sort_keys)), key=self.sort_keys.__getitem__)  # :414
        self.sort_keys = []
        return idxs

    def advantages(self, idxs, gamma: float, gae_lambda: float):
        """The reversed loop of :424-436 verbatim in semantics (0-dim float32 CPU tensors)."""
        advantages = torch.zeros(self.batch_size)
        lastgaelam = 0
        for t in reversed(range(self.batch_size)):
            i, i_nxt = idxs[t], idxs[t + 1]
            nextnonterminal = 1.0 - self.dones[i_nxt]
            nextvalues = self.values[i_nxt]
            delta = self.rewards[i_nxt] + gamma * nextvalues * nextnonterminal - self.values[i]
            advantages[t] = lastgaelam = delta + gamma * gae_lambda * nextnonterminal * lastgaelam
        return advantages

    def batch(self, idxs, advantages, batch_rows: int, bptt_horizon: int):
        num_mb = self.batch_size // bptt_horizon // batch_rows
        b_idxs = torch.Tensor(idxs).long()[:-1].reshape(batch_rows, num_mb, bptt_horizon).transpose(0, 1)
        b_values = torch.Tensor(self.values.numpy()[b_idxs])
        b_adv = advantages.reshape(batch_rows, num_mb, bptt_horizon).transpose(0, 1)
        return {"b_idxs": b_idxs, "b_values": b_values, "b_advantages": b_adv, "b_returns": b_adv + b_values,
                "b_obs": self.obs.numpy()[b_idxs], "b_actions": self.actions.numpy()[b_idxs],
                "b_logprobs": self.logprobs.numpy()[b_idxs], "b_dones": self.dones.numpy()[b_idxs],
                "num_minibatches": num_mb}
