"""One rank of the 2-rank C5 content check (tests/test_gpu_multirank.py), launched under
torch.distributed.run with gloo, both ranks on cuda:0.

Each rank steps its env batches through WireGather (wire obs, learner gather one step behind);
rank 0 decodes every gathered buffer (its own in place, the peer's received) into the native
layout and stores the learner-mask rows of every step into a DeviceExperience straight from the
wire records, then writes per step and global env the sha256 of the native obs and of the
reward / term / trunc / mask bytes, plus digests of the experience buffers, to argv[1] (JSON).
The test compares them with one engine stepping all envs alone. argv[2] = "eager" (per-step
episode ends on each batch's stream, graphs=False) or "graphs" (the bench's mode: each (batch,
ring slot) replayed from its hipGraph, the 3-slot ring reused across steps with cross-stream done
events; episode phases staggered by the pre-roll only and ended by a short horizon). argv[3] =
"even" (N_PER_BATCH envs per batch on both ranks) or "uneven" (the learner's smaller share,
bench.py --root-envs: SPLIT envs per batch by rank). argv[4] = "store" also gives rank 0 the
gather's own compact record store (WireGather store=: the fused checked store, peers received
straight into their arena slots) and records each step's stored rows; "store-noplan" the same
with the arena receive off (peers received into the exchange's buffers and copied). Not
collected by pytest."""

import hashlib
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

# shared with the test's one-engine reference run
N_PER_BATCH, BATCHES, SEED, PSEED, PREROLL, TICKS, MAP_N = 3, 2, 11, 77, 36, 18, 8
SPLIT = {"even": (N_PER_BATCH, N_PER_BATCH), "uneven": (1, 5)}  # envs per batch on rank 0, rank 1


def horizon(mode):
    """graphs mode has no per-step episode ends: a horizon inside the checked window ends them"""
    return 40 if mode == "graphs" else 1024


def end_mask(ids, t):
    """Envs (global ids) whose episode the pool ends before checked step t (staggered resets)."""
    return (ids * 7 + t) % 11 == 0


def preroll_mask(ids, k):
    return ids % 12 == k if k < 12 else ids < 0


def digest(t):
    return hashlib.sha256(t.contiguous().cpu().numpy().tobytes()).hexdigest()[:24]


def main():
    import numpy as np
    import torch
    import torch.distributed as dist

    from nmmo_amd import abi, wire
    from nmmo_amd.config import Config
    from nmmo_amd.distributed import WireGather
    from nmmo_amd.engine import NmmoEngine
    from nmmo_amd.storage import DeviceExperience

    out_path = sys.argv[1]
    mode = sys.argv[2] if len(sys.argv) > 2 else "eager"
    split = sys.argv[3] if len(sys.argv) > 3 else "even"
    store_mode = sys.argv[4] if len(sys.argv) > 4 else ""
    rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    torch.cuda.set_device(0)
    dev = torch.device("cuda", 0)
    dist.init_process_group("gloo")
    nb = BATCHES
    per_rank = SPLIT[split]
    n = per_rank[rank]
    envs = n * nb
    base0 = sum(p * nb for p in per_rank[:rank])  # this rank's first global env
    total = sum(p * nb for p in per_rank)
    cfg = Config.preset("C4", MAP_N=MAP_N, early_stop_agent_num=8, obs_layout=abi.OBS_WIRE, HORIZON=horizon(mode))
    engs = [NmmoEngine(cfg, n, seed=SEED, device=dev, env_index_base=base0 + j * n) for j in range(nb)]
    P = engs[0].P
    for e in engs:
        e.reset()
    for k in range(PREROLL):
        for j, e in enumerate(engs):
            e.end_episodes(preroll_mask(np.arange(n) + base0 + j * n, k))
            e.scripted_actions(PSEED)
            e.step(write_obs=False)
    torch.cuda.synchronize()

    def before(t, j, e):
        e.end_episodes(end_mask(np.arange(n) + base0 + j * n, t))

    rec = {"native": {}, "small": {}, "stored": {}}
    x = DeviceExperience(TICKS * total * P, engs[0].obs_elems, total * P, device=dev) if rank == 0 else None
    gs = None
    if store_mode and rank == 0:  # the gather's own record store: every row of every step, reset per step
        from nmmo_amd import wire as nw

        gs = DeviceExperience(total * P, engs[0].obs_elems, total * P, device=dev,
                              record_arena_bytes=sum(nw.max_bytes(p, P) + 64 for p in per_rank for _ in range(nb)))

    def on_step(s, got):
        for (r, j) in sorted(got):
            w, sm = got[r, j]
            m = g.counts[r][j]
            z = torch.zeros(m * P, device=dev)
            nat = wire.unpack(w, m, P)
            sm3 = sm.view(m, P, 8)
            base = g.env_base[r, j]
            for i in range(m):
                rec["native"][f"{s}:{base + i}"] = digest(nat[i])
                rec["small"][f"{s}:{base + i}"] = digest(sm3[i, :, :7])
            rew = sm3[..., 0:4].contiguous().view(torch.float32).view(-1)
            x.store(w, rew, sm3[..., 4].reshape(-1), sm3[..., 6].reshape(-1), torch.zeros((m * P, 12), dtype=torch.int32),
                    z, z, step=s + 1, env_id_base=base * P, engine=engs[0])
        if gs is not None:  # the step's rows as the gather stored them (global env order)
            k = gs.ptr
            idx = torch.arange(k, dtype=torch.int32, device=dev)
            rec["stored"][str(s)] = {"ptr": k, "obs": digest(gs.gather_obs(idx)), "rewards": digest(gs.rewards[:k]),
                                     "dones": digest(gs.dones[:k]), "env_id": digest(gs.env_id[:k])}

    graphs = mode == "graphs"
    g = WireGather(engs, PSEED, rank, world, graphs=graphs, on_step=on_step if rank == 0 else None,
                   before_step=None if graphs else before, backend="gloo", store=gs)
    if store_mode == "store-noplan" and rank == 0:
        g._arena_plan = lambda s: None  # received into the exchange's buffers, then copied by the store
    for _ in range(TICKS):
        g.step()
    g.drain()
    torch.cuda.synchronize()
    status = g.check_status()
    g.close()
    if rank == 0:
        k = x.ptr
        rec["status"] = status
        rec["exp"] = {"ptr": k, "obs": digest(x.obs[:k]), "rewards": digest(x.rewards[:k]),
                      "dones": digest(x.dones[:k]), "env_id": digest(x.env_id[:k]), "step": digest(x.step[:k])}
        rec["payload_bytes"] = g.x.payload_bytes
        rec["store_status"] = gs.status if gs is not None else 0
        with open(out_path, "w") as f:
            json.dump(rec, f)
    dist.barrier()
    for e in engs:
        e.close()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
