#!/usr/bin/env python3
"""bench.py — agent-steps/sec of the MI355X Neural MMO stepper (BASELINE.json metric).

One "step" = one tick of every env on this GPU: the scripted masked-uniform policy kernel
(SPEC.md §10, the synthetic action input) + nmmo_step (tick kernel [+ obs kernel]).
Inputs/state are resident in HBM before the timed region. Envs shard across ranks with no
data-path collective (weak scaling: envs per GPU fixed); each rank times K steps between a
barrier + device sync, rank 0 reports the max over ranks.

  python bench.py [--gpus N] [--steps K] [--warmup W] [--config C2|C3|C4] [--envs E]
  torchrun --nproc-per-node N bench.py --gpus N ...

value = alive agent-steps/s over the whole job (the reference's agent_SPS = sum(mask)/time,
reinforcement_learning/clean_pufferl.py:306,365); slot-steps/s (envs x 128 x ticks / s, the
padded count, :307,364) is reported beside it. cpu_baseline = the CPU oracle (a port of the
same semantics, not nmmo 2.1, which is absent) on the host's cores, rank 0 at N=1 only.
"""

from __future__ import annotations

import argparse
import json
import os
import sys
import threading
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "agent-steps/sec (whole node), 128-agent envs at 1/2/4/8 MI355X"
HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec

WORKLOADS = {
    # BASELINE.json configs[1..3]; early stop 8 = config.yaml reward_wrapper.early_stop_agent_num
    "C2": dict(envs=256, preset="C2", obs=False,
               desc="C2: 256 envs x 128 agents, movement + food/water (Resource)"),
    "C3": dict(envs=1024, preset="C3", obs=False,
               desc="C3: 1024 envs x 128 agents, + melee/range/mage combat, NPC spawn/AI, progression"),
    "C4": dict(envs=1024, preset="C4", obs=True,
               desc="C4: 1024 envs x 128 agents, all systems + per-agent flat obs gather"),
    # BASELINE.json configs[4]: C4 per GPU (8192 envs on 8) + the learner gather every step
    "C5": dict(envs=1024, preset="C4", obs=True, gather=True, layout="native",
               desc="C5: 1024 envs x 128 agents per GPU, all systems + obs, RCCL gather of "
                    "obs/reward/dones/mask to the learner (rank 0) every step"),
}


# the agent sections' reward_wrapper weights (config.yaml:103-106, 118-126, 137-140)
WRAPPER_KW = {"neurips23_start_kit": dict(heal_bonus_weight=0.03, explore_bonus_weight=0.01),
              "takeru": dict(explore_bonus_weight=0.01, disable_give=True),
              "yaofeng": dict(hp_bonus_weight=0.03, exp_bonus_weight=0.002, defense_bonus_weight=0.04,
                              attack_bonus_weight=0.0, gold_bonus_weight=0.001, custom_bonus_scale=0.1,
                              disable_give=True, donot_attack_dangerous_npc=True)}


def tick_bytes_per_env(S: int, P: int, items: bool) -> int:
    """Algorithmic HBM bytes of one tick of one env: the env state read and
    written once (45 int16 entity fields x slots, free-row ring, depleted-tile bitmap, env
    scalars; with the Item system the 12-slot inventories and the item-row ring), the actions
    read, the outputs written and the map tiles a player touches (own tile + 4 neighbours for
    harvest/drink, 1 move target)."""
    state = 45 * S * 2 + S * 2 + 800 * 4 + 16 * 4
    if items:
        state += P * 12 * 8 + 12 * P * 2
    return 2 * state + P * 12 * 4 + P * (4 + 1 + 1 + 1) + P * 6


def pmc_traffic(cfg_name: str, kernel: str, envs: int):
    """HBM bytes per launch of `kernel` from the committed rocprofv3 PMC summary of the same
    bench command (profiles/<round>/<cfg>/pmc.json, tools/pmc_summary.py): 2 x FETCH_SIZE +
    WRITE_SIZE, gfx950-corrected. None when no summary matches this workload."""
    import glob

    for path in sorted(glob.glob(os.path.join(ROOT, "profiles", "r*", cfg_name, "pmc.json")), reverse=True):
        try:
            d = json.load(open(path))
            k = d["kernels"][kernel]
            if d.get("bench", {}).get("config", {}).get("envs_per_gpu") != envs:
                continue
            return k["hbm_bytes_per_dispatch"], os.path.relpath(path, ROOT)
        except (KeyError, ValueError, OSError):
            continue
    return None, None


def obs_bytes_per_env(S: int, P: int, elems: int, native: bool = False) -> int:
    """Obs rows written (flat fp32: 23,987 x 4 B per agent; native, SPEC §8b: 9,552 B per agent
    + the env's 32 KB Market once) + the entity columns staged once per 16-agent workgroup +
    the 15x15 tile window read per agent."""
    from nmmo_amd import abi

    rows = abi.native_env_bytes(P) if native else P * elems * 4
    return rows + (P // 16) * (33 * S * 2) + P * 225


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=300)
    ap.add_argument("--warmup", type=int, default=50)
    ap.add_argument("--config", default="C2", choices=sorted(WORKLOADS))
    ap.add_argument("--envs", type=int, default=None, help="envs per GPU (default: config's)")
    ap.add_argument("--seed", type=int, default=1)
    ap.add_argument("--cpu-seconds", type=float, default=12.0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-graph", action="store_true", help="eager launches instead of hipGraph replay")
    ap.add_argument("--graph-steps", type=int, default=10, help="ticks captured per hipGraph")
    ap.add_argument("--obs", default=None, choices=["flat", "native"],
                    help="obs layout for the obs configs (default: flat for C4 = the pufferlib row "
                         "the reference's learner reads, native for C5 = SURVEY §8e's gather layout)")
    ap.add_argument("--wrapper", default="none",
                    choices=["none", "base", "neurips23_start_kit", "takeru", "yaofeng"],
                    help="run env_creator's RewardWrapper on the device (SPEC §13) with the "
                         "config.yaml weights")
    return ap.parse_args()


def cpu_baseline(cfg, seconds: float):
    """The CPU oracle (oracle/, a port of SPEC.md) on the host cores: one Python thread per core,
    each stepping its own env range through ctypes (the GIL is released inside the C calls)."""
    import numpy as np

    from oracle.oracle import OracleEnvs

    try:
        cores = len(os.sched_getaffinity(0))
    except AttributeError:
        cores = os.cpu_count() or 1
    threads = max(1, min(cores, 16))
    per = 4
    n = threads * per
    o = OracleEnvs(cfg, n, seed=7)
    o.reset()
    acts = np.zeros((n, cfg.PLAYER_N, 12), np.int32)
    from oracle.oracle import lib as olib

    def worker(k, counter, stop_at):
        lo, hi = k * per, (k + 1) * per
        t = 0
        while time.perf_counter() < stop_at:
            olib().oracle_scripted_actions_range(o.h, lo, hi, 1000 + t, acts.ctypes.data)
            o.step_range(lo, hi, acts)
            counter[k] += int(o.mask[lo:hi].sum())
            t += 1

    counter = [0] * threads
    stop_at = time.perf_counter() + 1.0  # warmup
    ths = [threading.Thread(target=worker, args=(k, [0] * threads, stop_at)) for k in range(threads)]
    [t.start() for t in ths]
    [t.join() for t in ths]
    t0 = time.perf_counter()
    stop_at = t0 + seconds
    ths = [threading.Thread(target=worker, args=(k, counter, stop_at)) for k in range(threads)]
    [t.start() for t in ths]
    [t.join() for t in ths]
    dt = time.perf_counter() - t0
    return {
        "value": round(sum(counter) / dt, 1),
        "unit": "agent-steps/s",
        "cores": threads,
        "kind": "port",
        "sample": f"CPU oracle (SPEC.md port, not nmmo 2.1) on {threads} host threads x {per} envs "
                  f"= {n} envs x {cfg.PLAYER_N} agents, same systems/obs as the GPU workload, "
                  f"{dt:.1f} s wall incl. the scripted policy",
    }


def main():
    args = parse()
    # The JSON line is the only thing on stdout: native libraries (RCCL prints a version banner
    # on stdout when a communicator is created) are sent to stderr by pointing fd 1 at fd 2.
    json_out = os.fdopen(os.dup(1), "w")
    sys.stdout.flush()
    os.dup2(2, 1)
    import torch
    import torch.distributed as dist

    from nmmo_amd import abi
    from nmmo_amd.config import Config
    from nmmo_amd.engine import NmmoEngine

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    else:
        torch.cuda.set_device(0)
    dev = torch.device("cuda", torch.cuda.current_device())

    wl = WORKLOADS[args.config]
    envs = args.envs or wl["envs"]
    native = wl["obs"] and (args.obs or wl.get("layout", "flat")) == "native"
    obs_layout = (abi.OBS_NATIVE if native else abi.OBS_FLAT) if wl["obs"] else abi.OBS_NONE
    cfg = Config.preset(wl["preset"], early_stop_agent_num=8, obs_layout=obs_layout)
    import numpy as np

    task = None
    gpath = os.path.join(ROOT, "tests", "golden", "task_embeddings.npz")
    if os.path.exists(gpath):
        task = np.load(gpath)["heldout_emb"][0]  # TickGE(1024) task, SURVEY §8d
    eng = NmmoEngine(cfg, envs, seed=args.seed, device=dev, task_embedding=task,
                     env_index_base=rank * envs)
    if args.wrapper != "none":
        from nmmo_amd.wrappers import wrapper_config

        eng.set_wrapper(wrapper_config(args.wrapper, **WRAPPER_KW.get(args.wrapper, {})))
    eng.reset()
    # device counters the tick kernel adds into: [0] = sum(mask) (agent-steps), [1] = episodes
    counters = torch.zeros(2, dtype=torch.int64, device=dev)
    eng.set_counters(counters)
    pseed = args.seed * 1_000_003  # the policy's Philox counter already walks (tick, episode)

    gather = wl.get("gather", False)
    if gather:
        # learner-side receive buffers on rank 0 (one gather per tick over xGMI);
        # the four small outputs travel packed in one buffer with the obs in another
        small = torch.empty((envs, cfg.PLAYER_N, 8), dtype=torch.uint8, device=dev)
        recv_obs = [torch.empty_like(eng.obs) for _ in range(world)] if rank == 0 else None
        recv_small = [torch.empty_like(small) for _ in range(world)] if rank == 0 else None
        if world == 1:  # a one-rank RCCL group: the gather degenerates to the root's own copy
            dist.init_process_group("nccl", init_method="tcp://127.0.0.1:29533", rank=0, world_size=1,
                                    device_id=dev)

    def one():
        eng.scripted_actions(pseed)
        eng.step()
        if gather:
            small[..., 0:4] = eng.rew.view(torch.uint8).view(envs, cfg.PLAYER_N, 4)
            small[..., 4] = eng.term
            small[..., 5] = eng.trunc
            small[..., 6] = eng.mask
            dist.gather(eng.obs, recv_obs, dst=0)
            dist.gather(small, recv_small, dst=0)

    for _ in range(args.warmup):
        one()
    torch.cuda.synchronize(dev)
    graphs = []
    if not args.no_graph and not gather:  # the step is capture-safe: no sync / alloc inside nmmo_step
        g_n = max(1, min(args.graph_steps, args.steps))
        for n in sorted({g_n, args.steps % g_n} - {0}):
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g):
                for _ in range(n):
                    one()
            graphs.append((n, g))
        torch.cuda.synchronize(dev)
    plan = []
    if graphs:
        big = graphs[-1] if graphs[-1][0] == max(n for n, _ in graphs) else graphs[0]
        q, r = divmod(args.steps, big[0])
        plan = [big[1]] * q + [g for n, g in graphs if n == r and r]
    counters.zero_()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    if plan:
        for g in plan:
            g.replay()
    else:
        for _ in range(args.steps):
            one()
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    alive = counters[0].clone()
    # per-kernel durations: HIP events on the launch stream around each kernel of nmmo_step,
    # over an equal number of eager steps right after the timed region (same state stream)
    eng.set_timing(True)
    for _ in range(min(args.steps, 8192)):
        one()
    tick_ms, obs_ms, n_timed, wrap_ms = eng.read_timing()
    eng.set_timing(False)
    # The roofline's tick duration without per-kernel event overhead (which inflates a ~15 us
    # launch by ~20%): the timed step (policy + nmmo_step, graph-replayed) minus a hipGraph of
    # `batch` policy-only launches timed with HIP events on the same stream. Timing nmmo_step
    # alone would need stale actions, which change the tick's work (attack rounds) at C3/C4.
    batch = 20
    pol_graph = torch.cuda.CUDAGraph()
    with torch.cuda.graph(pol_graph):
        for _ in range(batch):
            eng.scripted_actions(pseed)
    b0, b1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    pol_graph.replay()
    b0.record()
    reps = 10
    for _ in range(reps):
        pol_graph.replay()
    b1.record()
    torch.cuda.synchronize(dev)
    policy_avg_ms = b0.elapsed_time(b1) / (reps * batch)
    # practical HBM write ceiling on THIS box: the vendor fill kernel over the same obs buffer
    # (the same byte count the obs kernel writes per launch), HIP events on the current stream
    fill_gbs = None
    if wl["obs"]:
        s0, s1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        eng.obs.zero_()
        s0.record()
        for _ in range(10):
            eng.obs.zero_()
        s1.record()
        torch.cuda.synchronize(dev)
        fill_gbs = eng.obs.numel() * eng.obs.element_size() / (s0.elapsed_time(s1) / 10 * 1e-3) / 1e9

    vals = torch.tensor([elapsed, float(alive.item()), float(envs * cfg.PLAYER_N * args.steps)],
                        dtype=torch.float64, device=dev)
    if world > 1:
        t_max = vals[0:1].clone()
        dist.all_reduce(t_max, op=dist.ReduceOp.MAX)
        sums = vals[1:3].clone()
        dist.all_reduce(sums, op=dist.ReduceOp.SUM)
        elapsed = float(t_max.item())
        alive_total, slots_total = float(sums[0].item()), float(sums[1].item())
    else:
        alive_total, slots_total = float(vals[1].item()), float(vals[2].item())

    if rank == 0:
        S, P = eng.S, cfg.PLAYER_N
        tick_avg_ms = tick_ms / max(n_timed, 1)
        obs_avg_ms = obs_ms / max(n_timed, 1)
        tick_b = tick_bytes_per_env(S, P, "Item" in cfg.systems) * envs
        obs_b = obs_bytes_per_env(S, P, eng.obs_elems, native) * envs if wl["obs"] else 0
        if wl["obs"] and obs_avg_ms > tick_avg_ms:
            kern, byts, ms = "obs_kernel", obs_b, obs_avg_ms
            timing = "HIP events around each obs_kernel launch on the launch stream"
        else:
            kern, byts, ms = "tick_kernel", tick_b, tick_avg_ms
            timing = "HIP events around each tick_kernel launch on the launch stream"
            if not wl["obs"] and args.wrapper == "none" and plan and not gather:
                # nmmo_step = the tick kernel alone: timed step minus the policy launch
                ms = elapsed * 1e3 / args.steps - policy_avg_ms
                timing = (f"timed step (hipGraph: policy + tick) minus a {batch}-launch policy-only "
                          f"hipGraph, HIP events on the launch stream")
        achieved = byts / (ms * 1e-3) / 1e9 if ms > 0 else 0.0
        traffic, traffic_src = pmc_traffic(args.config + ("-native" if native and args.config != "C5" else ""),
                                           kern, envs)
        cpu = None
        if world == 1 and not args.no_cpu_baseline:
            # the CPU leg always builds the flat pufferlib row when the workload has obs (the
            # reference's CPU path; the oracle has no native writer)
            cpu = cpu_baseline(Config.preset(wl["preset"], early_stop_agent_num=8,
                                             obs_layout=abi.OBS_FLAT if wl["obs"] else abi.OBS_NONE),
                               args.cpu_seconds)
        line = {
            "metric": METRIC,
            "value": round(alive_total / elapsed, 1),
            "unit": "agent-steps/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(elapsed * 1e3 / args.steps, 4),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "int16",
            "data": "synthetic: generated map bank (SPEC §3), masked-uniform scripted actions (SPEC §10)",
            "config": {
                "workload": wl["desc"],
                "envs_per_gpu": envs,
                "agents_per_env": P,
                "npcs_per_env": S - P,
                "systems": list(cfg.systems),
                "obs": ("native nmmo dtypes (SPEC §8b, 9,552 B/agent + 32 KB Market/env)" if native else
                        "pufferlib-flat fp32 (23,987/agent)") if wl["obs"] else "none",
                "early_stop_agent_num": 8,
                "parallelism": f"env-shard x{world}",
            },
            "slot_steps_per_sec": round(slots_total / elapsed, 1),
            "alive_fraction": round(alive_total / slots_total, 4),
            "kernel_ms": {"policy": round(policy_avg_ms, 5), "tick": round(tick_avg_ms, 5),
                          "obs": round(obs_avg_ms, 5) if wl["obs"] else None,
                          "wrapper": round(wrap_ms / max(n_timed, 1), 5) if args.wrapper != "none" else None},
            "wrapper": None if args.wrapper == "none" else args.wrapper,
            "launch": "eager" if (args.no_graph or gather) else f"hipGraph x{min(args.graph_steps, args.steps)} ticks",
            "gather": f"RCCL gather of {eng.obs.numel() * eng.obs.element_size() + envs * cfg.PLAYER_N * 8} "
                      f"B/rank/step to rank 0" if gather else None,
            "roofline": {
                "kernel": kern,
                "bound": "hbm",
                "achieved": round(achieved, 2),
                "peak": HBM_PEAK_GBS,
                "unit": "GB/s",
                "frac": round(achieved / HBM_PEAK_GBS, 5),
                "traffic": traffic,
                "traffic_source": traffic_src,
                "bytes_per_launch": byts,
                "avg_launch_ms": round(ms, 5),
                "timing": timing,
                "write_ceiling_gbs": None if fill_gbs is None else round(fill_gbs, 1),
                "frac_of_write_ceiling": None if not fill_gbs or kern != "obs_kernel" else round(achieved / fill_gbs, 4),
            },
            "cpu_baseline": cpu,
        }
        print(json.dumps(line), file=json_out, flush=True)
    eng.close()
    if world > 1 or gather:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
