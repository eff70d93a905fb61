#!/usr/bin/env python3
"""bench.py — agent-steps/sec of the MI355X Neural MMO stepper (BASELINE.json metric).

One "step" = one tick of every env on this GPU: the scripted masked-uniform policy kernel
(SPEC.md §10, the synthetic action input) + nmmo_step (tick kernel + obs kernel). Inputs and
state are resident in HBM before the timed region. Envs shard across ranks with no data-path
collective (weak scaling: envs per GPU fixed); each rank times K steps between a barrier +
device sync, rank 0 reports the max over ranks.

  python bench.py [--gpus N] [--steps K] [--warmup W] [--config C2|C3|C4|C5] [--obs flat|native]

`--gpus N` with N > 1 and no WORLD_SIZE in the environment starts N ranks itself (a child
`torch.distributed.run --nproc-per-node N`, before anything touches the GPU) and exits with its
status; under torchrun WORLD_SIZE must equal N.

Headline workload: at N = 1, BASELINE.json configs[3] = C4, 1024 envs x 128 agents per GPU,
all ten systems, the pufferlib-flat float32 obs row the reference learner reads; the line also
carries `extra_configs` (C2, C3, C4 with the native obs layout, C5 at one GPU, C4 under the
start-kit RewardWrapper env_creator always applies) measured the same way. At N > 1 the
headline is configs[4] = C5: 1024 envs per GPU (8192 on 8), every rank's observations + packed
reward / dones / mask gathered into rank 0 every step (RCCL point-to-point over xGMI, wire
records, nmmo_amd.distributed.WireGather), with gather-free C4 as the extra. C5 reports
"delivered" (value: every agent's observation landed and validated in rank 0's HBM in the form
the experience store decodes its kept rows from), "stored" (rank 0 also stores every row of
every step as experience: compact record storage, nmmo_exp_store_records) and "decoded" (rank 0
also decodes every rank's buffers into the native layout each step).

Steady state: envs start with staggered episode phases (`--stagger L`: during an untimed
pre-roll of L ticks, the envs e = k mod L end their episode at pre-roll tick k, via
nmmo_end_episodes, the per-env reset of an async pool), so every timed window holds deaths,
culls and in-kernel auto-resets in the proportions of a long run, as in the reference's async
worker pool (config.yaml env_pool: True) where envs never run in lockstep.

value = alive agent-steps/s over the whole job (the reference's agent_SPS = sum(mask)/time,
reinforcement_learning/clean_pufferl.py:306,365), counted on the device; slot-steps/s (envs x
128 x ticks / s, the padded count, :307,364) is reported beside it. cpu_baseline = the CPU
oracle (a port of the same semantics, not nmmo 2.1, which is absent) on the host cores,
rank 0 at N = 1 only: one thread per usable core, plus the single-thread 1 env x 128 agents
C1 leg (BASELINE.json configs[0]).
"""

from __future__ import annotations

import argparse
import contextlib
import json
import os
import socket
import subprocess
import sys
import threading
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "agent-steps/sec (whole node), 128-agent envs at 1/2/4/8 MI355X"
HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec

WORKLOADS = {
    # BASELINE.json configs[1..4]
    "C2": dict(envs=256, preset="C2", obs=False,
               desc="C2: 256 envs x 128 agents, movement + food/water (Resource)"),
    "C3": dict(envs=1024, preset="C3", obs=False,
               desc="C3: 1024 envs x 128 agents, + melee/range/mage combat, NPC spawn/AI, progression"),
    "C4": dict(envs=1024, preset="C4", obs=True, layout="flat",
               desc="C4: 1024 envs x 128 agents, all systems + per-agent obs gather"),
    # C4 per GPU (8192 envs on 8) + the learner gather of every rank's obs/outputs each step
    "C5": dict(envs=1024, preset="C4", obs=True, gather=True, layout="wire",
               desc="C5: 1024 envs x 128 agents per GPU (8192 on 8), all systems + obs, RCCL "
                    "point-to-point gather of every rank's obs/reward/dones/mask to the learner "
                    "(rank 0) every step"),
}
# (config, obs layout, wrapper) measured beside the headline
EXTRAS = [("C2", None, None), ("C3", None, None), ("C4", "native", None), ("C5", None, None),
          ("C4", None, "neurips23_start_kit"), ("C4", "flat-tile-writer", "neurips23_start_kit"),
          ("C4", "flat-rezero", None)]
EXTRAS_MULTI = [("C4", None, None)]

# the agent sections' reward_wrapper weights (config.yaml:103-106, 118-126, 137-140)
WRAPPER_KW = {"neurips23_start_kit": dict(heal_bonus_weight=0.03, explore_bonus_weight=0.01),
              "takeru": dict(explore_bonus_weight=0.01, disable_give=True),
              "yaofeng": dict(hp_bonus_weight=0.03, exp_bonus_weight=0.002, defense_bonus_weight=0.04,
                              attack_bonus_weight=0.0, gold_bonus_weight=0.001, custom_bonus_scale=0.1,
                              disable_give=True, donot_attack_dangerous_npc=True)}
EVENT_ROW_BYTES = 9 * 4
TASK_STATE_BYTES = 40  # NmmoTaskState (include/nmmo_hip.h), abi.TASK_STATE_BYTES


def tick_bytes_per_env(S: int, P: int, items: bool, events_per_env: float = 0.0, slim: bool = False) -> int:
    """Algorithmic HBM bytes of one tick of one env: the env state read and
    written once (the staged int16 entity fields x slots -- 45, or 30 for the slim system sets
    without Item/Equipment/Profession/Exchange -- free-row ring, depleted-tile bitmap, env
    scalars; with the Item system the 12-slot inventories and the item-row ring), the actions
    read, the outputs written, the map tiles a player touches (own tile + 4 neighbours for
    harvest/drink, 1 move target), each player's task assignment read and its 40-B task state
    read and written (the reward's progress, SPEC §12) and the event-log rows appended (36 B
    each; measured mean per env-tick)."""
    state = (30 if slim else 45) * S * 2 + S * 2 + 800 * 4 + 16 * 4 + P * TASK_STATE_BYTES
    if items:
        state += P * 12 * 8 + 12 * P * 2
    return int(2 * state + P * 4 + P * 12 * 4 + P * (4 + 1 + 1 + 1) + P * 6 + events_per_env * EVENT_ROW_BYTES)


ROW_STATE_READ = 16 + 8 * 23   # per agent row: zrow + zst, then the extended state (ObsParams::zext, kZext u64)
ROW_STATE_WRITE = 16 + 88      # per row written in the realm: zrow + zst, the 10 chunk masks + position (the
                               # 12 item words, 96 B more, only when they changed: not counted)


def obs_bytes_per_env(S: int, P: int, elems: int, native: bool = False, wire_bytes: float | None = None,
                      stored: float | None = None, alive_frac: float = 1.0) -> float:
    """Algorithmic bytes of one env's obs gather, each byte counted once:
    the rows written (flat fp32: 23,987 x 4 B per agent; native, SPEC §8b: 9,552 B per agent +
    the env's 32 KB Market once; wire, SPEC §8c: the measured record + header bytes per env)
    + the env's 33 obs-relevant int16 entity columns read once + each agent's 15x15 window
    materials and 12 item words read. stored: the bytes one env's rows took in stores, as the
    kernel counted them (nmmo_set_obs_counter: a flat row stores only what differs from what
    the buffer holds already, nmmo_hip.h nmmo_obs_invalidate); alive_frac: the fraction of agents
    in the realm (whose windows and items are read). The incremental flat rows also read each
    row's state and write it back for the rows in the realm (ROW_STATE_READ / ROW_STATE_WRITE,
    flat_obs.hip: what lets a row store only what differs)."""
    from nmmo_amd import abi

    state = 0.0
    if wire_bytes is not None:
        rows = wire_bytes
    elif stored is not None:
        rows = stored + (abi.native_env_bytes(P) - P * abi.NATIVE_ROW_BYTES if native else 0)  # + Market
        if not native:
            state = P * (ROW_STATE_READ + ROW_STATE_WRITE * alive_frac)
    elif native:
        rows = abi.native_env_bytes(P)
    else:
        rows = P * elems * 4
    return rows + state + 33 * S * 2 + P * (225 + 12 * 8) * alive_frac


def pmc_traffic(cfg_name: str, kernel, envs: int):
    """HBM bytes per launch of `kernel` (a name, or a list of kernels one launch runs: the wire
    obs gather is wire_scan + wire_obs_kernel, after wire_count_kernel where the tick does not
    write the count words itself; a name ending in "?" counts when the summary has it) from the
    newest committed rocprofv3 PMC
    summary of the same workload (profiles/<round>/<cfg>/pmc.json, tools/pmc_summary.py):
    2 x FETCH_SIZE + WRITE_SIZE, gfx950-corrected, scaled per env to a launch of `envs` envs (the
    summary's launches covered its roofline.envs_per_launch, or its envs_per_gpu). None when no
    summary matches this workload."""
    import glob

    names = [kernel] if isinstance(kernel, str) else list(kernel)
    for path in sorted(glob.glob(os.path.join(ROOT, "profiles", "r*", cfg_name, "pmc.json")), reverse=True):
        try:
            d = json.load(open(path))
            ks = d["kernels"]
            tot = sum(ks[k]["hbm_bytes_per_dispatch"] for k in names if not k.endswith("?")) + \
                sum(ks[k[:-1]]["hbm_bytes_per_dispatch"] for k in names if k.endswith("?") and k[:-1] in ks)
            b = d.get("bench", {})
            pe = b.get("roofline", {}).get("envs_per_launch") or b.get("config", {}).get("envs_per_gpu")
            if not pe:
                continue
            return round(tot * envs / pe), os.path.relpath(path, ROOT)
        except (KeyError, ValueError, OSError, TypeError):
            continue
    return None, None


def parse(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=300)
    ap.add_argument("--warmup", type=int, default=50)
    ap.add_argument("--config", default=None, choices=sorted(WORKLOADS),
                    help="default: C4 at --gpus 1, C5 (the learner gather) at --gpus > 1")
    ap.add_argument("--envs", type=int, default=None, help="envs per GPU (default: config's)")
    ap.add_argument("--seed", type=int, default=1)
    ap.add_argument("--stagger", type=int, default=64,
                    help="pre-roll ticks over which env episode phases are staggered (0 = lockstep)")
    ap.add_argument("--cpu-seconds", type=float, default=12.0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-extras", action="store_true", help="skip the extra_configs at N = 1")
    ap.add_argument("--no-graph", action="store_true", help="eager launches instead of hipGraph replay")
    ap.add_argument("--graph-steps", type=int, default=10, help="ticks captured per hipGraph")
    ap.add_argument("--batches", type=int, default=2,
                    help="env batches per GPU, each on its own stream (1 = one handle in lockstep)")
    ap.add_argument("--obs", default=None, choices=["flat", "native"],
                    help="obs layout for the obs configs (default: flat for C4 = the pufferlib row "
                         "the reference's learner reads, native for C5 = SURVEY §8e's gather layout)")
    ap.add_argument("--wrapper", default="none",
                    choices=["none", "base", "neurips23_start_kit", "takeru", "yaofeng"],
                    help="run env_creator's RewardWrapper on the device (SPEC §13) with the "
                         "config.yaml weights")
    ap.add_argument("--no-decode", action="store_true", help="C5: skip the decoded pass")
    ap.add_argument("--root-rehearsal", type=int, default=8,
                    help="C5 at N = 1: model the node of this many GPUs from measured pieces (a peer's step at "
                         "its share, rank 0's step at its share with the other ranks' buffers received, checked "
                         "and stored: measure_root_model); 0 = off")
    ap.add_argument("--root-envs", type=int, default=None,
                    help="C5: envs on rank 0 (the learner) at N GPUs; the other ranks split the rest of "
                         "1024 x N (default: ROOT_ENVS[N])")
    ap.add_argument("--rehearse-copy", action="store_true",
                    help="C5 model: also time the root with the phantom transfers as copies (read + write)")
    ap.add_argument("--no-c5-reference", action="store_true",
                    help="N > 1: skip the one-GPU C5 reference pass (the like-for-like scaling base)")
    ap.add_argument("--dry-launch", action="store_true",
                    help="launcher check: each rank prints its RANK/WORLD_SIZE and exits (no GPU)")
    ap.add_argument("--inject-fault", action="store_true", help=argparse.SUPPRESS)  # tests: nmmo_inject_fault
    return ap.parse_args(argv)


def _free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def launch_ranks(args) -> int:
    """Start args.gpus ranks of this script under torch.distributed.run (one process per GPU,
    127.0.0.1 rendezvous) as a child process; returns its exit status. Runs before any GPU
    call in this process (the parent never initialises HIP)."""
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
           f"--nproc-per-node={args.gpus}", "--master-addr", "127.0.0.1",
           "--master-port", str(_free_port()), os.path.abspath(__file__), *sys.argv[1:]]
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    env.setdefault("OMP_NUM_THREADS", "1")
    return subprocess.call(cmd, env=env)


# ------------------------------------------------------------------------------- CPU baseline
def cpu_info() -> dict:
    """The host cores this process may use: the affinity mask, capped by a cgroup CPU quota
    when one is set (the GPU box gives each one-GPU job a share of a larger machine), and the
    CPU model."""
    try:
        affinity = len(os.sched_getaffinity(0))
    except AttributeError:
        affinity = os.cpu_count() or 1
    quota = None
    try:
        q, period = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if q != "max":
            quota = max(1, int(int(q) // int(period)))
    except (OSError, ValueError):
        pass
    model = None
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                model = line.split(":", 1)[1].strip()
                break
    except OSError:
        pass
    usable = min(affinity, quota) if quota else affinity
    return {"affinity": affinity, "cgroup_quota_cpus": quota, "usable": usable, "model": model}


def _cpu_rate(cfg, n_envs: int, threads: int, seconds: float, seed: int):
    """agent-steps/s of the CPU oracle stepping n_envs envs on `threads` Python threads (each owns
    an env range; the GIL is released inside the C calls), scripted actions included."""
    import numpy as np

    from oracle.oracle import OracleEnvs
    from oracle.oracle import lib as olib

    o = OracleEnvs(cfg, n_envs, seed=seed)
    o.reset()
    acts = np.zeros((n_envs, cfg.PLAYER_N, 12), np.int32)
    per = n_envs // threads

    def worker(k, counter, stop_at):
        lo, hi = k * per, (k + 1) * per
        t = 0
        while time.perf_counter() < stop_at:
            olib().oracle_scripted_actions_range(o.h, lo, hi, 1000 + t, acts.ctypes.data)
            o.step_range(lo, hi, acts)
            counter[k] += int(o.mask[lo:hi].sum())
            t += 1

    def run(secs, counter):
        stop_at = time.perf_counter() + secs
        ths = [threading.Thread(target=worker, args=(k, counter, stop_at)) for k in range(threads)]
        [t.start() for t in ths]
        [t.join() for t in ths]

    run(min(1.0, seconds / 4), [0] * threads)  # warm-up (page in the obs buffer)
    counter = [0] * threads
    t0 = time.perf_counter()
    run(seconds, counter)
    dt = time.perf_counter() - t0
    del o
    return sum(counter) / dt, dt


def cpu_baseline(cfg, seconds: float):
    """BASELINE.md's two CPU legs on the GPU box's host: (i) one thread per usable core over
    2 envs per thread, (ii) the single-thread 1 env x 128 agents C1 analogue."""
    info = cpu_info()
    threads = info["usable"]
    rate, dt = _cpu_rate(cfg, 2 * threads, threads, seconds, seed=7)
    c1, dt1 = _cpu_rate(cfg, 1, 1, max(2.0, seconds / 3), seed=7)
    return {
        "value": round(rate, 1),
        "unit": "agent-steps/s",
        "cores": threads,
        "kind": "port",
        "cpu_model": info["model"],
        "affinity_cpus": info["affinity"],
        "cgroup_quota_cpus": info["cgroup_quota_cpus"],
        "c1_single_thread": round(c1, 1),
        "sample": f"CPU oracle (SPEC.md port, not nmmo 2.1) on {threads} host threads (one per usable "
                  f"core) x 2 envs x {cfg.PLAYER_N} agents, same systems/obs as the GPU workload, "
                  f"{dt:.1f} s wall incl. the scripted policy; c1_single_thread = 1 thread x 1 env x "
                  f"{cfg.PLAYER_N} agents ({dt1:.1f} s)",
    }


# ------------------------------------------------------------------------------- GPU workload
def _task_embedding():
    import numpy as np

    gpath = os.path.join(ROOT, "tests", "golden", "task_embeddings.npz")
    if os.path.exists(gpath):
        return np.load(gpath)["heldout_emb"][0]  # TickGE(1024) task, SURVEY §8d
    return None


def _stagger(engs, L: int, per: int, base: int, pseed: int):
    """Staggered episode phases (module docstring): during an untimed pre-roll of L ticks, the
    envs e = k mod L (global index) end their episode at pre-roll tick k; no obs gathered."""
    import numpy as np

    for k in range(max(0, L)):
        for i, e in enumerate(engs):
            ids = np.arange(per) + base + i * per
            e.end_episodes(ids % L == k)
            e.scripted_actions(pseed)
            e.step(write_obs=False)


def _check_faults(args, engs, name, world, dist, dev):
    """The tick fault word of every engine of this workload (nmmo_get_fault), max over ranks: a
    launch that hit a loop bound did not compute the serial-order tick, so the workload fails
    (no bench line) on every rank instead of reporting a number."""
    import torch

    from nmmo_amd.engine import TickFault

    if args.inject_fault:
        engs[0].inject_fault(1)
    words = [e.get_fault() for e in engs]
    word = next((w for w in words if w), 0)
    if world > 1:
        t = torch.tensor([word], dtype=torch.int64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        word = int(t.item())
    if word:
        raise TickFault(word, f"bench {name}")


def _kernel_timing(eng, pseed: int, steps: int):
    """Per-kernel durations: HIP events on the launch stream around each kernel of nmmo_step,
    over eager steps after the timed region (same state stream), one batch alone (no overlap).
    rocprofv3's kernel trace of the same command splits these solo dispatches from the
    overlapped ones of the timed region (tools/pmc_summary.py solo_avg_ns / overlapped_avg_ns)."""
    eng.set_timing(True)
    for _ in range(min(steps, 8192)):
        eng.scripted_actions(pseed)
        eng.step()
    tick_ms, obs_ms, n_timed, wrap_ms = eng.read_timing()
    eng.set_timing(False)
    n = max(n_timed, 1)
    return tick_ms / n, obs_ms / n, wrap_ms / n


def _write_ceiling(t, dev):
    """Practical HBM write ceiling on THIS box: the vendor fill kernel over the same buffer."""
    import torch

    s0, s1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    t.zero_()
    s0.record()
    for _ in range(10):
        t.zero_()
    s1.record()
    torch.cuda.synchronize(dev)
    return t.numel() * t.element_size() / (s0.elapsed_time(s1) / 10 * 1e-3) / 1e9


_T0 = time.perf_counter()


def _progress(msg: str) -> None:
    """A progress line on stderr (stdout carries only the JSON line): long runs stay visibly alive."""
    if int(os.environ.get("RANK", "0")) == 0:
        print(f"bench.py [{time.perf_counter() - _T0:7.1f} s] {msg}", file=sys.stderr, flush=True)


def measure(args, name, layout_name, envs, rank, world, dev, steps, warmup, dist=None, wrapper=None):
    """Build, stagger, warm up and time one gather-free workload on this rank; returns a result
    dict.

    The rank's envs run as `--batches` batches (one handle each, consecutive global env indices,
    so the rollout is the same as one handle's) on their own streams (issue()), as the
    reference's async pool (config.yaml env_pool: True) overlaps env batches: with obs, a
    batch's policy and tick run under another batch's HBM-bound obs writes; without, one batch's
    bandwidth-bound state load overlaps the other's issue-bound phases. Every env still ticks
    (and writes its obs) once per step."""
    import torch

    from nmmo_amd import abi
    from nmmo_amd.config import Config
    from nmmo_amd.engine import NmmoEngine

    wrapper = wrapper or args.wrapper
    wl = WORKLOADS[name]
    native = wl["obs"] and (layout_name or wl.get("layout", "flat")) == "native"
    obs_layout = (abi.OBS_NATIVE if native else abi.OBS_FLAT) if wl["obs"] else abi.OBS_NONE
    cfg = Config.preset(wl["preset"], early_stop_agent_num=8, obs_layout=obs_layout)
    task = _task_embedding()
    nb = max(1, args.batches)
    if envs % nb:
        raise SystemExit(f"--batches {nb} must divide the {envs} envs per GPU")
    per = envs // nb
    # "flat-rezero": every obs row written in full every step (NMMO_OBS_REZERO, nmmo_hip.h
    # nmmo_obs_invalidate), beside the headline's incremental rows
    rezero = layout_name == "flat-rezero"
    # "flat-tile-writer": the start-kit consumer's contract (GpuVecEnv obs_writes={"Tile"}): every
    # step first forgets every row's Tile section (nmmo_obs_invalidate_sections), as the pool does
    # for rows whose Tile[:, :, :2] the start-kit TileEncoder edited in place (baseline_policy.py:96-97)
    tile_writer = layout_name == "flat-tile-writer"
    if rezero:
        os.environ["NMMO_OBS_REZERO"] = "1"
    try:
        engs = [NmmoEngine(cfg, per, seed=args.seed, device=dev, task_embedding=task,
                           env_index_base=rank * envs + i * per) for i in range(nb)]
    finally:
        if rezero:
            del os.environ["NMMO_OBS_REZERO"]
    eng = engs[0]
    for e in engs:
        if wrapper != "none":
            from nmmo_amd.wrappers import wrapper_config

            e.set_wrapper(wrapper_config(wrapper, **WRAPPER_KW.get(wrapper, {})))
        e.reset()
    pseed = args.seed * 1_000_003  # the policy's Philox counter already walks (tick, episode)
    _progress(f"{name}: {nb} engines built and reset")
    _stagger(engs, args.stagger, per, rank * envs, pseed)
    _progress(f"{name}: staggered over {args.stagger} ticks")
    # device counters the tick kernel adds into: [0] = sum(mask) (agent-steps), [1] = episodes,
    # [2] = event-log rows appended
    counters = [torch.zeros(3, dtype=torch.int64, device=dev) for _ in engs]
    obs_rows = [torch.zeros((per, 2), dtype=torch.int64, device=dev) for _ in engs]  # rows / bytes per env
    for e, c, r in zip(engs, counters, obs_rows):
        e.set_counters(c)
        if wl["obs"]:
            e.set_obs_counter(r)
    # nb > 1: all side streams (a capture cannot run on the legacy default stream)
    streams = [torch.cuda.current_stream(dev)] if nb == 1 else [torch.cuda.Stream(device=dev) for _ in engs]

    def issue(k, batches=None):
        """k steps of the given batches (default: all): batch j's steps (policy + nmmo_step) queue
        on stream j (nb == 1: the current stream, torch's capture stream inside
        torch.cuda.graph), and the hardware interleaves the streams."""
        for j in (range(nb) if batches is None else batches):
            with torch.cuda.stream(streams[j]) if nb > 1 else contextlib.nullcontext():
                for _ in range(k):
                    engs[j].scripted_actions(pseed)
                    if tile_writer:
                        engs[j].obs_invalidate_sections(abi.OBS_SEC_TILE)
                    engs[j].step()

    torch.cuda.synchronize(dev)  # the pre-roll ran on the default stream
    issue(warmup)
    torch.cuda.synchronize(dev)
    plans = []  # per batch: the hipGraphs its stream replays
    if not args.no_graph:  # capture-safe: no sync / alloc inside nmmo_step
        g_n = max(1, min(args.graph_steps, steps))
        q, r = divmod(steps, g_n)
        for j in range(nb):
            graphs = {}
            for n in sorted({g_n, r} - {0}):
                g = torch.cuda.CUDAGraph()
                with torch.cuda.graph(g, stream=streams[j] if nb > 1 else None):
                    issue(n, [j])
                graphs[n] = g
            plans.append([graphs[g_n]] * q + ([graphs[r]] if r else []))
        torch.cuda.synchronize(dev)
    for c in counters + obs_rows:
        c.zero_()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    if plans:
        for k in range(len(plans[0])):
            for j in range(nb):
                with torch.cuda.stream(streams[j]) if nb > 1 else contextlib.nullcontext():
                    plans[j][k].replay()
    else:
        issue(steps)
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    tot = torch.stack(counters).sum(0)
    alive = float(tot[0].item())
    episodes = int(tot[1].item())
    obs_cnt = torch.stack(obs_rows).sum((0, 1))
    rows_written, bytes_stored = float(obs_cnt[0].item()), float(obs_cnt[1].item())
    events_per_env_tick = float(tot[2].item()) / (envs * steps) if cfg.event_cap > 0 else None
    _progress(f"{name}: timed {steps} steps in {elapsed:.3f} s")
    tick_avg_ms, obs_avg_ms, wrap_avg_ms = _kernel_timing(eng, pseed, steps)
    # The roofline's tick duration without per-kernel event overhead (which inflates a ~15 us
    # launch by ~20%): the timed step (policy + nmmo_step, graph-replayed) minus a hipGraph of
    # `batch` policy-only launches timed with HIP events on the same stream. Timing nmmo_step
    # alone would need stale actions, which change the tick's work (attack rounds).
    batch, reps = 20, 10
    pol_graph = torch.cuda.CUDAGraph()
    with torch.cuda.graph(pol_graph):
        for _ in range(batch):
            eng.scripted_actions(pseed)
    b0, b1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    pol_graph.replay()
    b0.record()
    for _ in range(reps):
        pol_graph.replay()
    b1.record()
    torch.cuda.synchronize(dev)
    policy_avg_ms = b0.elapsed_time(b1) / (reps * batch)
    solo_step_ms = None
    if not wl["obs"] and wrapper == "none" and plans and nb > 1:
        # one batch alone (the timed region overlaps the batches): a hipGraph of `batch` steps
        step_graph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(step_graph):
            for _ in range(batch):
                eng.scripted_actions(pseed)
                eng.step()
        step_graph.replay()
        b0.record()
        for _ in range(reps):
            step_graph.replay()
        b1.record()
        torch.cuda.synchronize(dev)
        solo_step_ms = b0.elapsed_time(b1) / (reps * batch)
    fill_gbs = _write_ceiling(eng.obs, dev) if wl["obs"] else None

    S, P = eng.S, cfg.PLAYER_N
    slim = not any(x in cfg.systems for x in ("Item", "Equipment", "Profession", "Exchange"))
    tick_b = tick_bytes_per_env(S, P, "Item" in cfg.systems, events_per_env_tick or 0.0, slim) * per
    row_frac = rows_written / (envs * P * steps)  # the timed steps' rows written per agent row
    obs_b = obs_bytes_per_env(S, P, eng.obs_elems, native, stored=bytes_stored / (envs * steps),
                              alive_frac=alive / (envs * P * steps)) * per if wl["obs"] else 0
    if wl["obs"] and obs_avg_ms > tick_avg_ms:
        # incremental flat rows: flat_obs_kernel; every row in full (rezero): obs_kernel
        kern = "native_obs_kernel" if native else "obs_kernel" if rezero else "flat_obs_kernel"
        byts, ms = obs_b, obs_avg_ms
        timing = f"HIP events around each {kern} launch on the launch stream"
    else:
        kern, byts, ms = "tick_kernel", tick_b, tick_avg_ms
        timing = "HIP events around each tick_kernel launch on the launch stream"
        if not wl["obs"] and wrapper == "none" and plans:
            if nb == 1:
                ms = elapsed * 1e3 / steps - policy_avg_ms  # nmmo_step = the tick kernel alone
                timing = (f"timed step (hipGraph: policy + tick) minus a {batch}-launch policy-only "
                          f"hipGraph, HIP events on the launch stream")
            else:
                ms = solo_step_ms - policy_avg_ms
                timing = (f"one batch alone after the timed region: a {batch}-step hipGraph (policy + "
                          f"tick) minus a {batch}-launch policy-only hipGraph, HIP events on the "
                          f"launch stream")
    full_b = None  # §8(d)'s model: every row written in full
    if wl["obs"] and kern != "tick_kernel" and not rezero:
        full_b = obs_bytes_per_env(S, P, eng.obs_elems, native, alive_frac=alive / (envs * P * steps)) * per
    prof_name = name + ("-native" if native else "-rezero" if rezero else "-tilewriter" if tile_writer else "") + \
        ("" if wrapper == "none" else "+" + wrapper)
    launch = "eager" if not plans else f"hipGraph x{min(args.graph_steps, steps)} ticks"
    if nb > 1:
        launch += f", {nb} batches of {per} envs on {nb} streams"
    res = {
        "name": prof_name, "envs": envs, "cfg": cfg, "layout": "native" if native else "flat", "S": S, "P": P,
        "elapsed": elapsed, "alive": alive, "slots": float(envs * P * steps), "episodes": episodes,
        "events_per_env_tick": events_per_env_tick, "gather": False, "launch": launch, "wrapper": wrapper,
        "kernel_ms": {"policy": round(policy_avg_ms, 5), "tick": round(tick_avg_ms, 5),
                      "obs": round(obs_avg_ms, 5) if wl["obs"] else None,
                      "wrapper": round(wrap_avg_ms, 5) if wrapper != "none" else None},
        "roofline": _roofline(prof_name, kern, byts, ms, per, timing, nb, elapsed / steps, fill_gbs, full_b=full_b,
                              byte_model=None if not wl["obs"] or kern == "tick_kernel" else
                              "full rows" if rezero else "stored bytes"),
        "batches": nb,
        "obs_contract": None if not wl["obs"] else
        ("every row written in full each step (GpuVecEnv obs_writes=\"all\": a consumer that may edit any "
         "section in place)" if rezero else
         "incremental rows with every Tile section rewritten each step (GpuVecEnv obs_writes={\"Tile\"}, the "
         "start-kit agent's default: its TileEncoder edits Tile[:, :, :2] in place)" if tile_writer else
         "incremental rows into the engine's bound buffer: a row stores only what differs from what the buffer "
         "holds (DESIGN.md §3.2c); valid for a read-only consumer (GpuVecEnv obs_writes=set(): the takeru and "
         "yaofeng agents' default)"),
        "obs_rows_written_frac": round(row_frac, 4) if wl["obs"] else None,
        "obs_bytes_stored_per_agent_row": round(bytes_stored / (envs * P * steps), 1) if wl["obs"] else None,
    }
    _check_faults(args, engs, name, world, dist, dev)  # every tick of this workload ran (timed and after)
    for e in engs:
        e.close()
    del eng, engs
    torch.cuda.empty_cache()
    return res


def _roofline(prof_name, kern, byts, ms, per, timing, nb, step_s, fill_gbs, pmc_kernels=None, full_b=None,
              byte_model=None):
    """The dominant kernel's roofline entry. byte_model names what `achieved` counts: "stored
    bytes" for the incremental obs rows (the bytes the kernel stored, counted on the device, plus
    its reads: DESIGN.md §3.2c), "full rows" for every row written in full (§8(d)'s model). With
    stored bytes, `full_row_model` puts §8(d)'s full-row bytes over the same launch beside it: a
    frac > 1 there says the launch stores far less than a full write, not that it beats HBM."""
    achieved = byts / (ms * 1e-3) / 1e9 if ms > 0 else 0.0
    traffic, traffic_src = pmc_traffic(prof_name, pmc_kernels or kern, per)
    full = None
    if full_b is not None and ms > 0:
        fa = full_b / (ms * 1e-3) / 1e9
        full = {"bytes_per_launch": round(full_b), "achieved": round(fa, 1), "frac": round(fa / HBM_PEAK_GBS, 4)}
    return {
        "kernel": kern, "bound": "hbm", "byte_model": byte_model, "full_row_model": full,
        "achieved": round(achieved, 2), "peak": HBM_PEAK_GBS,
        "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 5), "traffic": traffic,
        "traffic_source": traffic_src, "bytes_per_launch": round(byts), "envs_per_launch": per,
        "avg_launch_ms": round(ms, 5), "timing": timing,
        # the dominant kernel's bytes of a whole step over the timed step time: a floor on its
        # in-run rate (policy and tick share the step; --batches overlaps them)
        "timed_step_gbs": round(byts * nb / step_s / 1e9, 1),
        "concurrent_batches": nb,
        "write_ceiling_gbs": None if fill_gbs is None else round(fill_gbs, 1),
        "frac_of_write_ceiling": None if not fill_gbs or kern != "obs_kernel" else round(achieved / fill_gbs, 4),
    }


# C5's learner share (distributed.env_shares): envs on rank 0 at N GPUs (8 * 1024 envs on 8),
# the other ranks split the rest. The root validates and stores every peer's buffers each step
# besides its own compute, so it holds fewer envs; DESIGN.md §5 derives the shares from the
# measured root and peer steps (bench C5 extra at N = 1: root_loaded / peer passes).
ROOT_ENVS = {2: 984, 4: 832, 8: 448}
XGMI_LINK_GBS = 153.6   # per xGMI link (task brief: 7 links x ~153 GB/s per GPU)
LINK_EFF = 0.75         # the share of it the N = 8 model assumes a point-to-point send gets


def c5_shares(args, world: int, nb: int):
    """Per-rank env counts of C5 at `world` ranks (1024 per GPU in total)."""
    from nmmo_amd.distributed import env_shares

    total = (args.envs or WORKLOADS["C5"]["envs"]) * world
    k = args.root_envs if args.root_envs is not None else ROOT_ENVS.get(world) if args.envs is None else None
    return env_shares(total, world, None if world == 1 else k, granule=nb)


def _wire_engines(args, cfg, task, envs, base, nb, dev, pseed):
    from nmmo_amd.engine import NmmoEngine

    if envs % nb:
        raise SystemExit(f"--batches {nb} must divide the {envs} envs of this rank")
    per = envs // nb
    engs = [NmmoEngine(cfg, per, seed=args.seed, device=dev, task_embedding=_task_embedding(),
                       env_index_base=base + i * per) for i in range(nb)]
    for e in engs:
        e.reset()
    _stagger(engs, args.stagger, per, base, pseed)
    return engs


def _gather_pass(args, engs, g, steps, warmup, world, dist, dev, counters, store=None):
    """Warm up, then time `steps` steps of WireGather g (barrier + device sync on both sides)."""
    import torch

    for _ in range(warmup):
        g.step()
    g.drain()
    torch.cuda.synchronize(dev)
    if store is not None:
        g.stored_rows()  # the warm-up's rows do not count
    for c in counters:
        c.zero_()
    b0 = g.x.payload_bytes
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    g.host_s = g.x.wait_s = 0.0
    t0 = time.perf_counter()
    for _ in range(steps):
        g.step()
    host_work = (g.host_s - g.x.wait_s) / steps
    g.drain()
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    tot = torch.stack(counters).sum(0)
    status = g.check_status()
    if status:
        raise RuntimeError(f"the received-buffer check flagged wire buffers (status {status})")
    stored = g.stored_rows() if store is not None else None
    if store is not None and store.status:
        raise RuntimeError(f"the root's record store dropped rows (status {store.status})")
    return {"elapsed": elapsed, "alive": float(tot[0].item()), "episodes": int(tot[1].item()),
            "events": float(tot[2].item()), "stored_rows": stored,
            "payload_bytes_per_step": (g.x.payload_bytes - b0) / steps, "host_ms_per_step": host_work * 1e3}


def _record_store(per_list, dev, P):
    """Compact record storage for every row of one step of buffers of per_list envs (rank 0)."""
    from nmmo_amd import wire as nw
    from nmmo_amd.storage import DeviceExperience

    rows = sum(per_list) * P
    arena = sum(nw.max_bytes(n, P) + 64 for n in per_list)
    return DeviceExperience(rows, 23987, rows, device=dev, record_arena_bytes=arena)


def measure_gather(args, name, envs, rank, world, dev, steps, warmup, dist=None, backend="nccl", shares=None,
                   modes=None):
    """C5: the rank's envs (its share of the node) as `--batches` wire-obs handles stepped by
    WireGather (policy + nmmo_step into a ring of wire buffers, hipGraph-captured, one stream per
    batch; the learner gather into rank 0 one step behind on a comm stream). Timed passes over
    the same engines: "delivered" (rank 0 validates every received buffer on the device),
    "stored" (rank 0 also stores every row of every step in compact record storage, the check
    fused into the store) and "decoded" (rank 0 also decodes every rank's buffers into the native
    layout each step)."""
    import torch

    from nmmo_amd import abi
    from nmmo_amd.config import Config
    from nmmo_amd.distributed import WireGather

    wl = WORKLOADS[name]
    cfg = Config.preset(wl["preset"], early_stop_agent_num=8, obs_layout=abi.OBS_WIRE)
    nb = max(1, args.batches)
    shares = shares or [envs]
    envs = shares[rank]
    base = sum(shares[:rank])
    pseed = args.seed * 1_000_003
    engs = _wire_engines(args, cfg, None, envs, base, nb, dev, pseed)
    per = envs // nb
    _progress(f"{name}: {nb} engines of {per} envs built, reset and staggered over {args.stagger} ticks")
    counters = [torch.zeros(3, dtype=torch.int64, device=dev) for _ in engs]
    for e, c in zip(engs, counters):
        e.set_counters(c)
    torch.cuda.synchronize(dev)
    passes = {}
    modes = modes or (("delivered",) if args.no_decode else ("delivered", "stored", "decoded"))
    for mode in modes:
        store = None
        if mode == "stored" and rank == 0:  # compact record storage of every row of every step
            store = _record_store([n // nb for n in shares for _ in range(nb)], dev, cfg.PLAYER_N)
        g = WireGather(engs, pseed, rank, world, decode=mode == "decoded", graphs=not args.no_graph,
                       backend=backend, store=store)
        passes[mode] = _gather_pass(args, engs, g, steps, warmup, world, dist, dev, counters, store)
        _progress(f"{name}: timed {steps} steps in {passes[mode]['elapsed']:.3f} s ({mode})")
        g.close()
        del store
    eng = engs[0]
    tick_avg_ms, obs_avg_ms, _ = _kernel_timing(eng, pseed, steps)
    _check_faults(args, engs, name, world, dist, dev)
    from nmmo_amd import wire as nw

    wire_env_bytes = nw.total_bytes(eng.obs) / per  # this batch's last step: header + records
    S, P = eng.S, cfg.PLAYER_N
    d = passes["delivered"]
    events_per_env_tick = d["events"] / (envs * steps)
    tick_b = tick_bytes_per_env(S, P, True, events_per_env_tick) * per
    obs_b = obs_bytes_per_env(S, P, eng.obs_elems, wire_bytes=wire_env_bytes) * per
    if obs_avg_ms > tick_avg_ms:
        kern, byts, ms = "wire_obs_kernel", obs_b, obs_avg_ms
        timing = ("HIP events around each wire obs gather (wire_scan + wire_obs_kernel; the count words come "
                  "from the tick, tick.hip wire_count_fused) on the launch stream")
    else:
        kern, byts, ms = "tick_kernel", tick_b, tick_avg_ms
        timing = "HIP events around each tick_kernel launch on the launch stream"
    res = {
        "name": name, "envs": envs, "cfg": cfg, "layout": "wire", "S": S, "P": P,
        "elapsed": d["elapsed"], "alive": d["alive"], "slots": float(envs * P * steps), "episodes": d["episodes"],
        "events_per_env_tick": events_per_env_tick, "gather": True, "wrapper": "none",
        "launch": f"hipGraph per step and ring slot, {nb} batches of {per} envs on {nb} streams, gather on a "
                  f"comm stream one step behind",
        "kernel_ms": {"policy": None, "tick": round(tick_avg_ms, 5), "obs": round(obs_avg_ms, 5), "wrapper": None},
        "roofline": _roofline(name, kern, byts, ms, per, timing, nb, d["elapsed"] / steps, None,
                              ["wire_count_kernel?", "wire_scan_kernel", "wire_obs_kernel"] if kern == "wire_obs_kernel"
                              else None),
        "batches": nb,
        "shares": list(shares),
        "gather_bytes": d["payload_bytes_per_step"] if world > 1 else 0,
        "host_ms_per_step": round(d["host_ms_per_step"], 4),
        "wire_bytes_per_env": round(wire_env_bytes, 1),
        "wire_bytes_per_agent_in_realm": round(wire_env_bytes * per * nb * steps / max(d["alive"], 1.0), 1),
        "decoded": passes.get("decoded"),
        "stored": passes.get("stored"),
    }
    for e in engs:
        e.close()
    del eng, engs
    torch.cuda.empty_cache()
    return res


def measure_root_model(args, dev, steps, warmup, n_model: int = 8):
    """The N = n_model node of C5 from its measured pieces on one GPU:
      peer: one peer's step at its share of the node (C5 delivered, world 1, peer-share envs);
      root_loaded: rank 0's step at its share with n_model - 1 phantom peers' buffers received
        (write-only fills of their bytes), validated and stored every step (the fused checked
        store): the root's whole load (WireGather rehearse, phantom = the peer pass's buffers);
      link: the bytes one peer sends per step over its own xGMI link at LINK_EFF of XGMI_LINK_GBS.
    The node delivers (root's + peers' agents in the realm per step) / max(root, peer, link)."""
    import torch

    from nmmo_amd import abi
    from nmmo_amd.config import Config
    from nmmo_amd.distributed import WireGather

    nb = max(1, args.batches)
    shares = c5_shares(args, n_model, nb)
    k_root, e_peer = shares[0], shares[1]
    cfg = Config.preset("C4", early_stop_agent_num=8, obs_layout=abi.OBS_WIRE)
    P = cfg.PLAYER_N
    pseed = args.seed * 1_000_003
    # 1. a peer's share, stepped alone (rank 1's env block); its last buffers become the phantoms
    engs = _wire_engines(args, cfg, None, e_peer, shares[0], nb, dev, pseed)
    counters = [torch.zeros(3, dtype=torch.int64, device=dev) for _ in engs]
    for e, c in zip(engs, counters):
        e.set_counters(c)
    g = WireGather(engs, pseed, 0, 1, graphs=not args.no_graph)
    peer = _gather_pass(args, engs, g, steps, warmup, 1, None, dev, counters)
    _progress(f"C5 model: peer share {e_peer} envs, {peer['elapsed'] * 1e3 / steps:.4f} ms/step")
    from nmmo_amd import wire as nw

    # the phantoms = the peer's last step: its wire buffers (the announced bytes) and step records
    k = (g.t - 1) % g.ring
    phantom, peer_bytes = [], 0
    for j, e in enumerate(engs):
        w = g.wires[j][k]
        tot = nw.total_bytes(w)
        peer_bytes += tot + g.smalls[j][k].numel()  # what a peer sends per step: wire bytes + step records
        phantom.append((w[:tot].clone(), g.smalls[j][k].clone(), e.n_envs))
    g.close()
    for e in engs:
        e.close()
    del engs, g
    torch.cuda.empty_cache()
    # 2. the root's share with n_model - 1 phantom peers received, checked and stored each step
    engs = _wire_engines(args, cfg, None, k_root, 0, nb, dev, pseed)
    counters = [torch.zeros(3, dtype=torch.int64, device=dev) for _ in engs]
    for e, c in zip(engs, counters):
        e.set_counters(c)
    R = n_model - 1
    store = _record_store([k_root // nb] * nb + [n for _, _, n in phantom] * R, dev, P)
    out = {}
    for mode in ("fill", "copy") if args.rehearse_copy else ("fill",):
        store.reset()
        g = WireGather(engs, pseed, 0, 1, graphs=not args.no_graph, store=store, rehearse=R, phantom=phantom,
                       rehearse_mode=mode)
        out[mode] = _gather_pass(args, engs, g, steps, warmup, 1, None, dev, counters, store)
        _progress(f"C5 model: root share {k_root} envs + {R} phantom peers ({mode}), "
                  f"{out[mode]['elapsed'] * 1e3 / steps:.4f} ms/step")
        g.close()
    for e in engs:
        e.close()
    del engs, g, store
    torch.cuda.empty_cache()
    root = out["fill"]
    root_ms = root["elapsed"] * 1e3 / steps
    peer_ms = peer["elapsed"] * 1e3 / steps
    link_ms = peer_bytes / (LINK_EFF * XGMI_LINK_GBS * 1e9) * 1e3
    alive_step = root["alive"] / steps + R * peer["alive"] / steps
    step_ms = max(root_ms, peer_ms, link_ms)
    res = {
        "n_gpus": n_model, "shares": shares,
        "root_loaded": {"envs": k_root, "phantom_peers": R, "ms_per_step": round(root_ms, 4),
                        "host_ms_per_step": round(root["host_ms_per_step"], 4),
                        "stored_rows_per_step": round((root["stored_rows"] or 0) / steps, 1),
                        "what": f"rank 0's step at its share ({k_root} envs) with {R} phantom peers' buffers "
                                f"({e_peer} envs each) received (write-only fills of their bytes), validated and "
                                f"stored every step (nmmo_exp_store_records_checked)"},
        "peer": {"envs": e_peer, "ms_per_step": round(peer_ms, 4), "bytes_per_step": int(peer_bytes),
                 "what": f"one peer's step at its share ({e_peer} envs), gather-free"},
        "link": {"ms_per_step": round(link_ms, 4), "gbs": round(LINK_EFF * XGMI_LINK_GBS, 1),
                 "what": f"a peer's wire buffers + step records over its own xGMI link at {LINK_EFF:.0%} of "
                         f"{XGMI_LINK_GBS} GB/s"},
        "step_ms": round(step_ms, 4),
        "bound": "root" if step_ms == root_ms else "peer" if step_ms == peer_ms else "link",
        "value": round(alive_step / (step_ms * 1e-3), 1),
    }
    if "copy" in out:
        res["root_loaded"]["copy_ms_per_step"] = round(out["copy"]["elapsed"] * 1e3 / steps, 4)
    return res


def _node_model(m, one_gpu_value):
    m = dict(m)
    m["ratio_vs_one_gpu"] = round(m["value"] / one_gpu_value, 3)
    m["what"] = (f"the N = {m['n_gpus']} C5 node from pieces measured here (DESIGN.md §5): agents in the realm per "
                 f"step of the root's and the peers' shares / max(root_loaded, peer, link); ratio_vs_one_gpu against "
                 f"C5 at N = 1 measured in this run")
    return m


def result_line(res, args, world, steps, alive_total, slots_total, elapsed, warmup):
    cfg = res["cfg"]
    wl_desc = WORKLOADS[res["name"].split("-")[0].split("+")[0]]["desc"]
    obs = {"flat": "pufferlib-flat fp32 (23,987/agent)",
           "native": "native nmmo dtypes (SPEC §8b, 9,552 B/agent + 32 KB Market/env)",
           "wire": "wire records (SPEC §8c) written straight from the state"}[res["layout"]] \
        if WORKLOADS[res["name"].split("-")[0].split("+")[0]]["obs"] else "none"
    line = {
        "value": round(alive_total / elapsed, 1),
        "ms_per_step": round(elapsed * 1e3 / steps, 4),
        "config": {
            "workload": wl_desc,
            "envs_per_gpu": res["envs"],
            "agents_per_env": res["P"],
            "npcs_per_env": res["S"] - res["P"],
            "systems": list(cfg.systems),
            "obs": obs,
            "wrapper": None if res.get("wrapper", "none") == "none" else res["wrapper"],
            "early_stop_agent_num": 8,
            "stagger_ticks": args.stagger,
            "env_batches": res["batches"],
            "parallelism": f"env-shard x{world}" + (", learner gather to rank 0" if res["gather"] else ""),
        },
        "slot_steps_per_sec": round(slots_total / elapsed, 1),
        "alive_fraction": round(alive_total / slots_total, 4),
        "episodes_ended": res["episodes"],
        "events_per_env_tick": None if res["events_per_env_tick"] is None else round(res["events_per_env_tick"], 3),
        "kernel_ms": res["kernel_ms"],
        "launch": res["launch"],
        "roofline": res["roofline"],
    }
    if res.get("obs_contract"):
        line["config"]["obs_contract"] = res["obs_contract"]
    if res.get("obs_rows_written_frac") is not None:
        # the obs rows are written incrementally: the buffer's bytes after every step equal a full
        # write (nmmo_hip.h nmmo_obs_invalidate, tests/test_gpu_zero_rows.py)
        line["obs_rows_written_frac"] = res["obs_rows_written_frac"]
        line["obs_bytes_stored_per_agent_row"] = res["obs_bytes_stored_per_agent_row"]
    if res["gather"]:
        line["wire_bytes_per_agent_in_realm"] = res["wire_bytes_per_agent_in_realm"]
        line["host_ms_per_step"] = res["host_ms_per_step"]  # rank 0's host work per step (no waits)
    return line


def _gather_fields(res, world, backend, steps):
    """The C5 line's gather description and its decoded pass (whole job, max over ranks)."""
    via = "RCCL" if backend == "nccl" else "gloo (rehearsal)"
    out = {"gather": (f"{via} point-to-point sends into rank 0 of {round(res['gather_bytes'])} B/step of wire "
                      f"records (+ reward/dones/mask), one step behind the compute on a comm stream; rank 0 "
                      f"validates every received buffer (nmmo_wire_check) and keeps its own in place"
                      if world > 1 else "N = 1: rank 0's own wire buffers in place, nothing sent"),
           "gather_bytes_per_step": round(res["gather_bytes"]) if world > 1 else 0}
    return out


def main():
    args = parse()
    world_env = os.environ.get("WORLD_SIZE")
    if args.dry_launch and world_env is not None:
        # one write() per line: the ranks share the launcher's stdout pipe, and print() issues the
        # text and its newline as two writes that another rank's line can land between
        sys.stdout.write(json.dumps({"rank": int(os.environ["RANK"]), "world_size": int(world_env),
                                     "local_rank": int(os.environ.get("LOCAL_RANK", "0"))}) + "\n")
        sys.stdout.flush()
        return 0
    if world_env is None and args.gpus > 1:
        return launch_ranks(args)
    world = int(world_env or "1")
    if world != args.gpus:
        print(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={world}", file=sys.stderr)
        return 2
    if args.dry_launch:
        print(json.dumps({"rank": 0, "world_size": 1, "local_rank": 0}), flush=True)
        return 0
    # The JSON line is the only thing on stdout: native libraries (RCCL prints a version banner
    # on stdout when a communicator is created) are sent to stderr by pointing fd 1 at fd 2.
    json_out = os.fdopen(os.dup(1), "w")
    sys.stdout.flush()
    os.dup2(2, 1)
    _progress("importing torch")
    import torch
    import torch.distributed as dist

    from nmmo_amd import _native
    _progress("torch imported")

    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # NMMO_BENCH_BACKEND=gloo rehearses the multi-rank path on fewer GPUs than ranks (ranks share
    # devices round-robin; gloo reduces the CUDA timing tensors through the host). The bench
    # proper is one rank per GPU over RCCL ("nccl").
    backend = os.environ.get("NMMO_BENCH_BACKEND", "nccl")
    ndev = torch.cuda.device_count()
    torch.cuda.set_device((local % ndev if backend == "gloo" else local) if world > 1 else 0)
    dev = torch.device("cuda", torch.cuda.current_device())
    if world > 1:
        if backend == "gloo":
            dist.init_process_group("gloo")
        else:
            dist.init_process_group("nccl", device_id=dev)

    name = args.config or ("C4" if world == 1 else "C5")
    wl = WORKLOADS[name]
    envs = args.envs or wl["envs"]

    def run(nm, lay, wrapper, n_envs, steps, warmup):
        t0 = time.perf_counter()
        if WORKLOADS[nm].get("gather"):
            shares = c5_shares(args, world, max(1, args.batches))
            r = measure_gather(args, nm, n_envs, rank, world, dev, steps, warmup, dist, backend, shares=shares)
            if world == 1 and args.root_rehearsal > 1 and args.envs is None:
                r["n_model"] = measure_root_model(args, dev, steps, warmup, args.root_rehearsal)
        else:
            r = measure(args, nm, lay, n_envs, rank, world, dev, steps, warmup, dist, wrapper)
        _progress(f"{r['name']} measured in {time.perf_counter() - t0:.1f} s")
        return r

    def reduce(res, key="elapsed", alive="alive"):
        vals = torch.tensor([res[key], res[alive], res["slots"]], dtype=torch.float64, device=dev)
        if world > 1:
            t_max = vals[0:1].clone()
            dist.all_reduce(t_max, op=dist.ReduceOp.MAX)
            sums = vals[1:3].clone()
            dist.all_reduce(sums, op=dist.ReduceOp.SUM)
            return float(t_max.item()), float(sums[0].item()), float(sums[1].item())
        return res[key], res[alive], res["slots"]

    def learner_passes(r, steps):
        """The C5 line's learner-side passes (whole job, max over ranks): "stored" (rank 0 keeps
        every row of every step in compact record storage) and "decoded"."""
        out = {}
        for mode, what in (("stored", "rank 0 also stores every rank's rows in the realm each step as "
                                      "experience (nmmo_exp_store_records: the rows' fields + their wire "
                                      "records in an arena, flat rows expanded per minibatch)"),
                           ("decoded", "rank 0 also decodes every rank's wire buffers into the native layout "
                                       "(nmmo_wire_unpack) each step: the full learner-ready obs tensor"),
                           ):
            if not r.get(mode):
                continue
            pr = dict(r, elapsed=r[mode]["elapsed"], alive=r[mode]["alive"])
            el, al, _ = reduce(pr)
            out[mode] = {"value": round(al / el, 1), "ms_per_step": round(el * 1e3 / steps, 4), "what": what}
            if r[mode].get("stored_rows") is not None:
                out[mode]["rows_stored_per_sec"] = round(r[mode]["stored_rows"] / el, 1)
        return out

    res = run(name, args.obs, None, envs, args.steps, args.warmup)
    elapsed, alive_total, slots_total = reduce(res)
    passes = learner_passes(res, args.steps) if res.get("gather") else {}
    one_gpu = None
    if res.get("gather") and world > 1 and not args.no_c5_reference:
        # the like-for-like scaling base: C5 at N = 1 (1024 envs, the root's own buffers in place,
        # nothing sent) on rank 0's GPU in this run, while the other ranks wait
        if rank == 0:
            n1 = args.envs or WORKLOADS["C5"]["envs"]
            r1 = measure_gather(args, "C5", n1, 0, 1, dev, args.steps, args.warmup, None, backend, shares=[n1],
                                modes=("delivered",))
            one_gpu = {"value": round(r1["alive"] / r1["elapsed"], 1),
                       "ms_per_step": round(r1["elapsed"] * 1e3 / args.steps, 4), "envs": n1,
                       "what": "C5 at N = 1 measured in this run on rank 0's GPU (its own wire buffers in place, "
                               "nothing sent): the base of a like-for-like N > 1 scaling ratio"}
        dist.barrier()

    extras = {}
    if not args.no_extras and not args.envs and args.config is None:
        ex_steps, ex_warm = max(args.steps, 100), max(args.warmup, 20)
        for nm, lay, wrapper in (EXTRAS if world == 1 else EXTRAS_MULTI):
            r = run(nm, lay, wrapper, WORKLOADS[nm]["envs"], ex_steps, ex_warm)
            el, al, sl = reduce(r)
            line = result_line(r, args, world, ex_steps, al, sl, el, ex_warm)
            line["steps"], line["warmup"] = ex_steps, ex_warm
            if r.get("gather"):
                line.update(_gather_fields(r, world, backend, ex_steps))
                line.update(learner_passes(r, ex_steps))
                if r.get("n_model"):
                    line["node_model"] = _node_model(r["n_model"], line["value"])
            extras[r["name"]] = line

    if rank == 0:
        cpu = None
        if world == 1 and not args.no_cpu_baseline:
            from nmmo_amd import abi
            from nmmo_amd.config import Config

            # the CPU leg builds the flat pufferlib row when the workload has obs (the
            # reference's CPU path; the oracle has no native writer)
            _progress("CPU baseline")
            cpu = cpu_baseline(Config.preset(wl["preset"], early_stop_agent_num=8,
                                             obs_layout=abi.OBS_FLAT if wl["obs"] else abi.OBS_NONE),
                               args.cpu_seconds)
        body = result_line(res, args, world, args.steps, alive_total, slots_total, elapsed, args.warmup)
        line = {
            "metric": METRIC,
            "value": body.pop("value"),
            "unit": "agent-steps/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": body.pop("ms_per_step"),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "int16",
            "data": "synthetic: generated map bank (SPEC §3), masked-uniform scripted actions "
                    f"(SPEC §10), episode phases staggered over {args.stagger} pre-roll ticks",
        }
        line.update(body)
        line["wrapper"] = None if args.wrapper == "none" else args.wrapper
        if res["gather"]:
            line.update(_gather_fields(res, world, backend, args.steps))
            line["value_kind"] = "delivered"
            line.update(passes)
            line["config"]["envs_per_rank"] = res["shares"]
            if res.get("n_model"):
                line["node_model"] = _node_model(res["n_model"], line["value"])
            if one_gpu:
                line["c5_one_gpu"] = one_gpu
                line["scaling_vs_c5_one_gpu"] = round(line["value"] / one_gpu["value"], 3)
                line["like_for_like"] = ("scaling_vs_c5_one_gpu divides this line's value by C5 at N = 1 measured in "
                                         "the same run; the N = 1 headline (bench.py --gpus 1) is C4 with flat obs, a "
                                         "different workload, so value(N) / value(1) across the two lines is not a "
                                         "scaling ratio")
        else:
            line["gather"] = None
        line["cpu_baseline"] = cpu
        fw = extras.get("C4-rezero") if res["name"] == "C4" else None
        if fw:  # the headline's full-write figure (a consumer that may edit its rows) beside it
            line["full_write"] = {"value": fw["value"], "ms_per_step": fw["ms_per_step"],
                                  "obs_ms": fw["kernel_ms"]["obs"], "roofline_frac": fw["roofline"]["frac"],
                                  "frac_of_write_ceiling": fw["roofline"]["frac_of_write_ceiling"],
                                  "see": "extra_configs.C4-rezero"}
        tw = extras.get("C4-tilewriter+neurips23_start_kit") if res["name"] == "C4" else None
        if tw:  # the reference's start-kit loop: its wrapper, its policy's Tile edit (obs_writes={"Tile"})
            line["start_kit_consumer"] = {"value": tw["value"], "ms_per_step": tw["ms_per_step"],
                                          "obs_ms": tw["kernel_ms"]["obs"], "see": "extra_configs.C4-tilewriter"
                                          "+neurips23_start_kit"}
        line["extra_configs"] = extras or None
        line["build"] = _native.build_info()
        print(json.dumps(line), file=json_out, flush=True)
    if world > 1:
        dist.destroy_process_group()
    return 0


if __name__ == "__main__":
    sys.exit(main())
