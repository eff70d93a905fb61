"""Debug: tracked flat vs full-rewrite flat vs native expand, start_kit wrapper, after reset."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from nmmo_amd import abi  # noqa: E402
from nmmo_amd.config import Config  # noqa: E402
from nmmo_amd.engine import NmmoEngine  # noqa: E402
from nmmo_amd.wrappers import wrapper_config  # noqa: E402

n = 3
task = (np.arange(2048) % 53 / 53.0 - 0.25).astype(np.float16)
for wrapper in [None, "neurips23_start_kit", "neurips23_start_kit"]:
    flat = NmmoEngine(Config.preset("C4", MAP_N=4, early_stop_agent_num=8), n, seed=13, task_embedding=task)
    os.environ["NMMO_OBS_REZERO"] = "1"
    full = NmmoEngine(Config.preset("C4", MAP_N=4, early_stop_agent_num=8), n, seed=13, task_embedding=task)
    del os.environ["NMMO_OBS_REZERO"]
    nat = NmmoEngine(Config.preset("C4", MAP_N=4, early_stop_agent_num=8, obs_layout=abi.OBS_NATIVE), n,
                     seed=13, task_embedding=task)
    engs = [flat, full, nat]
    if wrapper:
        for e in engs:
            e.set_wrapper(wrapper_config(wrapper, heal_bonus_weight=0.03))
    for e in engs:
        e.reset()
    for t in range(4):
        if t:
            a = flat.scripted_actions(900 + t)
            for e in engs:
                e.step(a)
        ex = nat.expand_obs()
        torch.cuda.synchronize()
        d1 = (flat.obs != full.obs).nonzero()
        d2 = (ex != full.obs).nonzero()
        print(wrapper, "t", t, "flat!=full", d1.shape[0], d1[:3].tolist(), "nat!=full", d2.shape[0], d2[:3].tolist(),
              flush=True)
        if d1.shape[0]:
            e_, a_, k_ = d1[0].tolist()
            print("  flat", flat.obs[e_, a_, k_ - 2:k_ + 4].tolist(), "full", full.obs[e_, a_, k_ - 2:k_ + 4].tolist())
    for e in engs:
        e.close()

# chunk-mapped buffer reuse: allocate, fill, check, free, over and over (small buffers too)
from nmmo_amd import devmem  # noqa: E402

devmem.MIN_BYTES = 4 << 20
bad = 0
for it in range(12):
    bufs = [devmem.empty(((8 + 7 * k + it) << 18,), torch.float32, torch.device("cuda", 0)) for k in range(4)]
    for k, b in enumerate(bufs):
        b.fill_(float(it * 10 + k))
    torch.cuda.synchronize()
    for k, b in enumerate(bufs):
        if not bool((b == float(it * 10 + k)).all()):
            bad += 1
            print("vmm reuse: iteration", it, "buffer", k, "ptr", hex(b.data_ptr()), "wrong content", flush=True)
    del bufs, b
    devmem.release_pending()
print("vmm reuse check done, bad buffers:", bad, flush=True)
