"""Diagnostic: C4 flat, one engine of 1,024 envs vs two engines of 512 on two streams
(graph-replayed, same process): step time."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from nmmo_amd.config import Config  # noqa: E402
from nmmo_amd.engine import NmmoEngine  # noqa: E402

cfg = Config.preset("C4", early_stop_agent_num=8)
dev = torch.device("cuda", 0)


def build(parts, n=1024):
    engs = [NmmoEngine(cfg, n // parts, seed=1, device=dev, env_index_base=i * (n // parts)) for i in range(parts)]
    for e in engs:
        e.reset()
    ids = np.arange(n // parts)
    for k in range(32):
        for i, e in enumerate(engs):
            e.end_episodes((ids + i * (n // parts)) % 32 == k)
            e.scripted_actions(7)
            e.step(write_obs=False)
    streams = [torch.cuda.Stream(device=dev) for _ in engs]
    graphs = []
    for e, s in zip(engs, streams):
        with torch.cuda.stream(s):
            for _ in range(3):
                e.scripted_actions(7)
                e.step()
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g, stream=s):
                for _ in range(10):
                    e.scripted_actions(7)
                    e.step()
            graphs.append(g)
    torch.cuda.synchronize()
    return engs, streams, graphs


def run(engs, streams, graphs, reps=20):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        for g, s in zip(graphs, streams):
            with torch.cuda.stream(s):
                g.replay()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / (reps * 10) * 1e3


for parts in (1, 2, 1, 2, 4):
    engs, streams, graphs = build(parts)
    ms = run(engs, streams, graphs)
    print(f"parts={parts}: {ms:.4f} ms/step")
    for e in engs:
        e.close()
    del engs, graphs
    torch.cuda.empty_cache()
