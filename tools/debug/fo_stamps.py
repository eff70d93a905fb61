"""Diagnostic: per-section s_memtime stamps of the flat obs kernel (flat_obs.hip, NMMO_FO_STAMPS=1
variant: python tools/debug/variants.py fost=-DNMMO_FO_STAMPS=1). One C4 batch (512 envs),
staggered, warmed up; then per launch the stamps of every alive row are read and summarised:
per section the median / p90 cycles, and the row span (first stamp to last).

  NMMO_LIB=nmmo_amd/lib/libnmmo_hip_fost.so NMMO_ALLOW_STALE=1 python tools/debug/fo_stamps.py
"""
import ctypes
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)

NAMES = ["setup+compaction", "sections", "chunks 0-1", "Buy-only chunks", "tail chunks", "Entity", "Inventory",
         "Market", "Task", "Tile", "state"]


def main():
    import torch

    import bench
    from nmmo_amd import abi
    from nmmo_amd._native import lib
    from nmmo_amd.config import Config
    from nmmo_amd.engine import NmmoEngine

    envs, steps = 512, int(os.environ.get("FO_STEPS", "4"))
    dev = torch.device("cuda:0")
    cfg = Config.preset("C4", early_stop_agent_num=8, obs_layout=abi.OBS_FLAT)
    eng = NmmoEngine(cfg, envs, seed=1, device=dev, task_embedding=bench._task_embedding())
    eng.reset()
    pseed = 1_000_003
    bench._stagger([eng], 64, envs, 0, pseed)
    for _ in range(30):
        eng.scripted_actions(pseed)
        eng.step()
    torch.cuda.synchronize()
    f = lib().nmmo_debug_fo_stamps
    f.argtypes = [ctypes.c_void_p, ctypes.c_size_t]
    n = envs * eng.P
    buf = np.zeros((1 << 17, len(NAMES) + 1), dtype=np.uint64)
    f(buf.ctypes.data, buf.nbytes)  # clear
    fw = lib().nmmo_debug_fo_wave_stamps
    fw.argtypes = [ctypes.c_void_p, ctypes.c_size_t]
    wbuf = np.zeros((1 << 15, 6), dtype=np.uint64)
    fw(wbuf.ctypes.data, wbuf.nbytes)
    spans, secs, waves = [], [], []
    for _ in range(steps):
        eng.scripted_actions(pseed)
        eng.step()
        torch.cuda.synchronize()
        f(buf.ctypes.data, buf.nbytes)
        fw(wbuf.ctypes.data, wbuf.nbytes)
        w = wbuf[: envs * ((eng.P + 15) // 16) * 4].astype(np.int64)
        waves.append(w[w[:, 0] != 0])
        st = buf[:n].astype(np.int64)
        alive = st[:, 0] != 0
        st = st[alive]
        d = np.diff(st, axis=1)
        secs.append(d)
        spans.append(st[:, -1] - st[:, 0])
    d = np.concatenate(secs)
    span = np.concatenate(spans)
    print(f"alive rows per launch {d.shape[0] // steps}; row span cycles: median {np.median(span):.0f} "
          f"p90 {np.percentile(span, 90):.0f} mean {span.mean():.0f}")
    w = np.concatenate(waves)
    t0 = w[:, 0]
    print(f"waves {w.shape[0] // steps} per launch; per wave cycles (median / p90 / mean):")
    for k, nm in enumerate(["ao_stage", "stage windows", "to loop", "agent loop"]):
        x = w[:, k + 1] - w[:, k]
        print(f"  {nm:14s} {np.median(x):8.0f} {np.percentile(x, 90):8.0f} {x.mean():8.0f}")
    life = w[:, 4] - t0
    print(f"  {'lifetime':14s} {np.median(life):8.0f} {np.percentile(life, 90):8.0f} {life.mean():8.0f}; "
          f"rows per wave {np.mean(w[:, 5] >> 32):.2f}")
    tot = d.mean(0).sum()
    for k, nm in enumerate(NAMES):
        print(f"  {nm:18s} median {np.median(d[:, k]):7.0f}  p90 {np.percentile(d[:, k], 90):7.0f}  "
              f"mean {d[:, k].mean():7.0f}  share {d[:, k].mean() / tot:5.1%}")


if __name__ == "__main__":
    main()
