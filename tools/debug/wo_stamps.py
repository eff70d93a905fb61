"""Diagnostic: per-section s_memtime stamps of the wire records kernel (wire_obs.hip,
NMMO_WO_STAMPS=1 variant: python tools/debug/variants.py wost=-DNMMO_WO_STAMPS=1). One C5 batch
(512 envs, wire layout), staggered, warmed up; per launch the stamps of every record and every
wave are read: per section the median / p90 cycles, per wave its phases.

  NMMO_LIB=nmmo_amd/lib/libnmmo_hip_wost.so NMMO_ALLOW_STALE=1 python tools/debug/wo_stamps.py
"""
import ctypes
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)

SECTIONS = ["window materials", "compaction", "ActionTargets sections", "mask stream", "record stores"]
PHASES = ["prologue", "windows", "record loop", "tail (listings, table)"]


def main():
    import torch

    import bench
    from nmmo_amd import abi
    from nmmo_amd._native import lib
    from nmmo_amd.config import Config
    from nmmo_amd.engine import NmmoEngine

    envs, steps = 512, int(os.environ.get("WO_STEPS", "4"))
    dev = torch.device("cuda:0")
    cfg = Config.preset("C4", early_stop_agent_num=8, obs_layout=abi.OBS_WIRE)
    eng = NmmoEngine(cfg, envs, seed=1, device=dev)
    eng.reset()
    pseed = 1_000_003
    bench._stagger([eng], 64, envs, 0, pseed)
    for _ in range(30):
        eng.scripted_actions(pseed)
        eng.step()
    torch.cuda.synchronize()
    f = lib().nmmo_debug_wo_stamps
    f.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_void_p, ctypes.c_size_t]
    rbuf = np.zeros((1 << 17, 6), dtype=np.uint64)
    wbuf = np.zeros((1 << 15, 6), dtype=np.uint64)
    f(rbuf.ctypes.data, rbuf.nbytes, wbuf.ctypes.data, wbuf.nbytes)  # clear
    recs, waves = [], []
    for _ in range(steps):
        eng.scripted_actions(pseed)
        eng.step()
        torch.cuda.synchronize()
        f(rbuf.ctypes.data, rbuf.nbytes, wbuf.ctypes.data, wbuf.nbytes)
        r = rbuf[: envs * eng.P].astype(np.int64)
        recs.append(np.diff(r[r[:, 0] != 0], axis=1))
        w = wbuf[: envs * ((eng.P + 15) // 16) * 4].astype(np.int64)
        waves.append(w[w[:, 0] != 0])
    d = np.concatenate(recs)
    w = np.concatenate(waves)
    print(f"records per launch {d.shape[0] // steps}; record span cycles: median {np.median(d.sum(1)):.0f} "
          f"p90 {np.percentile(d.sum(1), 90):.0f}")
    tot = d.mean(0).sum()
    for k, nm in enumerate(SECTIONS):
        print(f"  {nm:24s} median {np.median(d[:, k]):7.0f}  p90 {np.percentile(d[:, k], 90):7.0f}  "
              f"share {100 * d[:, k].mean() / tot:5.1f}%")
    print(f"waves {w.shape[0] // steps} per launch; per wave cycles (median / p90 / mean):")
    for k, nm in enumerate(PHASES):
        x = w[:, k + 1] - w[:, k]
        print(f"  {nm:22s} {np.median(x):8.0f} {np.percentile(x, 90):8.0f} {x.mean():8.0f}")
    life = w[:, 4] - w[:, 0]
    print(f"  {'lifetime':22s} {np.median(life):8.0f} {np.percentile(life, 90):8.0f} {life.mean():8.0f}; "
          f"records per wave {np.mean(w[:, 5] >> 32):.2f}")
    eng.close()


if __name__ == "__main__":
    main()
