"""Ad hoc: grid sub-phase cycles (needs a stamps build with STAMP 14/15 inside the grid)."""
import ctypes, os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
os.environ["NMMO_LIB"] = os.path.join(ROOT, "nmmo_amd", "lib", "libnmmo_hip_stamps.so")
import numpy as np, torch
from nmmo_amd import _native, abi
from nmmo_amd.config import Config
from nmmo_amd.engine import NmmoEngine
envs = int(sys.argv[1]) if len(sys.argv) > 1 else 1024
cfg = Config.preset(sys.argv[2] if len(sys.argv) > 2 else "C3", early_stop_agent_num=8, obs_layout=abi.OBS_NONE)
eng = NmmoEngine(cfg, envs, seed=1); eng.reset()
L = _native.lib(); L.nmmo_debug_read_stamps.argtypes = [ctypes.c_void_p, ctypes.c_int]
out = []
for t in range(50):
    eng.scripted_actions(1000 + t); eng.step(); torch.cuda.synchronize()
    if t >= 40:
        buf = np.zeros(4096 * 16, np.uint64)
        L.nmmo_debug_read_stamps(buf.ctypes.data_as(ctypes.c_void_p), buf.size)
        f = buf.reshape(4096, 16)[:min(envs, 4096)].astype(np.int64)
        ok = (f[:, 2] > 0) & (f[:, 11] > f[:, 0])
        f = f[ok]
        out.append(np.stack([f[:, 14] - f[:, 7], f[:, 15] - f[:, 14], f[:, 8] - f[:, 15], f[:, 1] - f[:, 0], f[:, 11] - f[:, 0]], 1))
o = np.concatenate(out)
for i, n in enumerate(["A", "B", "C", "load+rowslot", "total"]):
    print(f"envs={envs} {n:20s} median {np.median(o[:, i]):8.0f} p90 {np.percentile(o[:, i], 90):8.0f}")
