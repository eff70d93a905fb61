"""Debug: first policy mismatch GPU vs oracle after reset (prints differing agents/heads)."""
import sys

import numpy as np
import torch

sys.path.insert(0, ".")
from nmmo_amd.config import Config  # noqa: E402
from nmmo_amd.engine import NmmoEngine  # noqa: E402
from oracle.oracle import OracleEnvs  # noqa: E402

preset = sys.argv[1] if len(sys.argv) > 1 else "C3"
cfg = Config.preset(preset, MAP_N=8, early_stop_agent_num=8)
n = int(sys.argv[2]) if len(sys.argv) > 2 else 6
task = (np.arange(2048) % 97 / 97.0 - 0.5).astype(np.float16)
eng = NmmoEngine(cfg, n, seed=11, task_embedding=task)
orc = OracleEnvs(cfg, n, seed=11, task_embedding=task)
eng.reset()
orc.reset()
a = orc.scripted_actions(1000)
g = eng.scripted_actions(1000).cpu().numpy()
bad = np.argwhere(a != g)
print("n mismatches", len(bad))
for e, p, h in bad[:20]:
    print(f"env {e} agent {p} head {h}: gpu {g[e, p, h]} oracle {a[e, p, h]}")
for rep in range(5):
    g2 = eng.scripted_actions(1000).cpu().numpy()
    print("repeat", rep, "mismatches vs oracle", int((g2 != a).sum()), "vs first gpu", int((g2 != g).sum()))
from nmmo_amd import abi  # noqa: E402
from oracle.oracle import split_state  # noqa: E402

st = split_state(orc.get_state(), n, orc.S, orc.P)
F = abi.F
for e, p, h in bad[:3]:
    ent = st["ent"][e]
    r, c = ent[F["row"], p], ent[F["col"], p]
    alive = ent[F["alive"]] == 1
    rows = ent[F["ds_row"]]
    cand = [s for s in range(orc.S) if alive[s] and max(abs(ent[F["row"], s] - r), abs(ent[F["col"], s] - c)) <= 7]
    cand.sort(key=lambda s: rows[s])
    print("agent", p, "at", r, c, "row", rows[p])
    for i, s in enumerate(cand[:100]):
        d = max(abs(ent[F["row"], s] - r), abs(ent[F["col"], s] - c))
        print(f"  vis {i}: slot {s} row {rows[s]} d {d} time_alive {ent[F['time_alive'], s]} pos {ent[F['row'], s]},{ent[F['col'], s]}")
