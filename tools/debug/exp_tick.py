import sys, os, torch
sys.path.insert(0, os.getcwd())
from nmmo_amd import abi
from nmmo_amd.config import Config
from nmmo_amd.engine import NmmoEngine
cfg = Config.preset(sys.argv[1], early_stop_agent_num=8, obs_layout=abi.OBS_NONE)
n = int(sys.argv[2])
eng = NmmoEngine(cfg, n, seed=1)
eng.reset()
for t in range(50):
    eng.scripted_actions(t); eng.step()
torch.cuda.synchronize()
def graph_of(fn, k=20):
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for _ in range(k): fn()
    return g
def t_graph(g, reps=10, k=20):
    g.replay(); torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(reps): g.replay()
    b.record(); torch.cuda.synchronize()
    return a.elapsed_time(b) / (reps * k) * 1e3
cnt = [0]
def pol_tick():
    cnt[0] += 1
    eng.scripted_actions(12345); eng.step()
def pol_only():
    eng.scripted_actions(12345)
gp = graph_of(pol_tick); gt = graph_of(eng.step); go = graph_of(pol_only)
print("graph policy+tick us", t_graph(gp))
print("graph tick only (stale actions) us", t_graph(gt))
print("graph policy only us", t_graph(go))
print("graph policy+tick us", t_graph(gp))
eng.actions.zero_()
print("graph tick only, zero actions us", t_graph(gt))
