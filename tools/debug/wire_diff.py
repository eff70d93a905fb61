"""Locate the first bytes where nmmo_wire_pack and oracle/wire.py disagree (diagnostic)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import numpy as np  # noqa: E402

from tests.test_gpu_wire import _engine  # noqa: E402
from nmmo_amd import wire  # noqa: E402
from oracle import wire as ow  # noqa: E402

eng = _engine(3, seed=21)
eng.reset()
for t in range(45):
    if t == 20:
        eng.end_episodes(np.array([0, 1, 0], bool))
    eng.scripted_actions(500 + t)
    eng.step()
    import torch
    w = wire.pack(eng, out=torch.full((wire.max_bytes(3, eng.P),), 0xAB, dtype=torch.uint8, device='cuda'))
    total = wire.total_bytes(w)
    nat = eng.obs.cpu().numpy()
    ref = ow.pack(nat, eng.P)
    g = w[:total].cpu().numpy()
    if total == ref.nbytes and np.array_equal(g, ref):
        continue
    print("tick", t, "total", total, ref.nbytes)
    n, P = 3, eng.P
    H = ow.header_bytes(n, P)
    bad = np.flatnonzero(g[:min(len(g), len(ref))] != ref[:min(len(g), len(ref))])
    print("n bad", len(bad), "first", bad[:20], "H", H)
    env_off = ref[8:8 + 8 * n].copy().view(np.int64)
    cnt, nm = ow.counts(nat, P)
    for b in bad[:10]:
        if b < H:
            print("header byte", b)
            continue
        e = int(np.searchsorted(env_off, b, side="right") - 1)
        pos = int(env_off[e])
        for a in range(P):
            rb = ow.record_bytes(int(cnt[e, a]))
            if pos <= b < pos + rb:
                c = int(cnt[e, a])
                print(f"env {e} agent {a} rec byte {b - pos} of {rb} nv {c & 127} ninv {(c >> 7) & 15} gpu {g[b]} ref {ref[b]}")
                break
            pos += rb
        else:
            print(f"env {e} market byte {b - pos} nm {nm[e]} gpu {g[b]} ref {ref[b]}")
    break
