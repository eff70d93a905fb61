"""Throughput of the GPU experience storage kernels at the reference's
training batch (config.yaml train: batch_size 32768, batch_rows 128, bptt_horizon 8) fed by C4
rollouts (1024 envs x 128 agents per recv): store (flat copy / native expand-on-store), the
(env_id, step) sort, the advantage recurrence and the minibatch obs gather. HIP events on the
current stream. Prints one JSON line."""

import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import torch

    from nmmo_amd import abi
    from nmmo_amd.config import Config
    from nmmo_amd.engine import NmmoEngine
    from nmmo_amd.storage import DeviceExperience

    envs = int(os.environ.get("ENVS", "256"))
    B, rows, bptt = 32768, 128, 8
    out = {}
    for kind in ("flat", "native"):
        cfg = Config.preset("C4", early_stop_agent_num=8,
                            obs_layout=abi.OBS_NATIVE if kind == "native" else abi.OBS_FLAT)
        eng = NmmoEngine(cfg, envs, seed=1)
        n = envs * eng.P
        x = DeviceExperience(B, eng.obs_elems, n)
        eng.reset()
        eng.step(eng.scripted_actions(1))
        lp = torch.randn(n, device="cuda")
        v = torch.randn(n, device="cuda")
        mask = eng.mask.view(-1).clone()
        alive = int(mask.sum().item())
        act = eng.actions.view(n, 12)

        def store(step):
            x.store(eng.obs, eng.rew.view(-1), eng.term.view(-1), mask, act, lp, v, step,
                    engine=eng if kind == "native" else None)

        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        times, stored = [], 0
        for it in range(6):
            x.reset()
            torch.cuda.synchronize()
            e0.record()
            k = 0
            while True:  # fill the batch like evaluate(): one store per recv
                k += 1
                store(k)
                if k * alive >= B + 1:
                    break
            e1.record()
            torch.cuda.synchronize()
            if it:
                times.append(e0.elapsed_time(e1))
            stored = x.ptr
        ms = sum(times) / len(times)
        # bytes per stored row: obs row written + source read (flat row or native row + 1/16 Market)
        src = eng.obs_elems * 4 if kind == "flat" else abi.NATIVE_ROW_BYTES + abi.NATIVE_MARKET_BYTES / 16
        byts = stored * (eng.obs_elems * 4 + src)
        out[f"store_{kind}"] = {"ms_per_batch": round(ms, 4), "rows": stored, "GB/s": round(byts / ms / 1e6, 1)}
        eng.close()
    e0.record()
    idxs = x.sort()
    e1.record()
    torch.cuda.synchronize()
    out["sort_ms"] = round(e0.elapsed_time(e1), 4)
    e0.record()
    adv = x.advantages(idxs, 0.99, 0.95)
    e1.record()
    torch.cuda.synchronize()
    out["gae_ms"] = round(e0.elapsed_time(e1), 4)
    b = x.batch(idxs, adv, rows, bptt)
    e0.record()
    for mb in range(b["num_minibatches"]):
        x.gather(x.obs, b["b_idxs"][mb])
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1)
    out["gather_obs"] = {"ms_per_epoch": round(ms, 4),
                         "GB/s": round(2 * B * x.obs_elems * 4 / ms / 1e6, 1)}
    out["config"] = {"batch_size": B, "batch_rows": rows, "bptt_horizon": bptt, "envs_per_recv": envs}
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
