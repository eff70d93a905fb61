"""Diagnostic: the host cost of posting RCCL point-to-point ops through torch.distributed
(batch_isend_irecv), the learner gather's per-step transfer posting (nmmo_amd.distributed
WireExchange._p2p). One GPU: world size 1, every op a send to / receive from the rank itself in
one group (RCCL allows self P2P inside a group). Prints JSON: host microseconds per
batch_isend_irecv call and per op for batches of 2..32 ops of 1 MB. Launch with
torch.distributed.run --nproc-per-node 1 (127.0.0.1)."""
import json
import os
import time

import torch
import torch.distributed as dist


def main():
    torch.cuda.set_device(0)
    dev = torch.device("cuda", 0)
    dist.init_process_group("nccl", device_id=dev)
    out = {}
    bufs = [torch.zeros(1 << 20, dtype=torch.uint8, device=dev) for _ in range(32)]
    recv = [torch.empty(1 << 20, dtype=torch.uint8, device=dev) for _ in range(32)]
    for n_pairs in (1, 2, 4, 8, 16):
        ops = []
        for k in range(n_pairs):
            ops += [dist.P2POp(dist.isend, bufs[k], 0), dist.P2POp(dist.irecv, recv[k], 0)]
        for _ in range(5):
            for q in dist.batch_isend_irecv(ops):
                q.wait()
        torch.cuda.synchronize()
        reps = 50
        t0 = time.perf_counter()
        for _ in range(reps):
            for q in dist.batch_isend_irecv(ops):
                q.wait()
        host = (time.perf_counter() - t0) / reps
        torch.cuda.synchronize()
        wall = (time.perf_counter() - t0) / reps
        out[str(2 * n_pairs)] = {"host_us_per_call": round(host * 1e6, 1), "host_us_per_op": round(host * 1e6 / (2 * n_pairs), 2),
                                 "wall_us_per_call": round(wall * 1e6, 1)}
    print(json.dumps(out), flush=True)
    dist.destroy_process_group()


if __name__ == "__main__":
    os.environ.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    main()
