"""Env sharding across GPUs (one process per GPU) and the learner gather.

SURVEY.md §8e: envs are independent, so each rank steps a contiguous block of envs with no
collective on the data path; the only exchange is returning batched outputs to a single learner
(rank 0) when the trainer is centralised (BASELINE config 5). Global env indices
(env_index_base = rank * n_local) key every random stream, so a sharded run is env-for-env
identical to a single-GPU run of the same total envs (tests/test_distributed.py checks this on
gloo, tests/test_gpu_multirank.py on the GPU).

The reference has no collective at all (single-GPU learner fed by pufferlib worker processes,
clean_pufferl.py:106-114); this module replaces the worker-process IPC of pool.recv()/send()
(:293, :357) with torch.distributed (RCCL over xGMI on MI355X, gloo on CPU).

The learner gather moves observations as wire buffers (SPEC §8c, nmmo_amd.wire): every rank's
handles write them straight from the state (obs_layout OBS_WIRE), ~0.8 KB per agent in the realm
instead of 9,552 B native / 95,948 B flat. `WireExchange` is the transfer protocol and
`WireGather` the C5 step built on it.
"""

from __future__ import annotations

import os

import torch
import torch.distributed as dist


def shard(total_envs: int, world: int, rank: int):
    """Contiguous env block of `rank`: (env_index_base, n_local). Requires an even split."""
    if total_envs % world:
        raise ValueError(f"{total_envs} envs do not split evenly over {world} ranks")
    n = total_envs // world
    return rank * n, n


_COMMS = {}  # (world, rank, device index) -> the library's RCCL communicator (one per process)


def native_comm(world: int, rank: int, device):
    """This process's RCCL communicator for nmmo_p2p_group (created once, collectively: every rank
    calls this; rank 0's unique id reaches the others through a torch.distributed broadcast)."""
    import ctypes

    from . import abi
    from ._native import check, lib

    key = (world, rank, torch.device(device).index)
    if key in _COMMS:
        return _COMMS[key]
    check(lib().nmmo_p2p_load(os.path.join(os.path.dirname(torch.__file__), "lib", "librccl.so").encode()),
          "nmmo_p2p_load")
    idt = torch.zeros(abi.P2P_ID_BYTES, dtype=torch.uint8, device=device)
    if rank == 0:
        buf = (ctypes.c_uint8 * abi.P2P_ID_BYTES)()
        check(lib().nmmo_p2p_unique_id(buf), "nmmo_p2p_unique_id")
        idt.copy_(torch.tensor(list(bytes(buf)), dtype=torch.uint8))
    if world > 1:
        dist.broadcast(idt, src=0)
    ident = bytes(idt.cpu().tolist())
    comm = ctypes.c_void_p()
    check(lib().nmmo_p2p_init(ident, world, rank, ctypes.byref(comm)), "nmmo_p2p_init")
    _COMMS[key] = comm
    return comm


def env_shares(total_envs: int, world: int, root_envs: int | None = None, granule: int = 1):
    """Env counts per rank for a learner gather (BASELINE config 5): `root_envs` on rank 0 (the
    learner, which also validates and stores every peer's buffers each step, so it steps fewer
    envs of its own; None = an even split) and the rest over ranks 1..world-1 as evenly as
    possible, every count a multiple of `granule` (the env batches per rank). Contiguous blocks in
    rank order: rank r's env_index_base is the sum of the counts before it."""
    if world == 1:
        return [total_envs]
    if root_envs is None:
        if total_envs % world:
            raise ValueError(f"{total_envs} envs do not split evenly over {world} ranks")
        root_envs = total_envs // world
    rest = total_envs - root_envs
    if root_envs < granule or root_envs % granule or rest % granule:
        raise ValueError(f"root_envs {root_envs} and the {rest} other envs must be positive multiples of {granule}")
    units, extra = divmod(rest // granule, world - 1)
    if units == 0:
        raise ValueError(f"{rest} envs cannot give each of {world - 1} peers {granule}")
    return [root_envs] + [(units + (1 if r < extra else 0)) * granule for r in range(world - 1)]


def gather_to_learner(t: torch.Tensor, dst: int = 0):
    """Gather the rank-local batch `t` ([n_local, ...]) to rank `dst` as [world*n_local, ...].
    Each peer -> root transfer is a point-to-point xGMI link under RCCL (no ring)."""
    world = dist.get_world_size()
    if world == 1:
        return t
    if dist.get_rank() == dst:
        bufs = [torch.empty_like(t) for _ in range(world)]
        dist.gather(t.contiguous(), gather_list=bufs, dst=dst)
        return torch.cat(bufs, 0)
    dist.gather(t.contiguous(), dst=dst)
    return None


def scatter_from_learner(full, like: torch.Tensor, src: int = 0) -> torch.Tensor:
    """Scatter [world*n_local, ...] actions from `src` back to every rank's [n_local, ...]."""
    world = dist.get_world_size()
    if world == 1:
        return full
    out = torch.empty_like(like)
    if dist.get_rank() == src:
        chunks = list(full.contiguous().chunk(world, 0))
        dist.scatter(out, scatter_list=chunks, src=src)
    else:
        dist.scatter(out, src=src)
    return out


class WireExchange:
    """Transfer protocol of the learner gather: every rank's `n_bufs` wire buffers (one per env
    batch, SPEC §8c) and their fixed-size companions (`smalls`: reward / dones / mask) reach rank
    `dst` each step, over point-to-point sends (RCCL over xGMI: each peer uses its own link to
    the root; no ring, no collective on the payload).

    A wire buffer's size is known only on the device once its step has run, and a receive must
    be posted with its exact size, so the protocol runs a step behind the compute:
      sizes(t)   every sender's totals (8 B per buffer, read on the device from the headers)
                 reach the root on the comm stream, and are copied into pinned host memory;
      payload(t) posted after sizes(t) has landed (the host waits for that copy's event only, so
                 the caller posts payload(t - 1) after queueing step t: step t computes while
                 t - 1's buffers move); each receive is exactly the announced size.
    No `.item()`, no stream or device synchronisation on the data path. Buffers handed to
    sizes(t) / payload(t) must stay untouched until `done(t)` (an event on the comm stream).
    Ring slot k = t % ring indexes the per-step state.

    Each rank's sizes row carries one more word: its tick fault word of step t (nmmo_fault_into;
    0 = none). payload(t) raises on a rank whose own word is set and on the root for any rank's
    word, and likewise for an announced size outside [16, capacity] — on the sender as on the root,
    both before posting any transfer of step t, so neither side waits for a transfer the other
    will never post.

    On CPU tensors (gloo, tests) every call is synchronous. With gloo and CUDA tensors (the
    one-GPU rehearsal of a multi-rank run) transfers are staged through the host."""

    def __init__(self, world: int, rank: int, n_bufs: int, recv_caps, small_bytes, device, dst: int = 0,
                 ring: int = 3, backend: str | None = None):
        """recv_caps / small_bytes: per rank a list of n_bufs sizes (each rank's buffer j may hold a
        different env count), or one list of n_bufs sizes shared by every rank."""
        self.world, self.rank, self.dst, self.ring = world, rank, dst, ring
        self.n_bufs = n_bufs
        if recv_caps and not isinstance(recv_caps[0], (list, tuple)):
            recv_caps = [list(recv_caps)] * world
        if small_bytes and not isinstance(small_bytes[0], (list, tuple)):
            small_bytes = [list(small_bytes)] * world
        self.device = torch.device(device)
        self.cuda = self.device.type == "cuda"
        self.staged = (backend or (dist.get_backend() if world > 1 else "nccl")) == "gloo" and self.cuda
        d = self.device
        # [.., n_bufs] = the rank's tick fault word of the step
        self.sizes = torch.zeros((ring, world, n_bufs + 1), dtype=torch.int64, device=d)
        self.sizes_host = torch.zeros((ring, world, n_bufs + 1), dtype=torch.int64, pin_memory=self.cuda)
        self.caps = [[int(c) for c in row] for row in recv_caps]  # [rank][buffer] capacity bound
        self.comm = torch.cuda.Stream(device=d) if self.cuda else None
        self._sized = [None] * ring
        self._done = [None] * ring
        self.peers = [r for r in range(world) if r != dst]
        # RCCL groups posted natively (nmmo_p2p_group: ~1 us of host time per op instead of ~13.5
        # through batch_isend_irecv); NMMO_P2P=torch keeps torch.distributed's posting
        self._comm = None
        if world > 1 and self.cuda and not self.staged and os.environ.get("NMMO_P2P", "native") == "native":
            self._comm = native_comm(world, rank, d)
        self.recv_wire, self.recv_small = {}, {}
        if rank == dst:
            for r in self.peers:
                for j in range(n_bufs):
                    self.recv_wire[r, j] = torch.empty(int(recv_caps[r][j]), dtype=torch.uint8, device=d)
                    self.recv_small[r, j] = torch.empty(int(small_bytes[r][j]), dtype=torch.uint8, device=d)
        self.payload_bytes = 0  # wire bytes received by the root (all peers, all steps)
        self.wait_s = 0.0  # host seconds blocked on size rows (totals)

    # -- plumbing
    def _ctx(self):
        return torch.cuda.stream(self.comm) if self.cuda else _null()

    def _p2p(self, sends, recvs):
        """sends / recvs: [(tensor, peer)]; completes (stream-ordered on the comm stream with
        RCCL, synchronously with gloo)."""
        if not sends and not recvs:
            return
        if self.staged:  # gloo cannot read device memory: host copies, synchronously
            self.comm.synchronize()
            cs = [(t.cpu(), p) for t, p in sends]
            cr = [(torch.empty(t.shape, dtype=t.dtype), p) for t, p in recvs]
            reqs = [dist.isend(t, p) for t, p in cs] + [dist.irecv(t, p) for t, p in cr]
            for q in reqs:
                q.wait()
            with torch.cuda.stream(self.comm):
                for (t, _), (c, _) in zip(recvs, cr):
                    t.copy_(c)
            return
        if self._comm is not None:  # one RCCL group on the comm stream, enqueued (no host wait)
            import ctypes

            from . import abi
            from ._native import check, lib

            allops = [(t, p, 0) for t, p in sends] + [(t, p, 1) for t, p in recvs]
            arr = (abi.NmmoP2POp * len(allops))(*[abi.NmmoP2POp(t.data_ptr(), t.numel() * t.element_size(), p, r)
                                                  for t, p, r in allops])
            check(lib().nmmo_p2p_group(self._comm, arr, len(allops), ctypes.c_void_p(self.comm.cuda_stream)),
                  "nmmo_p2p_group")
            return
        ops = [dist.P2POp(dist.isend, t, p) for t, p in sends] + [dist.P2POp(dist.irecv, t, p) for t, p in recvs]
        with self._ctx():
            for q in dist.batch_isend_irecv(ops):
                q.wait()

    # -- protocol
    def post_sizes(self, t: int, wires, ready=(), fault=None):
        """Step t's totals: the sender's (or the root's own) buffers' first int64 into
        sizes[k][rank]; the peers' totals into the root's sizes[k]. `ready`: events the comm
        stream waits for (the compute that wrote `wires`); `fault`: a device int32 [1] holding
        this rank's tick fault word of step t (zeroed here once copied), or None."""
        k = t % self.ring
        # (sizes[k] / sizes_host[k] of step t - ring were read by then: the device reads are
        # earlier on the comm stream, the host read came before this call)
        with self._ctx():
            if self.cuda:
                for ev in ready:
                    self.comm.wait_event(ev)
                _sizes_row(wires, fault, self.sizes[k, self.rank], self.comm)  # one launch (nmmo_sizes_row)
            else:
                for j, w in enumerate(wires):
                    self.sizes[k, self.rank, j].copy_(w[:8].view(torch.int64)[0])
                if fault is None:
                    self.sizes[k, self.rank, self.n_bufs].zero_()
                else:
                    self.sizes[k, self.rank, self.n_bufs].copy_(fault[0])
                    fault.zero_()
        if self.world > 1:
            if self.rank == self.dst:
                self._p2p([], [(self.sizes[k, r], r) for r in self.peers])
            else:
                self._p2p([(self.sizes[k, self.rank], self.dst)], [])
        with self._ctx():
            self.sizes_host[k].copy_(self.sizes[k], non_blocking=self.cuda)
            if self.cuda:
                ev = torch.cuda.Event()
                ev.record(self.comm)
                self._sized[k] = ev

    def totals(self, t: int):
        """Step t's announced totals on the host ([rank][buffer], + the fault word), once sizes(t)
        has reached pinned memory (host wait on that copy only)."""
        k = t % self.ring
        if self.cuda and self._sized[k] is not None:
            import time

            w0 = time.perf_counter()
            self._sized[k].synchronize()
            self.wait_s += time.perf_counter() - w0
        return self.sizes_host[k].tolist()

    def post_payload(self, t: int, wires, smalls, recv_into=None):
        """Step t's buffers: exactly the announced bytes of every wire buffer + its smalls.
        Returns, on the root, {(rank, j): (wire bytes, small)} with the root's own buffers in
        place (no self-copy); {} elsewhere. recv_into (root): {(rank, j): uint8 tensor} to receive
        those buffers into instead of the exchange's own receive buffers (the learner's record
        arena). Everything is enqueued on the comm stream."""
        tot = self.totals(t)
        # the same checks on both ends of every transfer, before any of step t's transfers is posted
        ranks = range(self.world) if self.rank == self.dst else [self.rank]
        for r in ranks:
            if tot[r][self.n_bufs]:
                from .engine import TickFault

                raise TickFault(int(tot[r][self.n_bufs]), f"learner gather, rank {r}, step {t}")
            for j in range(self.n_bufs):
                n = int(tot[r][j])
                if n < 16 or n > self.caps[r][j]:
                    raise RuntimeError(f"rank {r} buffer {j} announces {n} B at step {t} (capacity {self.caps[r][j]})")
        got = {}
        if self.rank == self.dst:
            for j in range(self.n_bufs):
                got[self.rank, j] = (wires[j][:tot[self.rank][j]], smalls[j])
            recvs = []
            for r in self.peers:
                for j in range(self.n_bufs):
                    n = int(tot[r][j])
                    dst = self.recv_wire[r, j] if recv_into is None or (r, j) not in recv_into else recv_into[r, j]
                    w, s = dst[:n], self.recv_small[r, j]
                    recvs += [(w, r), (s, r)]
                    got[r, j] = (w, s)
                    self.payload_bytes += n
            self._p2p([], recvs)
        elif self.world > 1:
            sends = []
            for j in range(self.n_bufs):
                sends += [(wires[j][:int(tot[self.rank][j])], self.dst), (smalls[j], self.dst)]
            self._p2p(sends, [])
        return got

    def mark_done(self, t: int):
        """Everything enqueued on the comm stream for step t so far (its payload and whatever
        the caller consumed it with) is what done(t) waits for."""
        if self.cuda:
            ev = torch.cuda.Event()
            ev.record(self.comm)
            self._done[t % self.ring] = ev

    def done(self, t: int):
        return self._done[t % self.ring]


def _sizes_row(wires, fault, row, stream):
    """row[j] = wires[j]'s announced total, row[n] = *fault (then cleared): nmmo_sizes_row."""
    import ctypes

    from ._native import check, lib

    n = len(wires)
    ptrs = (ctypes.c_void_p * n)(*[w.data_ptr() for w in wires])
    check(lib().nmmo_sizes_row(ptrs, n, None if fault is None else ctypes.c_void_p(fault.data_ptr()),
                               ctypes.c_void_p(row.data_ptr()), ctypes.c_void_p(stream.cuda_stream)), "nmmo_sizes_row")


class _null:
    def __enter__(self):
        return self

    def __exit__(self, *a):
        return False


class WireGather:
    """BASELINE config 5's step on one rank: every env batch of this rank (an NmmoEngine with
    obs_layout OBS_WIRE on its own stream) runs the scripted policy + nmmo_step into a ring of
    wire buffers, and the learner gather (WireExchange) moves every rank's buffers + packed
    reward / term / trunc / mask into rank 0 one step behind, on a comm stream, so step t's
    transfer overlaps step t + 1's compute (reference: the recv -> store loop of
    clean_pufferl.py:293-346, fed here by every GPU of the node).

    Ranks may hold different env counts (`env_shares`: the learner root fewer, the peers the
    rest); every rank has the same number of batches and the same task table, and the root learns
    each rank's batch sizes once at construction. Global env ids are contiguous in rank order.

    On the root, each step's buffers are validated on the device (nmmo_wire_check: sizes,
    offsets, count words, record heads; `status` accumulates) — "delivered": every agent's
    observation landed, checked, in the learner's HBM, in the form the experience store decodes
    its kept rows from (nmmo_exp_store, wire input). decode=True additionally decodes every
    rank's buffers into the native layout (nmmo_wire_unpack, the full learner-ready tensor) on
    the comm stream. store=DeviceExperience (root; compact record storage) stores every step's
    learner rows (the agents in the realm) from every received buffer on the comm stream — the
    root's real work per step, clean_pufferl.py:331-346 — as a batch of its own (reset each step),
    with the check fused into the store's reservation pass (nmmo_exp_store_records_checked: a
    buffer that fails keeps no row), the peers' buffers received straight into their arena slots.
    on_step(t, got) (tests) runs on the root after step t's buffers landed, with the device
    synchronised: got = {(rank, batch): (wire bytes, smalls)}.

    The compute of each (batch, ring slot) is captured once in a hipGraph (graphs=True); with
    graphs=False, before_step(t, j, engine) (tests: per-env episode ends) runs on batch j's
    stream ahead of its step-t compute."""

    def __init__(self, engines, policy_seed: int, rank: int = 0, world: int = 1, decode: bool = False,
                 graphs: bool = True, ring: int = 3, on_step=None, backend: str | None = None,
                 before_step=None, store=None, rehearse: int = 0, phantom=None, rehearse_mode: str = "fill"):
        """rehearse = R > 0 (root, one GPU): the root also takes R phantom peers' buffers every
        step, so a one-GPU run carries the root's load of an N = world + R node. phantom: per batch
        j a (wire bytes, smalls, n_envs) snapshot of a peer's buffers (e.g. a rank of the node's
        peer share stepped beforehand); each phantom peer q "receives" that content every step:
        rehearse_mode "fill" stands in for the incoming transfers with write-only fills of the
        same bytes (the received data's HBM writes; the content sits in the record arena once,
        so the check and store read valid buffers in place), "copy" copies the snapshot into its
        arena slot every step (read + write: what a receive through an intermediate buffer costs).
        The phantoms are validated and stored like real peers (the xGMI links are not modelled)."""
        if before_step is not None and graphs:
            raise ValueError("before_step needs graphs=False")
        if rehearse_mode not in ("fill", "copy"):
            raise ValueError("rehearse_mode: fill or copy")
        self.before_step = before_step
        from . import abi, devmem
        from . import wire as nw

        self.engines = list(engines)
        self.rank, self.world, self.decode, self.on_step = rank, world, decode, on_step
        self.store = store if rank == 0 else None
        self._stored = torch.zeros((), dtype=torch.int64, device=engines[0].device)  # rows the root stored
        self.pseed = policy_seed
        e0 = self.engines[0]
        self.device = e0.device
        self.P = e0.P
        import numpy as np

        for e in self.engines:
            if e.config.obs_layout != abi.OBS_WIRE:
                raise ValueError("WireGather steps handles created with obs_layout OBS_WIRE")
            if not np.array_equal(e.task_table, e0.task_table):
                raise ValueError("WireGather: the batches' task tables differ (records decode with one table)")
        nb = len(self.engines)
        # every rank's batch sizes (the root sizes its receive buffers and places each buffer's
        # rows from them) and one task table for all (the root decodes every buffer with its own)
        mine = [e.n_envs for e in self.engines]
        self.counts = [mine]
        if world > 1:
            import zlib

            crc = zlib.crc32(np.ascontiguousarray(e0.task_table, np.float32).tobytes())
            sig = torch.tensor([nb, crc], dtype=torch.int64, device=self.device)
            lo, hi = sig.clone(), sig.clone()
            dist.all_reduce(lo, op=dist.ReduceOp.MIN)
            dist.all_reduce(hi, op=dist.ReduceOp.MAX)
            if not torch.equal(lo, hi):
                raise ValueError("WireGather: ranks differ in their number of env batches or task table (the root "
                                 "receives every rank's buffers and decodes them with its own table)")
            row = torch.zeros(world, nb, dtype=torch.int64, device=self.device)
            row[rank] = torch.tensor(mine, dtype=torch.int64)
            dist.all_reduce(row, op=dist.ReduceOp.SUM)
            self.counts = row.tolist()
        self.counts = [[int(c) for c in r] for r in self.counts]
        # global env id of (rank r, batch j)'s first env: contiguous blocks in rank order
        self.env_base = {}
        acc = 0
        for r in range(world):
            for j in range(nb):
                self.env_base[r, j] = acc
                acc += self.counts[r][j]
        self.ring = ring
        self.wires = [[e.obs] + [devmem.empty(tuple(e.obs.shape), torch.uint8, self.device) for _ in range(ring - 1)]
                      for e in self.engines]
        self.smalls = [[torch.zeros((e.n_envs, self.P, 8), dtype=torch.uint8, device=self.device) for _ in range(ring)]
                       for e in self.engines]
        caps = [[nw.max_bytes(c, self.P) for c in row] for row in self.counts]
        self.x = WireExchange(world, rank, nb, caps, [[c * self.P * 8 for c in row] for row in self.counts],
                              self.device, ring=ring, backend=backend)
        self.streams = [torch.cuda.Stream(device=self.device) for _ in self.engines]
        self.status = torch.zeros(1, dtype=torch.int32, device=self.device)
        # per ring slot: the first tick fault word of the step's batches (nmmo_fault_into), shipped
        # to the root with the step's sizes
        self.faults = torch.zeros((ring, 1), dtype=torch.int32, device=self.device)
        self._posted = -1  # the last step whose payload was posted
        self.native = None
        if decode and rank == 0:
            self.native = {(r, j): devmem.empty((self.counts[r][j], abi.native_env_bytes(self.P)), torch.uint8,
                                                self.device) for r in range(world) for j in range(nb)}
        self._zeros = self._acts = None
        self.rehearse = int(rehearse) if rank == 0 else 0
        self.rehearse_mode = rehearse_mode
        self._ph = []  # phantom peers' buffers: (key, arena slot or buffer, smalls, n_envs, expect)
        if self.rehearse:
            self._setup_phantoms(phantom, acc)
        self.graphs = None
        if graphs:
            self._capture()
        self.t = 0
        self.host_s = 0.0  # host seconds inside step() (WireExchange.totals' wait for step t - 1's sizes included)

    def _setup_phantoms(self, phantom, env0):
        """The rehearsal's phantom peers (see __init__): their content placed once, at the front of
        the record arena (fixed slots, so the store finds them in place every step), or in buffers
        of their own without a store. Phantom q's batch j takes global envs after the real ranks'."""
        from . import abi, devmem

        nb = len(self.engines)
        if phantom is None or len(phantom) != nb:
            raise ValueError("rehearse needs phantom = one (wire bytes, smalls, n_envs) per batch")
        d = self.device
        used = 0
        arena = self.store.arena if self.store is not None else None
        keys = [(self.world - 1 + q, j) for q in range(1, self.rehearse + 1) for j in range(nb)]
        self._rh_src = []
        sink = 0
        for (r, j) in keys:
            w0, sm0, n = phantom[j]
            w0 = w0.view(-1)
            tot = int(w0[:8].view(torch.int64)[0].item())
            if tot != w0.numel() or tot & 15:
                raise ValueError("phantom wire bytes must be one whole buffer (its announced total)")
            if arena is not None:
                base = (used + 15) & ~15
                if base + 16 + tot > arena.numel():
                    raise ValueError("the record arena cannot hold the phantom peers' buffers")
                w = arena[base + 16:base + 16 + tot]
                used = base + 16 + tot
            else:
                w = devmem.empty((tot,), torch.uint8, d)
            w.copy_(w0)
            sm = sm0.clone()
            expect = torch.tensor([tot], dtype=torch.int64, device=d)
            self._ph.append(((r, j), w, sm, int(n), expect))
            self._rh_src.append(w0.clone() if self.rehearse_mode == "copy" else None)
            sink += tot + sm.numel()
            self.env_base[r, j] = env0
            env0 += int(n)
        self._ph_arena_end = used
        # "fill": one write-only region as large as a step's phantom transfers
        self._sink = torch.empty(sink, dtype=torch.uint8, device=d) if self.rehearse_mode == "fill" else None
        self._rh_native = None if not self.decode else \
            {key: devmem.empty((n, abi.native_env_bytes(self.P)), torch.uint8, d) for key, _, _, n, _ in self._ph}

    def _body(self, j: int, k: int):
        e = self.engines[j]
        e.obs = self.wires[j][k]
        # reward | term | trunc | mask | 0 per agent and the tick fault word, by the step's wire gather
        e.set_step_records(self.smalls[j][k], self.faults[k])
        e.scripted_actions(self.pseed)
        e.step()

    def _capture(self):
        torch.cuda.synchronize(self.device)
        self.graphs = {}
        for j in range(len(self.engines)):
            for k in range(self.ring):
                g = torch.cuda.CUDAGraph()
                with torch.cuda.graph(g, stream=self.streams[j]):
                    self._body(j, k)
                self.graphs[j, k] = g
        # each graph keeps the step-record pointers it captured; the handles forget them, so an
        # eager step later cannot write into a ring slot the comm stream may still be sending
        for e in self.engines:
            e.set_step_records(None)
        torch.cuda.synchronize(self.device)

    def _n_envs(self, r, j):
        return self.counts[r][j] if r < self.world else next(n for key, _, _, n, _ in self._ph if key == (r, j))

    def _consume(self, s: int, got, plan=None):
        """On the comm stream, after step s's buffers landed on the root."""
        from . import wire as nw

        if self.rank != 0:
            return
        with torch.cuda.stream(self.x.comm):
            nb = len(self.engines)
            items = []  # (key, (wire, smalls), expect or None, check?) in the arena's store order
            if self._ph:  # the phantom peers' transfers of this step, then their buffers in place
                if self._sink is not None:
                    self._sink.fill_(s & 0xFF)
                for (key, w, sm, n, expect), src in zip(self._ph, self._rh_src):
                    if src is not None:
                        w.copy_(src)
                    items.append((key, (w, sm), expect, True))
            items += [((0, j), got[0, j], None, False) for j in range(nb)]
            items += [((r, j), got[r, j], self.x.sizes[s % self.ring, r, j:j + 1], True)
                      for r in range(1, self.world) for j in range(nb)]
            if self.store is None:  # every received buffer against its announced size, up to 16 per launch
                recv = [(w, self._n_envs(*key), ex) for key, (w, sm), ex, chk in items if chk]
                for k in range(0, len(recv), 16):
                    nw.check_buffers(recv[k:k + 16], self.P, self.status)
            if self.native is not None:
                for key, (w, sm), ex, chk in items:
                    nw.unpack(w, self._n_envs(*key), self.P,
                              out=self.native[key] if key[0] < self.world else self._rh_native[key])
            if self.store is not None:  # every buffer of the step as one store, checked in its reservation
                self.store.reset()
                self._store_step(s, items)
                self._stored += self.store.ptr_dev[0].to(torch.int64)
        if self.on_step is not None:
            torch.cuda.synchronize(self.device)
            self.on_step(s, got)

    def _store_step(self, s: int, items):
        """The root's store of step s's buffers (learner mask = in the realm; no policy outputs
        modelled) as nmmo_exp_store_records_checked calls of up to 16 inputs, from ctypes input
        arrays built once per ring slot: per step only the step number and the peers' buffer
        pointers (their arena slots move with the announced sizes) are patched, so the host's
        per-step work stays a few field writes and one call per 16 inputs."""
        import ctypes

        from . import abi
        from ._native import check, lib

        k = s % self.ring
        plan = self._store_plans.get(k) if hasattr(self, "_store_plans") else None
        if plan is None:
            if not hasattr(self, "_store_plans"):
                self._store_plans = {}
            n_max = max(self._n_envs(*key) for key, _, _, _ in items)
            if self._zeros is None or self._zeros.numel() < n_max * self.P:
                self._zeros = torch.zeros(n_max * self.P, device=self.device)
                self._acts = torch.zeros((n_max * self.P, 12), dtype=torch.int32, device=self.device)
            chunks = []
            for c0 in range(0, len(items), 16):
                part = items[c0:c0 + 16]
                arr = (abi.NmmoStoreInput * len(part))()
                exp = (ctypes.c_void_p * len(part))()
                mask = 0
                for i, (key, (w, sm), ex, chk) in enumerate(part):
                    n = self._n_envs(*key) * self.P
                    st = sm.data_ptr()  # 8 B per agent: reward f32 | term | trunc | mask | pad
                    arr[i] = abi.NmmoStoreInput(n, 0, None, None, st, st + 4, st + 6, None, self.env_base[key] * self.P,
                                                self._acts.data_ptr(), self._zeros.data_ptr(), self._zeros.data_ptr(),
                                                w.data_ptr())
                    exp[i] = None if ex is None else ex.data_ptr()
                    mask |= (1 << i) if chk else 0
                chunks.append((arr, exp, mask, len(part)))
            self.store._ensure_scratch(sum(self._n_envs(*key) for key, _, _, _ in items) * self.P,
                                       min(16, len(items)), n_max * self.P)
            if getattr(self.store, "_ctl", None) is None:
                self.store._ctl = torch.zeros(abi.STORE_CTL_INTS, dtype=torch.int32, device=self.device)
            self.store._engine = self.engines[0]
            plan = self._store_plans[k] = chunks
        st = self.store
        stream = ctypes.c_void_p(self.x.comm.cuda_stream)
        i0 = 0
        for arr, exp, mask, n in plan:
            for i in range(n):
                key, (w, _), _, _ = items[i0 + i]
                arr[i].step = s + 1
                if key[0] > 0 and key[0] < self.world:  # a peer's buffer: where this step received it
                    arr[i].wire = w.data_ptr()
            i0 += n
            check(lib().nmmo_exp_store_records_checked(self.engines[0].h, ctypes.byref(st.x), ctypes.byref(st.records),
                                                       arr, n, 8, exp, mask, ctypes.c_void_p(self.status.data_ptr()),
                                                       ctypes.c_void_p(st._ctl.data_ptr()),
                                                       ctypes.c_void_p(st.scratch.data_ptr()), stream),
                  "nmmo_exp_store_records_checked")

    def step(self):
        import time

        h0 = time.perf_counter()
        self._step(self.t)
        self.host_s += time.perf_counter() - h0  # the host's own time per step (posting, not waiting)

    def _step(self, t):
        k = t % self.ring
        ready = []
        for j in range(len(self.engines)):
            st = self.streams[j]
            done = self.x.done(t)  # slot k's previous step (t - ring) has been sent / consumed
            if done is not None:
                st.wait_event(done)
            with torch.cuda.stream(st):
                if self.graphs is not None:
                    self.graphs[j, k].replay()
                else:
                    if self.before_step is not None:
                        self.before_step(t, j, self.engines[j])
                    self._body(j, k)
                ev = torch.cuda.Event()
                ev.record(st)
            ready.append(ev)
        if t >= 1:  # step t - 1's payload, now that step t is queued
            self._payload(t - 1)
        self.x.post_sizes(t, [w[k] for w in self.wires], ready, fault=self.faults[k])
        self.t += 1

    def _arena_plan(self, s: int):
        """The root's record arena layout of step s, on the host: the store reserves its inputs in
        order (the rehearsal's phantoms at their fixed slots, the root's own buffers, every peer's),
        each at the 16-B-aligned end of the last plus a 16-B descriptor, with the plausibility rules
        of storage.hip record_reserve_serial (the arena restarts every step). Received buffers go
        straight to their slots, so the store finds them in place and copies only the root's own —
        instead of receiving into the exchange's buffers and copying every one into the arena.
        None when any buffer would not be reserved (implausible size, no room): the step is then
        received into the exchange's buffers and copied, and the store flags what it refuses —
        a plan that shifted later slots would have them refused as misplaced."""
        from . import wire as nw

        if self.store is None or self.store.records is None:
            return None
        tot = self.x.totals(s)
        nb = len(self.engines)
        used, plan = (self._ph_arena_end if self._ph else 0), {}
        cap = self.store.arena.numel()
        for (r, j) in [(0, j) for j in range(nb)] + [(r, j) for r in range(1, self.world) for j in range(nb)]:
            n = int(tot[r][j])
            if n & 15 or n > self.x.caps[r][j] or n < nw.header_bytes(self.counts[r][j], self.P):
                return None
            base = (used + 15) & ~15
            if base + 16 + n > cap:
                return None
            if r != 0:
                plan[r, j] = self.store.arena[base + 16:base + 16 + n]
            used = base + 16 + n
        return plan

    def _payload(self, s: int):
        if s <= self._posted:  # drain() already moved it
            return
        ks = s % self.ring
        plan = self._arena_plan(s) if self.rank == 0 else None
        got = self.x.post_payload(s, [w[ks] for w in self.wires], [sm[ks] for sm in self.smalls],
                                  recv_into=plan)
        self._posted = s
        self._consume(s, got, plan)
        self.x.mark_done(s)

    def drain(self):
        """Post the last step's payload (once: the next step() does not post it again) and make
        the current stream wait for every transfer."""
        if self.t >= 1:
            self._payload(self.t - 1)
        cur = torch.cuda.current_stream(self.device)
        for st in self.streams:
            cur.wait_stream(st)
        cur.wait_stream(self.x.comm)

    def stored_rows(self) -> int:
        """Rows the root's store pass kept since the last call (synchronising read)."""
        torch.cuda.synchronize(self.device)
        n = int(self._stored.item())
        self._stored.zero_()
        return n

    def check_status(self):
        """The accumulated received-buffer check bits (0 = every received buffer was consistent)."""
        return int(self.status.item())

    def close(self):
        torch.cuda.synchronize(self.device)
        for j, e in enumerate(self.engines):
            e.obs = self.wires[j][0]
        self.graphs = None
