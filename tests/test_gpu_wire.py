"""Wire codec (SPEC.md §8c, csrc/wire.hip) on MI355X: nmmo_wire_pack's bytes equal the numpy
restatement's (oracle/wire.py, which derives every count from the native bytes) and
nmmo_wire_unpack restores the native obs bit-exactly (Buy.MarketItem rebuilt from the
listings), small and at C4 size (1,024 envs, staggered episodes); the NMMO_OBS_WIRE layout writes
the same bytes straight from the state; the experience store decodes kept rows from it."""

import numpy as np
import pytest
import torch

from tests.conftest import gpu_available

pytestmark = [pytest.mark.gpu, pytest.mark.skipif(not gpu_available(), reason="needs a GPU")]


def _engine(n, seed, map_n=4):
    from nmmo_amd import abi
    from nmmo_amd.config import Config
    from nmmo_amd.engine import NmmoEngine

    cfg = Config.preset("C4", MAP_N=map_n, early_stop_agent_num=8, obs_layout=abi.OBS_NATIVE)
    return NmmoEngine(cfg, n, seed=seed)


def test_wire_pack_matches_restatement():
    from nmmo_amd import abi, wire
    from oracle import wire as owire
    from oracle.oracle import split_state

    eng = _engine(3, seed=21)
    eng.reset()
    for t in range(45):
        if t == 20:
            eng.end_episodes(np.array([0, 1, 0], bool))
        eng.scripted_actions(500 + t)
        eng.step()
        if t % 15 != 14:
            continue
        w = wire.pack(eng)
        total = wire.total_bytes(w)
        nat = eng.obs.cpu().numpy()
        gold = split_state(eng.get_state(), eng.n_envs, eng.S, eng.P)["ent"][:, abi.F["gold"], :eng.P]
        ref = owire.pack(nat, eng.P, gold)
        assert total == ref.nbytes, (t, total, ref.nbytes)
        assert np.array_equal(w[:total].cpu().numpy(), ref), f"wire bytes differ at tick {t}"
        back = wire.unpack(w, eng.n_envs, eng.P)
        assert torch.equal(back, eng.obs), f"unpack differs at tick {t}"
    eng.close()


def test_wire_roundtrip_fullsize():
    from nmmo_amd import wire

    n = 1024
    eng = _engine(n, seed=3, map_n=256)
    eng.reset()
    ids = np.arange(n)
    for k in range(24):  # staggered episode phases, as in the bench
        eng.end_episodes(ids % 24 == k)
        eng.scripted_actions(77 + k)
        eng.step()
    w = wire.pack(eng)
    back = wire.unpack(w, n, eng.P)
    assert torch.equal(back, eng.obs)
    total = wire.total_bytes(w)
    assert total * 4 < eng.obs.numel(), (total, eng.obs.numel())
    eng.close()


def _pair(n, seed, map_n=4, wrapper=None):
    """A native-obs engine and a wire-obs engine (NMMO_OBS_WIRE) over the same envs."""
    from nmmo_amd import abi
    from nmmo_amd.config import Config
    from nmmo_amd.engine import NmmoEngine

    engs = []
    for lay in (abi.OBS_NATIVE, abi.OBS_WIRE):
        cfg = Config.preset("C4", MAP_N=map_n, early_stop_agent_num=8, obs_layout=lay)
        e = NmmoEngine(cfg, n, seed=seed)
        if wrapper is not None:
            from nmmo_amd.wrappers import wrapper_config

            e.set_wrapper(wrapper_config(wrapper[0], **wrapper[1]))
        engs.append(e)
    return engs


@pytest.mark.parametrize("wrapper", [None, ("yaofeng", dict(disable_give=True, donot_attack_dangerous_npc=True)),
                                     ("neurips23_start_kit", dict(heal_bonus_weight=0.03))])
def test_wire_layout_equals_pack_of_native(wrapper):
    """The wire records the obs kernel writes straight from the state (NMMO_OBS_WIRE) are the
    bytes nmmo_wire_pack makes of the native obs of the same state, tick by tick (resets,
    staggered episodes, wrapper obs edits included)."""
    from nmmo_amd import wire

    nat, wir = _pair(4, seed=33, wrapper=wrapper)
    for e in (nat, wir):
        e.reset()
    for t in range(60):
        if t == 17:
            for e in (nat, wir):
                e.end_episodes(np.array([1, 0, 0, 1], bool))
        for e in (nat, wir):
            e.scripted_actions(900 + t)
            e.step()
        if t % 6 != 5:
            continue
        ref = wire.pack(nat)
        total = wire.total_bytes(ref)
        assert wire.total_bytes(wir.obs) == total, t
        assert torch.equal(wir.obs[:total], ref[:total]), f"wire layout differs from pack(native) at tick {t}"
        assert torch.equal(nat.rew, wir.rew) and torch.equal(nat.mask, wir.mask)
    for e in (nat, wir):
        e.close()


def test_tick_fused_count_equals_count_kernel(monkeypatch):
    """A whole-handle C4 step into a wire buffer has the tick write the header's count words
    (tick.hip wire_count_fused): the buffers, step records included, equal those of a handle whose
    count kernel runs (NMMO_WIRE_FUSE=0 at create), tick by tick over resets and episode ends."""
    from nmmo_amd import abi, wire
    from nmmo_amd.config import Config
    from nmmo_amd.engine import NmmoEngine

    engs = []
    for fuse in ("1", "0"):
        monkeypatch.setenv("NMMO_WIRE_FUSE", fuse)
        cfg = Config.preset("C4", MAP_N=4, early_stop_agent_num=8, obs_layout=abi.OBS_WIRE)
        engs.append(NmmoEngine(cfg, 8, seed=57))
    monkeypatch.delenv("NMMO_WIRE_FUSE")
    assert engs[0].S == 384 and engs[0].P == 128  # the fused specialisation's shape
    recs = [torch.zeros((8, e.P, 8), dtype=torch.uint8, device=e.device) for e in engs]
    for e, r in zip(engs, recs):
        e.reset()
        e.set_step_records(r)
    for t in range(48):
        if t == 11:
            for e in engs:
                e.end_episodes(np.array([1, 0, 0, 1, 0, 0, 1, 0], bool))
        for e in engs:
            e.scripted_actions(700 + t)
            e.step()
        total = wire.total_bytes(engs[1].obs)
        assert wire.total_bytes(engs[0].obs) == total, t
        assert torch.equal(engs[0].obs[:total], engs[1].obs[:total]), f"fused count differs at tick {t}"
        assert torch.equal(recs[0], recs[1]), t
    for e in engs:
        e.set_step_records(None)
        e.close()


def test_step_records_equal_step_outputs():
    """nmmo_set_step_records: every wire-obs step writes, per agent, reward f32 | term | trunc |
    mask | 0 -- the bytes of the step's own outputs (over deaths and an episode end); a step
    after records are switched off leaves the buffer alone; the native layout refuses them."""
    from nmmo_amd._native import NativeError

    nat, wir = _pair(4, seed=41)
    with pytest.raises(NativeError):
        nat.set_step_records(torch.zeros((4, nat.P, 8), dtype=torch.uint8, device=nat.device))
    wir.reset()
    rec = torch.full((4, wir.P, 8), 0xAB, dtype=torch.uint8, device=wir.device)
    wir.set_step_records(rec)
    ended = 0
    for t in range(40):
        if t == 13:
            wir.end_episodes(np.array([0, 1, 0, 0], bool))
        wir.scripted_actions(300 + t)
        wir.step()
        want = torch.cat([wir.rew.view(torch.uint8).view(4, wir.P, 4), wir.term[..., None], wir.trunc[..., None],
                          wir.mask[..., None], torch.zeros_like(wir.mask[..., None])], -1)
        assert torch.equal(rec, want), f"step records differ from the step outputs at tick {t}"
        ended += int(wir.trunc.sum()) + int(wir.term.sum())
    assert ended > 0  # dones were among the records
    fault = torch.zeros(1, dtype=torch.int32, device=wir.device)
    wir.set_step_records(rec, fault)
    wir.scripted_actions(500)
    wir.step()
    assert int(fault.item()) == 0
    wir.inject_fault(4)  # the tick's fault word, as a loop bound would set it
    wir.scripted_actions(501)
    wir.step()
    assert int(fault.item()) == 4  # what fault_into() would have stored
    wir.inject_fault(0)
    wir.set_step_records(None)
    before = rec.clone()
    wir.scripted_actions(999)
    wir.step()
    assert torch.equal(rec, before)
    for e in (nat, wir):
        e.close()


def test_wire_layout_fullsize_roundtrip_and_check():
    """1,024 envs with staggered episodes: the wire layout decodes to the native obs of the same
    state, passes nmmo_wire_check, and a corrupted count word / total is flagged."""
    from nmmo_amd import wire

    n = 1024
    nat, wir = _pair(n, seed=5, map_n=256)
    ids = np.arange(n)
    for e in (nat, wir):
        e.reset()
    for k in range(32):
        for e in (nat, wir):
            e.end_episodes(ids % 32 == k)
            e.scripted_actions(300 + k)
            e.step()
    back = wire.unpack(wir.obs, n, wir.P)
    assert torch.equal(back, nat.obs)
    total = wire.total_bytes(wir.obs)
    st = torch.zeros(1, dtype=torch.int32, device=wir.device)
    want = torch.tensor([total], dtype=torch.int64, device=wir.device)
    wire.check_buffer(wir.obs, n, wir.P, st, want)
    assert int(st.item()) == 0
    bad = wir.obs[:total].clone()
    wire.check_buffer(bad, n, wir.P, st, want + 16)
    assert int(st.item()) & 1
    st.zero_()
    hb = wire.header_bytes(n, wir.P)
    cnt = bad[8 + 8 * n:8 + 8 * n + 2 * n * wir.P].view(torch.int16)
    j = int(torch.nonzero(cnt < 0)[3, 0])  # bit 15: in the realm
    cnt[j] = cnt[j] + 1  # one more visible entity than the record holds
    wire.check_buffer(bad, n, wir.P, st)
    assert int(st.item()) & (2 | 8), int(st.item())
    assert hb < total
    # the batched form (nmmo_wire_check_many, one launch): clean buffers stay clean, and a bad one
    # among good ones sets the same bits
    good = wir.obs[:total]
    st.zero_()
    wire.check_buffers([(good, n, want), (good, n, None), (good, n, want)], wir.P, st)
    assert int(st.item()) == 0
    wire.check_buffers([(good, n, want), (bad, n, None)], wir.P, st)
    assert int(st.item()) & (2 | 8), int(st.item())
    st.zero_()
    wire.check_buffers([(good, n, want + 16)], wir.P, st)
    assert int(st.item()) & 1
    for e in (nat, wir):
        e.close()


def test_wire_store_equals_native_store():
    """nmmo_exp_store from a wire buffer decodes exactly the kept rows into the flat experience
    rows the native store expands (bit-exact), under a learner mask that drops rows."""
    from nmmo_amd.storage import DeviceExperience

    n = 6
    nat, wir = _pair(n, seed=8)
    for e in (nat, wir):
        e.reset()
    P = nat.P
    xs = [DeviceExperience(700, nat.obs_elems, n * P, device=nat.device) for _ in range(2)]
    g = torch.Generator(device="cpu").manual_seed(3)
    for t in range(12):
        for e in (nat, wir):
            e.scripted_actions(40 + t)
            e.step()
        keep = (nat.mask.view(-1).cpu() != 0) & (torch.rand(n * P, generator=g) < 0.7)
        m = keep.to(torch.uint8).to(nat.device)
        z = torch.zeros(n * P, device=nat.device)
        for x, e in zip(xs, (nat, wir)):
            x.store(e.obs, e.rew.view(-1), e.term.view(-1), m, e.actions.view(-1, 12), z, z, step=t, engine=e)
    torch.cuda.synchronize()
    assert xs[0].ptr == xs[1].ptr > 0
    k = xs[0].ptr
    assert torch.equal(xs[0].obs[:k], xs[1].obs[:k])
    assert torch.equal(xs[0].env_id[:k], xs[1].env_id[:k]) and torch.equal(xs[0].rewards[:k], xs[1].rewards[:k])
    for e in (nat, wir):
        e.close()


def test_record_store_gathers_the_flat_store_rows():
    """Compact storage (nmmo_exp_store_records): the kept rows' observations stay wire records in
    an arena and expand per gather; every row equals the flat store's row from the same wire
    buffers (bit-exact, in a shuffled gather order), the small fields are identical, and a store
    the arena has no room for keeps no row and raises status bit 2."""
    from nmmo_amd.storage import DeviceExperience

    from nmmo_amd import abi
    from nmmo_amd.config import Config
    from nmmo_amd.engine import NmmoEngine

    n = 5
    wir = NmmoEngine(Config.preset("C4", MAP_N=4, early_stop_agent_num=8, obs_layout=abi.OBS_WIRE), n, seed=9)
    wir.reset()
    P = wir.P
    flat = DeviceExperience(900, wir.obs_elems, n * P, device=wir.device)
    rec = DeviceExperience(900, wir.obs_elems, n * P, device=wir.device, record_arena_bytes=64 << 20)
    g = torch.Generator(device="cpu").manual_seed(4)
    for t in range(10):
        wir.scripted_actions(70 + t)
        wir.step()
        keep = (wir.mask.view(-1).cpu() != 0) & (torch.rand(n * P, generator=g) < 0.6)
        m = keep.to(torch.uint8).to(wir.device)
        lp = torch.randn(n * P, generator=g).to(wir.device)
        for x in (flat, rec):
            x.store(wir.obs, wir.rew.view(-1), wir.term.view(-1), m, wir.actions.view(-1, 12), lp, lp, step=t,
                    engine=wir)
    torch.cuda.synchronize()
    k = flat.ptr
    assert rec.ptr == k == 901 and rec.status == 0
    for name in ("actions", "rewards", "dones", "logprobs", "values", "env_id", "step", "seq"):
        assert torch.equal(getattr(flat, name)[:k], getattr(rec, name)[:k]), name
    order = torch.randperm(k, generator=g).to(torch.int32).to(wir.device)
    got = rec.gather_obs(order)
    assert torch.equal(got, flat.obs[order.long()])
    assert int(rec.arena_used.item()) < 4 << 20  # a few MB of records, not 900 x 96 KB
    small = DeviceExperience(900, wir.obs_elems, n * P, device=wir.device, record_arena_bytes=4096)
    small.store(wir.obs, wir.rew.view(-1), wir.term.view(-1), m, wir.actions.view(-1, 12), lp, lp, step=0,
                engine=wir)
    torch.cuda.synchronize()
    assert small.ptr == 0 and small.status & 2
    wir.close()


def test_record_store_many_equals_sequential_stores():
    """nmmo_exp_store_records_many (every buffer of a step in one store, the gather root's call,
    rewards / dones / mask read from 8-B packed per-agent records) keeps exactly the rows, fields
    and gathered observations of one nmmo_exp_store_records call per buffer in the same order."""
    from nmmo_amd import abi
    from nmmo_amd.config import Config
    from nmmo_amd.engine import NmmoEngine
    from nmmo_amd.storage import DeviceExperience

    cfg = Config.preset("C4", MAP_N=4, early_stop_agent_num=8, obs_layout=abi.OBS_WIRE)
    engs = [NmmoEngine(cfg, 3, seed=12, env_index_base=3 * i) for i in range(2)]
    P = engs[0].P
    for e in engs:
        e.reset()
    n = 3 * P
    seq = DeviceExperience(1500, engs[0].obs_elems, 2 * n, device=engs[0].device, record_arena_bytes=64 << 20)
    many = DeviceExperience(1500, engs[0].obs_elems, 2 * n, device=engs[0].device, record_arena_bytes=64 << 20)
    g = torch.Generator(device="cpu").manual_seed(6)
    acts = torch.zeros((n, 12), dtype=torch.int32, device=engs[0].device)
    for t in range(8):
        batch = []
        for i, e in enumerate(engs):
            e.scripted_actions(90 + t)
            e.step()
            keep = (e.mask.view(-1) != 0) & (torch.rand(n, generator=g) < 0.7).to(e.device)
            lp = torch.randn(n, generator=g).to(e.device)
            sm = torch.zeros((n, 8), dtype=torch.uint8, device=e.device)
            sm[:, 0:4] = e.rew.view(-1).view(torch.uint8).view(n, 4)
            sm[:, 4] = e.term.view(-1)
            sm[:, 6] = keep.to(torch.uint8)
            seq.store(e.obs, e.rew.view(-1), e.term.view(-1), keep, acts, lp, lp, step=t, env_id_base=i * n,
                      engine=e)
            st = sm.view(-1)
            batch.append((e.obs.clone(), st, st[4:], st[6:], acts, lp, lp, i * n))
        many.store_many(batch, t, engs[0], field_stride=8)
    torch.cuda.synchronize()
    k = seq.ptr
    assert many.ptr == k == 1501 and many.status == 0 and seq.status == 0
    for name in ("actions", "rewards", "dones", "logprobs", "values", "env_id", "step", "seq", "row_agent"):
        assert torch.equal(getattr(seq, name)[:k], getattr(many, name)[:k]), name
    idx = torch.arange(k, dtype=torch.int32, device=engs[0].device)
    assert torch.equal(seq.gather_obs(idx), many.gather_obs(idx))
    for e in engs:
        e.close()


def test_checked_store_refuses_bad_and_misplaced_buffers():
    """nmmo_exp_store_records_checked (the gather root's store with the received-buffer check fused
    into its reservation): a corrupt input among good ones sets the check bits and keeps no row
    while the good ones are stored exactly as unchecked stores keep them; a buffer already at its
    arena slot is stored in place; one inside the arena but not at its slot is refused (status
    bit 4), never copied over the rows before it."""
    from nmmo_amd import abi, wire
    from nmmo_amd.config import Config
    from nmmo_amd.engine import NmmoEngine
    from nmmo_amd.storage import DeviceExperience

    cfg = Config.preset("C4", MAP_N=4, early_stop_agent_num=8, obs_layout=abi.OBS_WIRE)
    engs = [NmmoEngine(cfg, 3, seed=14, env_index_base=3 * i) for i in range(3)]
    P = engs[0].P
    dev = engs[0].device
    for e in engs:
        e.reset()
    for t in range(6):
        for e in engs:
            e.scripted_actions(30 + t)
            e.step()
    n = 3 * P
    acts = torch.zeros((n, 12), dtype=torch.int32, device=dev)
    z = torch.zeros(n, device=dev)

    def inp(e, i, w=None):
        sm = torch.zeros((n, 8), dtype=torch.uint8, device=dev)
        sm[:, 0:4] = e.rew.view(-1).view(torch.uint8).view(n, 4)
        sm[:, 6] = e.mask.view(-1)
        st = sm.view(-1)
        return (e.obs if w is None else w, st, st[4:], st[6:], acts, z, z, i * n)

    tots = [wire.total_bytes(e.obs) for e in engs]
    bad = engs[1].obs[:tots[1]].clone()
    cnt = bad[8 + 8 * 3:8 + 8 * 3 + 2 * 3 * P].view(torch.int16)
    j = int(torch.nonzero(cnt < 0)[2, 0])
    cnt[j] = cnt[j] + 1  # one more visible entity than the record holds
    ref = DeviceExperience(2000, engs[0].obs_elems, 3 * n, device=dev, record_arena_bytes=64 << 20)
    ref.store_many([inp(engs[0], 0), inp(engs[2], 2)], 1, engs[0], field_stride=8)
    chk = DeviceExperience(2000, engs[0].obs_elems, 3 * n, device=dev, record_arena_bytes=64 << 20)
    cs = torch.zeros(1, dtype=torch.int32, device=dev)
    exp = [torch.tensor([t], dtype=torch.int64, device=dev) for t in tots]
    chk.store_many([inp(engs[0], 0), inp(engs[1], 1, bad), inp(engs[2], 2)], 1, engs[0], field_stride=8,
                   expect=exp, check_status=cs)
    torch.cuda.synchronize()
    assert int(cs.item()) & (2 | 8) and chk.status & 8, (int(cs.item()), chk.status)
    k = ref.ptr
    assert chk.ptr == k > 0
    for name in ("rewards", "dones", "env_id", "step", "seq", "row_agent"):
        assert torch.equal(getattr(ref, name)[:k], getattr(chk, name)[:k]), name
    idx = torch.arange(k, dtype=torch.int32, device=dev)
    assert torch.equal(ref.gather_obs(idx), chk.gather_obs(idx))
    assert int(chk._ctl.abs().sum().item()) == 0  # the control words are left zero
    # clean inputs: no bits; the announced total is compared
    cs.zero_()
    chk.reset()
    chk.status_dev.zero_()
    chk.store_many([inp(engs[0], 0), inp(engs[2], 2)], 2, engs[0], field_stride=8, expect=[exp[0], exp[2]],
                   check_status=cs)
    torch.cuda.synchronize()
    assert int(cs.item()) == 0 and chk.status == 0 and chk.ptr == k
    chk.reset()
    chk.store_many([inp(engs[0], 0)], 3, engs[0], field_stride=8, expect=[exp[0] + 16], check_status=cs)
    torch.cuda.synchronize()
    assert int(cs.item()) & 1 and chk.status & 8 and chk.ptr == 0
    # a buffer already at its slot is stored in place; one elsewhere in the arena is refused
    for ok_slot in (True, False):
        x = DeviceExperience(2000, engs[0].obs_elems, 3 * n, device=dev, record_arena_bytes=64 << 20)
        off = 16 if ok_slot else 4096 + 16
        w = x.arena[off:off + tots[0]]
        w.copy_(engs[0].obs[:tots[0]])
        x.store_many([inp(engs[0], 0, w)], 1, engs[0], field_stride=8)
        torch.cuda.synchronize()
        if ok_slot:
            assert x.status == 0 and x.ptr > 0
            m = x.ptr
            assert torch.equal(x.gather_obs(idx[:m]), ref.gather_obs(idx[:m]))
        else:
            assert x.status & 16 and x.ptr == 0
    for e in engs:
        e.close()


def test_wire_gather_rehearsal_stores_phantom_peers():
    """The one-GPU rehearsal of an N-rank root (WireGather rehearse=R, bench.py's C5 node model):
    every step the root stores its own rows and R phantom peers' rows, each phantom's records and
    fields equal to a plain store of the phantom buffer, with the fused check clean, in both the
    write-only fill and the copy mode."""
    from nmmo_amd import abi, wire
    from nmmo_amd.config import Config
    from nmmo_amd.distributed import WireGather
    from nmmo_amd.engine import NmmoEngine
    from nmmo_amd.storage import DeviceExperience

    cfg = Config.preset("C4", MAP_N=4, early_stop_agent_num=8, obs_layout=abi.OBS_WIRE)
    dev = torch.device("cuda", 0)
    peer = [NmmoEngine(cfg, 3, seed=5, env_index_base=100 + 3 * i) for i in range(2)]
    for e in peer:
        e.reset()
    g = WireGather(peer, 11, graphs=False)
    for _ in range(5):
        g.step()
    g.drain()
    torch.cuda.synchronize()
    k = (g.t - 1) % g.ring
    phantom = []
    for j, e in enumerate(peer):
        tot = wire.total_bytes(g.wires[j][k])
        phantom.append((g.wires[j][k][:tot].clone(), g.smalls[j][k].clone(), e.n_envs))
    g.close()
    P = peer[0].P
    ph_rows = sum(int(sm.view(-1, 8)[:, 6].sum().item()) for _, sm, _ in phantom)
    # a plain store of the phantom buffers: the rows every phantom peer must add
    one = DeviceExperience(4000, 23987, 12 * P, device=dev, record_arena_bytes=64 << 20)
    acts = torch.zeros((3 * P, 12), dtype=torch.int32, device=dev)
    zz = torch.zeros(3 * P, device=dev)
    one.store_many([(w, sm.view(-1), sm.view(-1)[4:], sm.view(-1)[6:], acts, zz, zz, j * 3 * P)
                    for j, (w, sm, _) in enumerate(phantom)], 1, peer[0], field_stride=8)
    torch.cuda.synchronize()
    assert one.ptr == ph_rows > 0
    want = one.gather_obs(torch.arange(ph_rows, dtype=torch.int32, device=dev))
    root = [NmmoEngine(cfg, 2, seed=5, env_index_base=2 * i) for i in range(2)]
    for e in root:
        e.reset()
    R = 2
    for mode in ("fill", "copy"):
        rows = []
        store = DeviceExperience(4000, 23987, 16 * P, device=dev, record_arena_bytes=64 << 20)

        def on_step(s, got):
            rows.append((store.ptr, store.gather_obs(torch.arange(store.ptr, dtype=torch.int32, device=dev)),
                         store.env_id[:store.ptr].clone()))

        g = WireGather(root, 11, graphs=False, store=store, rehearse=R, phantom=phantom, rehearse_mode=mode,
                       on_step=on_step)
        for _ in range(4):
            g.step()
        g.drain()
        torch.cuda.synchronize()
        assert g.check_status() == 0 and store.status == 0
        assert len(rows) == 4
        for ptr, obs, eid in rows:
            assert ptr > R * ph_rows
            # the phantoms come first in the arena, in peer order: each equals the plain store
            for q in range(R):
                assert torch.equal(obs[q * ph_rows:(q + 1) * ph_rows], want), (mode, q)
            # env ids: phantom q's rows sit after the real ranks' 4 envs
            assert int(eid[:R * ph_rows].min()) >= 4 * P
        g.close()
    for e in peer + root:
        e.close()


def test_wire_pack_rejects_stale_native():
    """nmmo_wire_pack refuses a native buffer a tick without an obs gather has made stale, or
    one that is not the buffer the last gather wrote."""
    from nmmo_amd import wire
    from nmmo_amd._native import NativeError

    eng = _engine(2, seed=4)
    eng.reset()
    eng.scripted_actions(1)
    eng.step()
    wire.pack(eng)
    eng.scripted_actions(2)
    eng.step(write_obs=False)
    with pytest.raises(NativeError, match="stale"):
        wire.pack(eng)
    eng.observe()
    wire.pack(eng)
    other = torch.zeros_like(eng.obs)
    with pytest.raises(NativeError, match="not the buffer"):
        wire.pack(eng, native=other)
    eng.close()
