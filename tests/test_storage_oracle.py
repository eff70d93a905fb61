"""CPU checks of the experience-storage checker (oracle/storage.py) and of
the storage structs of the C-ABI. The checker restates clean_pufferl.py's storage with the
reference's own torch CPU arithmetic; here it is checked against independent restatements:
numpy lexsort for the key order and a numpy float32 scalar loop for the advantages."""

import ctypes
import os
import subprocess
import tempfile

import numpy as np
import torch

from nmmo_amd import abi
from oracle.storage import ReferenceStorage

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _fill(rs, n_rows, steps, rng, elems):
    """Random recvs until the buffer is full (the evaluate loop's exit, clean_pufferl.py:290)."""
    env_id = np.arange(n_rows)
    step = 0
    while rs.ptr < rs.batch_size + 1:
        step += 1
        mask = rng.random(n_rows) < 0.7
        o = rng.integers(-50, 50, (n_rows, elems)).astype(np.float32)
        r = rng.standard_normal(n_rows).astype(np.float32)
        d = (rng.random(n_rows) < 0.1).astype(np.uint8)
        a = rng.integers(0, 100, (n_rows, 12)).astype(np.int32)
        lp = rng.standard_normal(n_rows).astype(np.float32)
        v = rng.standard_normal(n_rows).astype(np.float32)
        rs.store(o, r, d, mask, a, lp, v, env_id, step)
        assert step < steps
    return step


def test_store_cuts_at_capacity_and_sort_matches_lexsort():
    rng = np.random.default_rng(0)
    rs = ReferenceStorage(batch_size=255, obs_elems=7)
    _fill(rs, n_rows=40, steps=100, rng=rng, elems=7)
    assert rs.ptr == 256
    keys = np.array(rs.sort_keys)
    idxs = rs.sort()
    assert idxs == list(np.lexsort((keys[:, 1], keys[:, 0])))
    assert rs.sort_keys == []


def test_advantages_match_numpy_float32_loop():
    rng = np.random.default_rng(1)
    rs = ReferenceStorage(batch_size=127, obs_elems=3)
    _fill(rs, n_rows=16, steps=100, rng=rng, elems=3)
    idxs = rs.sort()
    adv = rs.advantages(idxs, 0.99, 0.95).numpy()
    # independent restatement: numpy float32 scalars, the Python-float constants cast per op
    g, gl = np.float32(0.99), np.float32(0.99 * 0.95)
    dn, vals, rew = rs.dones.numpy(), rs.values.numpy(), rs.rewards.numpy()
    last = np.float32(0)
    want = np.zeros(127, np.float32)
    for t in range(126, -1, -1):
        i, j = idxs[t], idxs[t + 1]
        nnt = np.float32(1) - dn[j]
        delta = (rew[j] + (g * vals[j]) * nnt) - vals[i]
        last = delta + (gl * nnt) * last
        want[t] = last
    assert np.array_equal(adv.view(np.uint32), want.view(np.uint32))
    # and close to the float64 recurrence
    last64, w64 = 0.0, np.zeros(127)
    for t in range(126, -1, -1):
        i, j = idxs[t], idxs[t + 1]
        nnt = 1.0 - float(dn[j])
        last64 = float(rew[j]) + 0.99 * float(vals[j]) * nnt - float(vals[i]) + 0.99 * 0.95 * nnt * last64
        w64[t] = last64
    assert np.allclose(adv, w64, rtol=1e-4, atol=1e-4)


def test_batch_shapes():
    rng = np.random.default_rng(2)
    rs = ReferenceStorage(batch_size=64, obs_elems=5)
    _fill(rs, n_rows=20, steps=100, rng=rng, elems=5)
    idxs = rs.sort()
    adv = rs.advantages(idxs, 0.99, 0.95)
    b = rs.batch(idxs, adv, batch_rows=4, bptt_horizon=8)
    assert b["num_minibatches"] == 2
    assert tuple(b["b_idxs"].shape) == (2, 4, 8)
    assert b["b_obs"].shape == (2, 4, 8, 5)
    assert torch.equal(b["b_returns"], b["b_advantages"] + b["b_values"])


def test_storage_structs_match_c_compiler():
    src = r"""
#include <stdio.h>
#include <stddef.h>
#include "nmmo_hip.h"
int main(void) {
  printf("%zu %zu %zu %zu %zu %zu\n", sizeof(NmmoExperience), offsetof(NmmoExperience, obs),
         offsetof(NmmoExperience, ptr), sizeof(NmmoStoreInput), offsetof(NmmoStoreInput, env_id_base),
         offsetof(NmmoStoreInput, values));
  return 0;
}
"""
    with tempfile.TemporaryDirectory() as d:
        c = os.path.join(d, "t.c")
        open(c, "w").write(src)
        exe = os.path.join(d, "t")
        subprocess.check_call(["gcc", "-I", os.path.join(ROOT, "include"), c, "-o", exe])
        got = list(map(int, subprocess.check_output([exe]).split()))
    want = [ctypes.sizeof(abi.NmmoExperience), abi.NmmoExperience.obs.offset, abi.NmmoExperience.ptr.offset,
            ctypes.sizeof(abi.NmmoStoreInput), abi.NmmoStoreInput.env_id_base.offset,
            abi.NmmoStoreInput.values.offset]
    assert got == want


def test_storage_calls_reject_bad_arguments():
    from nmmo_amd._native import lib

    L = lib()
    x = abi.NmmoExperience()
    assert L.nmmo_exp_sort(ctypes.byref(x), None, None, None) == abi.NMMO_E_INVALID
    assert b"capacity" in L.nmmo_last_error()
    assert L.nmmo_gather_rows(ctypes.c_void_p(16), 6, ctypes.c_void_p(16), 1, ctypes.c_void_p(16), None) \
        == abi.NMMO_E_INVALID
    assert L.nmmo_exp_scratch_ints(1000, 5) >= 1000 + 2
    assert L.nmmo_exp_scratch_ints(10, 5000) == 5000
