"""The C-ABI library loads and exports every symbol include/nmmo_hip.h declares; the ctypes
mirror (nmmo_amd/abi.py) matches the header's structs and enums; argument errors are reported
through the return code + nmmo_last_error without touching a GPU. CPU only."""

import ctypes
import os
import re
import subprocess
import tempfile

import pytest

from nmmo_amd import abi
from nmmo_amd.config import Config

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "nmmo_hip.h")


def header_text():
    return open(HEADER).read()


@pytest.fixture(scope="module")
def native():
    from nmmo_amd import _native

    return _native.lib()


def test_every_declared_symbol_is_exported(native):
    decl = re.findall(r"NMMO_API\s+[\w\s\*]+?\b(nmmo_\w+)\s*\(", header_text())
    assert len(decl) >= 14
    out = subprocess.check_output(["nm", "-D", "--defined-only",
                                   os.path.join(ROOT, "nmmo_amd", "lib", "libnmmo_hip.so")]).decode()
    exported = set(re.findall(r"\sT\s(nmmo_\w+)", out))
    assert set(decl) == exported, (set(decl) ^ exported)
    from nmmo_amd import _native

    assert set(_native.SYMBOLS) == set(decl)
    for name in decl:
        getattr(native, name)


def test_enums_match_header():
    text = header_text()
    ent = re.search(r"enum NmmoField \{(.*?)\};", text, re.S).group(1)
    names = [n.strip().split("=")[0].strip() for n in re.sub(r"/\*.*?\*/", "", ent, flags=re.S).split(",")]
    names = [n for n in names if n.startswith("F_")]
    assert [n[2:].lower() for n in names] == abi.ENTITY_FIELDS
    env = re.search(r"enum NmmoEnvField \{(.*?)\};", text, re.S).group(1)
    enames = [n.strip().split("=")[0].strip() for n in env.split(",")]
    assert [n[2:].lower() for n in enames if n.startswith("E_")] == abi.ENV_FIELDS
    for macro, val in [("NMMO_SYS_RESOURCE", abi.SYS_RESOURCE), ("NMMO_SYS_EXCHANGE", abi.SYS_EXCHANGE),
                       ("NMMO_OBS_FLAT", abi.OBS_FLAT), ("NMMO_ABI_VERSION", abi.ABI_VERSION),
                       ("NMMO_STORE_CTL_INTS", abi.STORE_CTL_INTS), ("NMMO_P2P_ID_BYTES", abi.P2P_ID_BYTES),
                       ("NMMO_OBS_SEC_TILE", abi.OBS_SEC_TILE)]:
        m = re.search(rf"#define {macro} (.*?)(?:/\*|$)", text, re.M)
        assert eval(m.group(1).replace("u", "").strip()) == val, macro


def test_struct_layout_matches_c_compiler():
    src = r"""
#include <stdio.h>
#include <stddef.h>
#include "nmmo_hip.h"
int main(void) {
  printf("%zu %zu %zu %zu %zu %zu %zu %zu %zu %zu %zu %zu %zu %zu\n", sizeof(NmmoConfig), offsetof(NmmoConfig, map_seed),
         sizeof(NmmoLayout), offsetof(NmmoLayout, off_tile), offsetof(NmmoLayout, state_bytes_per_env),
         offsetof(NmmoConfig, event_cap), sizeof(NmmoTaskTerm), sizeof(NmmoTask), offsetof(NmmoTask, combine),
         sizeof(NmmoTaskState), offsetof(NmmoTaskState, acc), sizeof(NmmoP2POp), offsetof(NmmoP2POp, peer),
         sizeof(NmmoStoreInput));
  return 0;
}
"""
    with tempfile.TemporaryDirectory() as d:
        c = os.path.join(d, "t.c")
        open(c, "w").write(src)
        exe = os.path.join(d, "t")
        subprocess.check_call(["gcc", "-I", os.path.join(ROOT, "include"), c, "-o", exe])
        got = list(map(int, subprocess.check_output([exe]).split()))
    want = [ctypes.sizeof(abi.NmmoConfig), abi.NmmoConfig.map_seed.offset,
            ctypes.sizeof(abi.NmmoLayout), abi.NmmoLayout.off_tile.offset,
            abi.NmmoLayout.state_bytes_per_env.offset, abi.NmmoConfig.event_cap.offset,
            ctypes.sizeof(abi.NmmoTaskTerm), ctypes.sizeof(abi.NmmoTask), abi.NmmoTask.combine.offset,
            ctypes.sizeof(abi.NmmoTaskState), abi.NmmoTaskState.acc.offset, ctypes.sizeof(abi.NmmoP2POp),
            abi.NmmoP2POp.peer.offset, ctypes.sizeof(abi.NmmoStoreInput)]
    assert got == want
    assert ctypes.sizeof(abi.NmmoTaskState) == abi.TASK_STATE_BYTES == abi.task_state_dtype().itemsize


def test_event_and_predicate_enums_match_header():
    text = header_text()
    ev = re.search(r"enum NmmoEventCode \{(.*?)\};", text, re.S).group(1)
    codes = dict((k.strip()[3:], int(v)) for k, v in (p.split("=") for p in ev.split(",")))
    assert codes == {k: v for k, v in vars(abi.EventCode).items() if k.isupper()}
    pr = re.search(r"enum NmmoPredicate \{(.*?)\};", text, re.S).group(1)
    names = [p.strip().split("=")[0].strip() for p in re.sub(r"/\*.*?\*/", "", pr, flags=re.S).split(",")]
    names = [n for n in names if n.startswith("PRED_")]
    assert len(names) == len(abi.PREDICATES)
    camel = [n[5:].replace("_", "").lower() for n in names]
    assert camel == [p.lower() for p in abi.PREDICATES]


def test_default_config_matches_python(native):
    c = abi.NmmoConfig()
    native.nmmo_default_config(ctypes.byref(c))
    py = Config().to_c()
    for name, _ in abi.NmmoConfig._fields_:
        assert getattr(c, name) == getattr(py, name), name


def test_invalid_arguments_report_errors(native):
    bad = Config().to_c()
    bad.player_n = 500
    h = ctypes.c_void_p()
    rc = native.nmmo_create(ctypes.byref(bad), 4, 0, 0, None, ctypes.byref(h))
    assert rc == abi.NMMO_E_INVALID and not h.value
    assert b"player_n" in native.nmmo_last_error()
    bad = Config().to_c()
    bad.abi_version = 99
    assert native.nmmo_create(ctypes.byref(bad), 4, 0, 0, None, ctypes.byref(h)) == abi.NMMO_E_INVALID
    assert native.nmmo_step(None, None, None, None, None, None, None, None) == abi.NMMO_E_INVALID
    assert native.nmmo_observe(None, None, None) == abi.NMMO_E_INVALID
    assert native.nmmo_get_state(None, None, 0) == abi.NMMO_E_INVALID


def test_state_blob_size(native):
    from nmmo_amd import _native

    for preset, slots in [("C2", 128), ("C3", 384)]:
        lay = _native.layout(Config.preset(preset).to_c())
        assert lay.slots == slots
        assert lay.state_bytes_per_env == abi.state_bytes_per_env(slots)


def test_wrapper_structs_match_c_compiler():
    src = r"""
#include <stdio.h>
#include <stddef.h>
#include "nmmo_hip.h"
int main(void) {
  printf("%zu %zu %zu %zu %zu %zu %zu %zu %zu\n", sizeof(NmmoWrapperConfig),
         offsetof(NmmoWrapperConfig, heal_bonus_weight), offsetof(NmmoWrapperConfig, custom_bonus_scale),
         sizeof(NmmoAgentInfo), offsetof(NmmoAgentInfo, performed), offsetof(NmmoAgentInfo, unique_events),
         sizeof(NmmoWrapState), offsetof(NmmoWrapState, max_item_level), (size_t)NMMO_UNIQ_WORDS);
  return 0;
}
"""
    with tempfile.TemporaryDirectory() as d:
        c = os.path.join(d, "t.c")
        open(c, "w").write(src)
        exe = os.path.join(d, "t")
        subprocess.check_call(["gcc", "-I", os.path.join(ROOT, "include"), c, "-o", exe])
        got = list(map(int, subprocess.check_output([exe]).split()))
    info, ws = abi.agent_info_dtype(), abi.wrap_state_dtype()
    want = [ctypes.sizeof(abi.NmmoWrapperConfig), abi.NmmoWrapperConfig.heal_bonus_weight.offset,
            abi.NmmoWrapperConfig.custom_bonus_scale.offset, info.itemsize, info.fields["performed"][1],
            info.fields["unique_events"][1], ws.itemsize, ws.fields["max_item_level"][1], abi.UNIQ_WORDS]
    assert got == want
    # 17 event codes x 18 item/skill types x 16 levels fit the experienced bitset
    assert abi.UNIQ_WORDS * 32 >= 17 * 18 * 16


def test_set_wrapper_rejects_bad_handles(native):
    assert native.nmmo_set_wrapper(None, None, None) == abi.NMMO_E_INVALID
    assert native.nmmo_get_wrapper_state(None, None, None) == abi.NMMO_E_INVALID


def test_storage_structs_and_wire_layout_match_c_compiler():
    src = r"""
#include <stdio.h>
#include <stddef.h>
#include "nmmo_hip.h"
int main(void) {
  printf("%zu %zu %zu %zu %d %zu %zu\n", sizeof(NmmoStoreInput), offsetof(NmmoStoreInput, values),
         offsetof(NmmoStoreInput, wire), sizeof(NmmoExperience), NMMO_OBS_WIRE, sizeof(NmmoRecordStore),
         offsetof(NmmoRecordStore, row_agent));
  return 0;
}
"""
    with tempfile.TemporaryDirectory() as d:
        c = os.path.join(d, "t.c")
        open(c, "w").write(src)
        exe = os.path.join(d, "t")
        subprocess.check_call(["gcc", "-I", os.path.join(ROOT, "include"), c, "-o", exe])
        got = list(map(int, subprocess.check_output([exe]).split()))
    assert got == [ctypes.sizeof(abi.NmmoStoreInput), abi.NmmoStoreInput.values.offset,
                   abi.NmmoStoreInput.wire.offset, ctypes.sizeof(abi.NmmoExperience), abi.OBS_WIRE,
                   ctypes.sizeof(abi.NmmoRecordStore), abi.NmmoRecordStore.row_agent.offset]


def test_wire_calls_report_errors(native):
    assert native.nmmo_wire_check(None, 4, 128, None, None, None) == abi.NMMO_E_INVALID
    assert native.nmmo_wire_pack(None, None, None, None) == abi.NMMO_E_INVALID
    assert native.nmmo_end_episodes(None, None, None) == abi.NMMO_E_INVALID
    assert native.nmmo_wire_header_bytes(4, 500) == abi.NMMO_E_INVALID
