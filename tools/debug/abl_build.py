"""Ablation builds (diagnostic only): copies of the library with one piece of a kernel switched
off by a source patch, built to nmmo_amd/lib/libnmmo_hip_<variant>.so for same-box timing A/B
(tools/debug/abl_run.sh). Outputs are wrong by construction; only kernel times are read.

Usage: python tools/debug/abl_build.py <variant> [...]   (variants: see PATCHES)
"""

import os
import shutil
import subprocess
import sys
from concurrent.futures import ThreadPoolExecutor

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
from nmmo_amd import build as B  # noqa: E402

NEVER = "p.S == 12345"  # a run-time false the compiler cannot fold
PATCHES = {
    "nobuy": [("native_obs.hip", "      if (exch) {\n        for (int j0 = 0; j0 < nm; j0 += 64) {",
               f"      if (exch && {NEVER}) {{\n        for (int j0 = 0; j0 < nm; j0 += 64) {{")],
    "notile": [("native_obs.hip", "        if (t < 225) {\n          d16[3 * t]", f"        if (t < 225 && {NEVER}) {{\n          d16[3 * t]")],
    "nozero": [("native_obs.hip", "for (int q = lane; q < body; q += 64) z4[q]", f"for (int q = lane; q < body && {NEVER}; q += 64) z4[q]")],
    "ntzero": [("native_obs.hip", "for (int q = lane; q < body; q += 64) z4[q] = make_uint4(0u, 0u, 0u, 0u);",
                "typedef unsigned int u32x4 __attribute__((ext_vector_type(4))); for (int q = lane; q < body; q += 64) __builtin_nontemporal_store((u32x4){0u, 0u, 0u, 0u}, reinterpret_cast<u32x4*>(&z4[q]));")],
    "wg32": [("agent_obs.h", "constexpr int kAoWaves = 4;", "constexpr int kAoWaves = 8;"),
             ("agent_obs.h", "constexpr int kAoAgents = 16; ", "constexpr int kAoAgents = 32; "),
             ("native_obs.hip", "__launch_bounds__(256)", "__launch_bounds__(512)"),
             ("wire_obs.hip", "__launch_bounds__(256)", "__launch_bounds__(512)")],
    "nomt": [("obs.hip", '  asm volatile("" : "+v"(my_task), "+v"(my_prev));', "")],
    "nomask": [("native_obs.hip", "        if (q < NMMO_NATIVE_MASK_BYTES / 16) {", f"        if (q < NMMO_NATIVE_MASK_BYTES / 16 && {NEVER}) {{")],
    "noent": [("native_obs.hip", "for (int k0 = 0; k0 < nv4; k0 += 4) {", f"for (int k0 = 0; k0 < nv4 && {NEVER}; k0 += 4) {{")],
    "nnoloop": [("native_obs.hip", "  for (int j = 0; j < per_wave; j++) {", f"  for (int j = 0; j < per_wave && {NEVER}; j++) {{")],
    # flat obs kernel (obs.hip)
    "fnomask": [("obs.hip", "  for (int k = lane_id(); k < n; k += 64)\n    obs_st(&row[lo + k]",
                 f"  for (int k = lane_id(); k < n && {NEVER}; k += 64)\n    obs_st(&row[lo + k]"),
                ("obs.hip", "      for (int k = lane; k < n; k += 64)\n        obs_st(&row[p.o_buy + k]",
                 f"      for (int k = lane; k < n && {NEVER}; k += 64)\n        obs_st(&row[p.o_buy + k]")],
    "fnotile": [("obs.hip", "    for (int t = lane; t < 225; t += 64) {", f"    for (int t = lane; t < 225 && {NEVER}; t += 64) {{")],
    "fnocomp": [("obs.hip", "    m.nv = compact(m.r, m.c);", f"    m.nv = {NEVER} ? compact(m.r, m.c) : 0;")],
    "fnoent": [("obs.hip", "      for (int k0 = 0; k0 < nv2; k0 += 2) {", f"      for (int k0 = 0; k0 < nv2 && {NEVER}; k0 += 2) {{")],
    "fnoinv": [("obs.hip", "    for (int k = lane; k < kInv * 16; k += 64) {", f"    for (int k = lane; k < kInv * 16 && {NEVER}; k += 64) {{")],
    "fnoloop": [("obs.hip", "  for (int j = 0; j < kPerWave; j++) {", f"  for (int j = 0; j < kPerWave && {NEVER}; j++) {{")],
    "noinv": [("native_obs.hip", "    if (ninv == 0) {\n      if (lane < kInv * 8 / 4)", f"    if (ninv == 0 || {NEVER}) {{\n      if (lane < kInv * 8 / 4)")],
}


def build_variant(v: str) -> str:
    top = os.path.join("/tmp", f"abl_{v}")
    src = os.path.join(top, "pkg", "csrc")  # csrc includes ../../include/nmmo_hip.h
    shutil.rmtree(top, ignore_errors=True)
    shutil.copytree(B.CSRC, src)
    shutil.copytree(os.path.join(ROOT, "include"), os.path.join(top, "include"))
    for fname, old, new in PATCHES[v]:
        p = os.path.join(src, fname)
        s = open(p).read()
        assert s.count(old) == 1, (v, fname, old)
        open(p, "w").write(s.replace(old, new))
    out = os.path.join(B.LIB_DIR, f"libnmmo_hip_{v}.so")
    cmd = [B._hipcc(), f"--offload-arch={B.ARCH}", "-O3", "-std=c++17", "-fPIC", "-shared", "-fvisibility=hidden",
           "-ffp-contract=off", f'-DNMMO_SRC_HASH="abl-{v}"', *[os.path.join(src, f) for f in B.SOURCES], "-o", out]
    subprocess.check_call(cmd)
    return out


if __name__ == "__main__":
    with ThreadPoolExecutor(4) as ex:
        for o in ex.map(build_variant, sys.argv[1:]):
            print(o)
