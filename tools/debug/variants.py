"""Variant builds (diagnostic only): the library compiled with extra -D flags (compile-time
knobs such as NMMO_AO_WAVES / NMMO_AO_AGENTS / NMMO_NO_XCD in native_obs.hip) to
nmmo_amd/lib/libnmmo_hip_<name>.so, for same-box timing A/B (tools/ab_obs.sh with
NMMO_ALLOW_STALE=1). Usage: python tools/debug/variants.py name=-DA=1,-DB=2 [...]"""

import os
import subprocess
import sys
from concurrent.futures import ThreadPoolExecutor

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
from nmmo_amd import build as B  # noqa: E402


def build_variant(spec: str) -> str:
    name, flags = spec.split("=", 1)
    out = os.path.join(B.LIB_DIR, f"libnmmo_hip_{name}.so")
    cmd = [B._hipcc(), f"--offload-arch={B.ARCH}", "-O3", "-std=c++17", "-fPIC", "-shared", "-fvisibility=hidden",
           "-ffp-contract=off", f'-DNMMO_SRC_HASH="var-{name}"', *[f for f in flags.split(",") if f],
           *[os.path.join(B.CSRC, f) for f in B.SOURCES], "-o", out]
    subprocess.check_call(cmd)
    return out


if __name__ == "__main__":
    with ThreadPoolExecutor(4) as ex:
        for o in ex.map(build_variant, sys.argv[1:]):
            print(o)
