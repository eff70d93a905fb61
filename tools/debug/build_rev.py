"""Diagnostic A/B helper: build the library from the sources of a git revision (default HEAD) into
nmmo_amd/lib/libnmmo_hip_<name>.so (NMMO_SRC_HASH "var-<name>"; load with NMMO_ALLOW_STALE=1).
Usage: python tools/debug/build_rev.py <name> [rev]"""
import os
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
from nmmo_amd import build as B  # noqa: E402

name, rev = sys.argv[1], (sys.argv[2] if len(sys.argv) > 2 else "HEAD")
with tempfile.TemporaryDirectory() as d:
    subprocess.check_call(f"git -C {ROOT} archive {rev} nmmo_amd/csrc include | tar -x -C {d}", shell=True)
    srcs = sorted(f for f in os.listdir(os.path.join(d, "nmmo_amd", "csrc")) if f.endswith(".hip"))
    out = os.path.join(B.LIB_DIR, f"libnmmo_hip_{name}.so")
    cmd = [B._hipcc(), f"--offload-arch={B.ARCH}", "-O3", "-std=c++17", "-fPIC", "-shared", "-fvisibility=hidden",
           "-ffp-contract=off", f'-DNMMO_SRC_HASH="var-{name}"', *[os.path.join(d, "nmmo_amd", "csrc", f) for f in srcs],
           "-o", out]
    subprocess.check_call(cmd)
    print(out)
