"""Build libnmmo_hip.so in-tree with hipcc for gfx950 (no JIT cache: the .so ships with the repo
snapshot to the GPU box)."""

from __future__ import annotations

import hashlib
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(HERE, "csrc")
LIB_DIR = os.path.join(HERE, "lib")
LIB_PATH = os.path.join(LIB_DIR, "libnmmo_hip.so")
STAMPS_PATH = os.path.join(LIB_DIR, "libnmmo_hip_stamps.so")
SOURCES = ["mapgen.hip", "tick.hip", "obs.hip", "wrap.hip", "storage.hip", "wire.hip", "wire_obs.hip", "native_obs.hip",
           "flat_obs.hip", "p2p.hip", "capi.hip"]
HEADERS = ["agent_obs.h", "common.h", "kernels.h", "wire.h"]
ARCH = os.environ.get("NMMO_OFFLOAD_ARCH", "gfx950")


def _hipcc() -> str:
    for cand in (os.environ.get("HIPCC"), "/opt/rocm/bin/hipcc", "hipcc"):
        if cand and (os.path.sep not in cand or os.path.exists(cand)):
            return cand
    raise RuntimeError("hipcc not found")


def source_hash() -> str:
    """sha256 (first 16 hex) over the HIP sources and headers the library is compiled from; the
    library embeds it (nmmo_build_info) and _native.lib() refuses a library built from other
    sources, so a run always reflects the tree it ships with."""
    h = hashlib.sha256()
    for f in [os.path.join(CSRC, f) for f in SOURCES + HEADERS] + [
            os.path.join(HERE, "..", "include", "nmmo_hip.h")]:
        with open(f, "rb") as fh:
            h.update(os.path.basename(f).encode() + b"\0" + fh.read())
    return h.hexdigest()[:16]


def stale() -> bool:
    """True unless the library exists and embeds the current source hash."""
    if not os.path.exists(LIB_PATH):
        return True
    with open(LIB_PATH, "rb") as fh:
        return ("src=" + source_hash()).encode() not in fh.read()


def build(force: bool = False, verbose: bool = False, stamps: bool = False) -> str:
    """Product library; `stamps=True` builds the diagnostic variant (phase clock stamps,
    tools/stamps.py) to lib/libnmmo_hip_stamps.so instead."""
    out = STAMPS_PATH if stamps else LIB_PATH
    if not force and not stamps and not stale():
        return LIB_PATH
    os.makedirs(LIB_DIR, exist_ok=True)
    tmp = out + ".tmp"
    flags = [
        f"--offload-arch={ARCH}", "-O3", "-std=c++17", "-fPIC", "-fvisibility=hidden", "-Wall", "-Werror",
        # no FMA contraction: hipcc contracts even __dadd_rn(__dmul_rn(..)) pairs, and the float /
        # double reward, wrapper and advantage arithmetic must round op by op like the oracle
        "-ffp-contract=off", *(["-DNMMO_STAMPS"] if stamps else []),
        f'-DNMMO_SRC_HASH="{source_hash()}"',
    ]
    # one hipcc per source in parallel (every kernel lives in its own translation unit), then link
    import concurrent.futures
    import tempfile

    with tempfile.TemporaryDirectory(prefix="nmmo_build_") as d:
        objs = [os.path.join(d, f + ".o") for f in SOURCES]
        cmds = [[_hipcc(), *flags, "-c", os.path.join(CSRC, f), "-o", o] for f, o in zip(SOURCES, objs)]
        if verbose:
            print("\n".join(" ".join(c) for c in cmds), file=sys.stderr)
        jobs = max(1, min(len(cmds), os.cpu_count() or 1, int(os.environ.get("MAX_JOBS", "8"))))
        with concurrent.futures.ThreadPoolExecutor(jobs) as ex:
            for f in [ex.submit(subprocess.check_call, c) for c in cmds]:
                f.result()
        subprocess.check_call([_hipcc(), f"--offload-arch={ARCH}", "-shared", "-fPIC", *objs, "-ldl", "-o", tmp])
    os.replace(tmp, out)
    return out


if __name__ == "__main__":
    print(build(force="--force" in sys.argv, verbose=True))
