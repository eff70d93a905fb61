"""Ad hoc diagnostic: build libnmmo_hip_stamps.so with stamps 14/15 moved to new places.

Usage: python tools/debug/temp_stamps.py 'anchor14' 'anchor15'
Each anchor is an exact source line fragment of tick.hip; `__syncthreads(); NMMO_STAMP(k);` is
inserted before the first line containing it (it must be at block scope). The source file is restored afterwards.
"""
import os
import shutil
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
SRC = os.path.join(ROOT, "nmmo_amd", "csrc", "tick.hip")


def main():
    keep = open(SRC).read()
    s = keep
    for k in (14, 15):
        s = s.replace(f"  NMMO_STAMP({k});\n", f"  // moved {k}\n", 1)
    lines = s.split("\n")
    for k, anchor in zip((14, 15), sys.argv[1:3]):
        i = next(i for i, ln in enumerate(lines) if anchor in ln)
        lines.insert(i, f"  __syncthreads(); NMMO_STAMP({k});")
    try:
        open(SRC, "w").write("\n".join(lines))
        subprocess.check_call([sys.executable, "-c", "from nmmo_amd import build; build.build(stamps=True)"], cwd=ROOT)
    finally:
        open(SRC, "w").write(keep)


if __name__ == "__main__":
    main()
