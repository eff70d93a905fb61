"""Compare one kernel's gfx950 ISA between two source trees (e.g. a round's tag and HEAD).

Usage: python tools/isa_diff.py <tree_a> <tree_b> <file.hip> <mangled_kernel_a> [<mangled_kernel_b>]
Each tree is a directory holding nmmo_amd/csrc and include (git archive <rev> nmmo_amd/csrc include).
Prints instruction / VGPR / SGPR / store / wait counts and the unified diff of the instruction
streams with branch labels normalised (kernel-argument offsets show up as s_load offsets)."""

import collections
import difflib
import os
import re
import subprocess
import sys


def asm(tree, src):
    out = f"/tmp/isa_{abs(hash(tree))}_{os.path.basename(src)}.s"
    subprocess.check_call(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-ffp-contract=off",
                           "--cuda-device-only", "-S", f"-I{tree}/include", f"{tree}/nmmo_amd/csrc/{src}", "-o", out],
                          stderr=subprocess.DEVNULL)
    return open(out).read()


def kernel(s, name):
    a = s.index("\n" + name + ":")
    b = s.index(".Lfunc_end", a)
    ins = [re.sub(r"\.LBB\d+_\d+", "L", ln.strip()) for ln in s[a:b].splitlines()
           if ln.startswith("\t") and not ln.strip().startswith((".", ";"))]
    meta = re.search(r"\.amdhsa_kernel " + re.escape(name) + r"(.*?)\.end_amdhsa_kernel", s, re.S).group(1)
    vg = int(re.search(r"\.amdhsa_next_free_vgpr (\d+)", meta).group(1))
    sg = int(re.search(r"\.amdhsa_next_free_sgpr (\d+)", meta).group(1))
    return ins, vg, sg


def stats(ins, vg, sg):
    c = collections.Counter(i.split()[0] for i in ins)
    return (f"instructions {len(ins)}, vgpr {vg}, sgpr {sg}, global stores "
            f"{sum(v for k, v in c.items() if k.startswith('global_store'))}, s_waitcnt {c['s_waitcnt']}, "
            f"ds {sum(v for k, v in c.items() if k.startswith('ds_'))}")


def main():
    ta, tb, src, ka = sys.argv[1:5]
    kb = sys.argv[5] if len(sys.argv) > 5 else ka
    a, b = kernel(asm(ta, src), ka), kernel(asm(tb, src), kb)
    print(f"A {ta} {ka}: {stats(*a)}")
    print(f"B {tb} {kb}: {stats(*b)}")
    d = list(difflib.unified_diff(a[0], b[0], "A", "B", lineterm="", n=0))
    print(f"differing instruction lines: {sum(1 for x in d if x[:1] in '+-' and x[:3] not in ('+++', '---'))}")
    print("\n".join(d))


if __name__ == "__main__":
    main()
