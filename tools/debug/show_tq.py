"""Summarise tools/debug/tick_quick.sh output (gpurun_out/tq)."""
import glob, json, os
for f in sorted(glob.glob("gpurun_out/tq/*.json")):
    j = json.loads(open(f).read().strip().splitlines()[-1])
    print(f"{os.path.basename(f):14s} {j['value'] / 1e6:9.1f} M  {j['ms_per_step']:.4f} ms/step  {j['kernel_ms']}")
for f in sorted(glob.glob("gpurun_out/tq/stamps_*.txt")):
    for line in open(f):
        if "median total" in line or "stepped" in line:
            print(os.path.basename(f), line.strip())
