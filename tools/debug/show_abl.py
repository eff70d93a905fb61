"""Summarise gpurun_out/abl/*.json (abl_run.sh): value and kernel_ms per library and repetition."""
import glob, json, os, sys
d = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/abl"
for f in sorted(glob.glob(os.path.join(d, "*.json"))):
    try:
        j = json.loads(open(f).read().strip().splitlines()[-1])
    except Exception as e:  # noqa: BLE001
        print(os.path.basename(f), "unreadable", e)
        continue
    print(f"{os.path.basename(f):24s} {j['value'] / 1e6:9.1f} M  {j['ms_per_step']:.4f} ms/step  kernel_ms {j.get('kernel_ms')}")
