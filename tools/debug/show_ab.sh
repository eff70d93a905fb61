# Prints what tick_ab.sh left under gpurun_out/.
tail -n 3 gpurun_out/par.log
grep -hv amdgpu.ids gpurun_out/stamps_C2.txt gpurun_out/stamps_C3.txt
for f in C2 C3 C4n C4; do
  [ -f gpurun_out/$f.json ] || continue
  python - "$f" <<'PY'
import json, sys
f = sys.argv[1]
d = json.loads(open(f"gpurun_out/{f}.json").read().strip().splitlines()[-1])
print(f, round(d["value"] / 1e6, 1), "M", d["ms_per_step"], d["kernel_ms"], d["roofline"]["avg_launch_ms"])
PY
done
