# The driver's round-end sequence on one GPU: smoke, then the default bench line (N = 1).
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || exit 1
tail -1 gpurun_out/smoke.log
timeout -k 10 600 python bench.py "$@" > gpurun_out/bench_default.json 2> gpurun_out/bench_default.err || exit 1
python - <<'PY'
import json
d = json.loads(open("gpurun_out/bench_default.json").read().strip().splitlines()[-1])
r = d["roofline"]
print("headline", round(d["value"] / 1e6, 2), "M", d["ms_per_step"], "ms", d["kernel_ms"], "frac", r["frac"], "fill", r["frac_of_write_ceiling"])
for k, v in (d.get("extra_configs") or {}).items():
    print(k, round(v["value"] / 1e6, 2), "M", v["kernel_ms"], v["roofline"]["frac"])
c = d["cpu_baseline"]
print("cpu", c["value"], c.get("c1_single_thread"), c["cores"])
PY
