# Diagnostic: the N = 8 C5 node model at several rank-0 env shares (bench.py --root-envs), one box.
# Usage (GPU box): bash tools/debug/root_share_sweep.sh 448 480 512
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/r6 && set -o pipefail
for k in "$@"; do
  timeout -k 10 300 python bench.py --config C5 --root-envs $k --no-decode --no-cpu-baseline --steps 200 --warmup 20 \
    > gpurun_out/r6/model_k$k.json 2>/dev/null || exit 1
  python - $k <<'PY'
import json, sys
k = sys.argv[1]
d = json.load(open(f"gpurun_out/r6/model_k{k}.json"))
m = d.get("node_model") or d["extra_configs"]["C5"]["node_model"]
print(k, round(d["value"] / 1e6, 1), m["root_loaded"]["ms_per_step"], m["peer"]["ms_per_step"], m["link"]["ms_per_step"],
      m["bound"], round(m["value"] / 1e9, 3), m["ratio_vs_one_gpu"])
PY
done
