# C5 at N = 1 vs C4-native on one box
set -o pipefail
for c in "--config C5" "--config C4 --obs native --batches 1" "--config C5"; do
  timeout -k 10 300 python bench.py $c --no-extras --no-cpu-baseline > gpurun_out/c5ab.json 2> gpurun_out/c5ab.err || exit 1
  python -c "import json;d=json.loads(open('gpurun_out/c5ab.json').read().strip().splitlines()[-1]);print('$c',round(d['value']/1e6,2),d['ms_per_step'],d['kernel_ms'],d['launch'])"
done
