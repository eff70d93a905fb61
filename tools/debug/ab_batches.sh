# A/B of bench.py --batches (env batches on separate streams) on one box: bash ab_batches.sh [bench args]
set -o pipefail
mkdir -p gpurun_out
for b in 2 1 2; do
  timeout -k 10 300 python bench.py --no-extras --no-cpu-baseline --batches $b "$@" > gpurun_out/bb$b.json 2> gpurun_out/bb$b.err || exit 1
  python -c "import json;d=json.loads(open('gpurun_out/bb$b.json').read().strip().splitlines()[-1]);print('batches',$b,round(d['value']/1e6,2),d['ms_per_step'],d['kernel_ms'],d['roofline']['frac'],d['launch'])"
done
