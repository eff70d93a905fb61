set -o pipefail
for b in 1 2 1 2 4; do
  timeout -k 10 300 python bench.py --config C3 --no-extras --no-cpu-baseline --batches $b > gpurun_out/c3b$b.json 2>gpurun_out/c3b.err || exit 1
  python -c "import json;d=json.loads(open('gpurun_out/c3b$b.json').read().strip().splitlines()[-1]);print('C3 batches',$b,round(d['value']/1e9,3),d['ms_per_step'],d['kernel_ms'])"
done
for b in 1 2; do
  timeout -k 10 300 python bench.py --config C2 --no-extras --no-cpu-baseline --batches $b > gpurun_out/c2b$b.json 2>gpurun_out/c2b.err || exit 1
  python -c "import json;d=json.loads(open('gpurun_out/c2b$b.json').read().strip().splitlines()[-1]);print('C2 batches',$b,round(d['value']/1e9,3),d['ms_per_step'],d['kernel_ms'])"
done
