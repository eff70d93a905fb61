# Multi-rank bench path rehearsed on one GPU: 2 ranks sharing cuda:0 over gloo
set -o pipefail
export NMMO_BENCH_BACKEND=gloo
for c in C4 C3; do
  timeout -k 10 300 python bench.py --gpus 2 --config $c --steps 50 --warmup 10 --no-cpu-baseline > gpurun_out/n2_$c.json 2> gpurun_out/n2_$c.err || exit 1
  python -c "import json;d=json.loads(open('gpurun_out/n2_$c.json').read().strip().splitlines()[-1]);print('$c',d['n_gpus'],round(d['value']/1e6,2),d['ms_per_step'],d['config']['parallelism'],d['launch'],d['alive_fraction'])"
done
# C5: the learner gather (wire pack, point-to-point sends, root decode) over gloo's host path
timeout -k 10 300 python bench.py --gpus 2 --config C5 --steps 30 --warmup 5 --no-cpu-baseline > gpurun_out/n2_C5.json 2> gpurun_out/n2_C5.err || exit 1
python -c "import json;d=json.loads(open('gpurun_out/n2_C5.json').read().strip().splitlines()[-1]);print('C5',d['n_gpus'],round(d['value']/1e6,3),d['ms_per_step'],d['gather'])"
