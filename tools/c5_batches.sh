# C5 at N = 1 with 1, 2 and 4 env batches per GPU (same box), delivered pass only
mkdir -p gpurun_out/c5b
for b in 2 4 1 2 4; do
  timeout -k 10 300 python bench.py --config C5 --no-cpu-baseline --no-decode --root-rehearsal 0 --batches $b --steps 200 --warmup 30 > gpurun_out/c5b/b$b.json 2> gpurun_out/c5b/b$b.err || exit 1
  python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print('batches', sys.argv[2], round(d['value']/1e6,1), d['ms_per_step'], d.get('kernel_ms'))" gpurun_out/c5b/b$b.json $b >> gpurun_out/c5b/summary.txt || exit 1
done
