set -e -o pipefail
mkdir -p gpurun_out/ab
for r in 1 2; do
  for m in 0 1; do
    NMMO_DEVMEM=$m timeout -k 10 240 python bench.py --config C4 --obs native --steps 100 --warmup 20 --no-cpu-baseline --no-extras \
      > gpurun_out/ab/devmemn_${m}_$r.json
    python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print('native devmem', sys.argv[2], round(d['value']/1e6,2), 'M', d['kernel_ms'])" gpurun_out/ab/devmemn_${m}_$r.json $m
  done
done
