# Same-box A/B of the obs buffer allocation: torch's allocator (NMMO_DEVMEM=0) vs chunk-mapped
# (nmmo_dev_alloc), alternating, each in a fresh process.
set -e -o pipefail
mkdir -p gpurun_out/ab
for r in 1 2 3; do
  for m in 0 1; do
    NMMO_DEVMEM=$m timeout -k 10 240 python bench.py --config C4 --steps 100 --warmup 20 --no-cpu-baseline --no-extras \
      > gpurun_out/ab/devmem_${m}_$r.json
    python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); r=d['roofline']; print('devmem', sys.argv[2], round(d['value']/1e6,2), 'M obs', d['kernel_ms']['obs'], 'fill', r['write_ceiling_gbs'], r['frac_of_write_ceiling'])" gpurun_out/ab/devmem_${m}_$r.json $m
  done
done
