# wrapper-layer cost on each BASELINE config (same box A/B)
set -o pipefail
mkdir -p gpurun_out
for c in ${CONFIGS:-C2 C3 C4}; do
  for w in ${WRAPPERS:-none base neurips23_start_kit yaofeng}; do
    timeout -k 10 200 python bench.py --config $c --steps 100 --warmup 20 --no-cpu-baseline --wrapper $w > gpurun_out/bw_${c}_${w}.json 2>> gpurun_out/bw.err || exit 1
  done
done
