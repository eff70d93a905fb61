# Same-box A/B of several builds of the library on one bench config: one discarded warm-up run,
# then the builds alternate for 2 rounds.
# Usage (on the GPU box): bash tools/ab_obs.sh <config> <lib>[,<lib>...] [extra bench args]
set -e -o pipefail
CFG=$1; LIBS=$2; shift 2
mkdir -p gpurun_out/ab
run() {  # lib tag
  NMMO_LIB=$1 NMMO_ALLOW_STALE=1 timeout -k 10 240 python bench.py --config $CFG --steps 60 --warmup 15 \
    --no-cpu-baseline --no-extras "${@:3}" > gpurun_out/ab/${CFG}_$2.json
  python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], round(d['value']/1e6, 2), 'M', d['kernel_ms'])" gpurun_out/ab/${CFG}_$2.json $2
}
run ${LIBS%%,*} warm "$@"
for r in 1 2; do
  for lib in ${LIBS//,/ }; do
    run $lib $(basename $lib .so)_$r "$@"
  done
done
