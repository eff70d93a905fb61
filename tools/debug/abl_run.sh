# Same-box timing A/B of ablation libraries (tools/debug/abl_build.py): bench lines of one config
# per library, alternating, two repetitions. Usage: abl_run.sh "<bench args>" v [v ...]
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && OUT=${ABL_OUT:-gpurun_out/abl} && mkdir -p $OUT && set -o pipefail
ARGS=$1; shift
timeout -k 10 200 python -c "import torch; torch.cuda.init()" || exit 1
for rep in 1 2; do
  for lib in base "$@"; do
    if [ $lib = base ]; then unset NMMO_LIB NMMO_ALLOW_STALE; else export NMMO_LIB=$PWD/nmmo_amd/lib/libnmmo_hip_$lib.so NMMO_ALLOW_STALE=1; fi
    timeout -k 10 150 python bench.py $ARGS --no-cpu-baseline --no-extras > $OUT/${lib}_$rep.json 2>$OUT/${lib}_$rep.err || exit 1
    echo "$lib $rep done"
  done
done
