# same-box A/B of tick library variants (lib/libnmmo_hip.so = "new", lib/libnmmo_hip_<v>.so built
# from other tick sources): C2 / C3 bench lines, alternating. Usage: ab_tick_lib.sh v [v ...]
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out/ab && set -o pipefail
timeout -k 10 200 python -c "import torch; torch.cuda.init()" || exit 1
for rep in 1 2; do
  for lib in new "$@"; do
    if [ $lib = new ]; then unset NMMO_LIB NMMO_ALLOW_STALE; else export NMMO_LIB=$PWD/nmmo_amd/lib/libnmmo_hip_$lib.so NMMO_ALLOW_STALE=1; fi
    for cfg in C2 C3; do
      timeout -k 10 120 python bench.py --config $cfg --steps 300 --warmup 50 --no-cpu-baseline --no-extras > gpurun_out/ab/${cfg}_${lib}_$rep.json 2>gpurun_out/ab/${cfg}_${lib}_$rep.err || exit 1
    done
  done
done
