# same-box A/B of two libraries (lib/libnmmo_hip.so vs lib/libnmmo_hip_ab.so built from other
# tick sources): C2 / C3 / C4 bench lines, alternating
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out/ab && set -o pipefail
timeout -k 10 200 python -c "import torch; torch.cuda.init()" || exit 1
for rep in 1 2; do
  for lib in new ab; do
    if [ $lib = ab ]; then export NMMO_LIB=$PWD/nmmo_amd/lib/libnmmo_hip_ab.so NMMO_ALLOW_STALE=1; else unset NMMO_LIB NMMO_ALLOW_STALE; fi
    for cfg in C2 C3 C4; do
      timeout -k 10 120 python bench.py --config $cfg --steps 300 --warmup 50 --no-cpu-baseline --no-extras > gpurun_out/ab/${cfg}_${lib}_$rep.json 2>gpurun_out/ab/${cfg}_${lib}_$rep.err || exit 1
    done
  done
done
