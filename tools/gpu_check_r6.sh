#!/bin/bash
# Round-6 GPU checks (run through gpurun from the repo root). Usage: tools/gpu_check_r6.sh <step>
set -o pipefail
out=gpurun_out/r6
mkdir -p $out
case "$1" in
scale)  # the checked store, the rehearsal, the uneven 2-rank gather; then the C5 node model by root share
  timeout -k 10 900 python -u -m pytest -x -v --timeout 170 --timeout-method thread \
    tests/test_gpu_wire.py tests/test_gpu_multirank.py > $out/tests_scale.log 2>&1 || exit 1
  for k in ${KS:-1024 768 512 256}; do
    timeout -k 10 400 python bench.py --config C5 --no-cpu-baseline --no-decode --steps 100 --warmup 20 \
      --root-envs $k --rehearse-copy > $out/c5_k$k.json 2> $out/c5_k$k.err || exit 1
  done
  ;;
*) echo "unknown step $1"; exit 2 ;;
esac
