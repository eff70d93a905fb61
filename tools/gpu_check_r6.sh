#!/bin/bash
# Round-6 GPU checks (run through gpurun from the repo root). Usage: tools/gpu_check_r6.sh <step>
set -o pipefail
out=gpurun_out/r6
mkdir -p $out
case "$1" in
scale)  # the checked store, the rehearsal, the uneven 2-rank gather; then the C5 node model by root share
  timeout -k 10 900 python -u -m pytest -x -v --timeout 170 --timeout-method thread \
    tests/test_gpu_wire.py tests/test_gpu_multirank.py tests/test_gpu_storage.py tests/test_gpu_faults.py \
    > $out/tests_scale.log 2>&1 || exit 1
  for k in ${KS:-1024 768 512 256}; do
    timeout -k 10 400 python bench.py --config C5 --no-cpu-baseline --no-decode --steps 100 --warmup 20 \
      --root-envs $k --rehearse-copy > $out/c5_k$k.json 2> $out/c5_k$k.err || exit 1
  done
  ;;
rootprof)  # kernel trace of the C5 passes incl. the N = 8 root rehearsal at one root share
  export TMPDIR=/tmp
  timeout -k 10 240 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_wire.py \
    > $out/tests_wire.log 2>&1 || exit 1
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $out/rootprof -o run -- \
    python3 bench.py --config C5 --no-decode --root-envs ${K:-512} --steps 100 --warmup 20 --no-cpu-baseline \
    > $out/rootprof.json 2> $out/rootprof.err || exit 1
  ;;
scale2)  # tests, then the root's kernel trace, then the model by root share
  export TMPDIR=/tmp
  timeout -k 10 900 python -u -m pytest -x -v --timeout 170 --timeout-method thread \
    tests/test_gpu_wire.py tests/test_gpu_multirank.py tests/test_gpu_storage.py tests/test_gpu_faults.py \
    > $out/tests_scale.log 2>&1 || exit 1
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $out/rootprof -o run -- \
    python3 bench.py --config C5 --no-decode --root-envs ${K:-512} --steps 100 --warmup 20 --no-cpu-baseline \
    > $out/rootprof.json 2> $out/rootprof.err || exit 1
  for k in ${KS:-1024 512 256}; do
    timeout -k 10 400 python bench.py --config C5 --no-cpu-baseline --no-decode --steps 100 --warmup 20 \
      --root-envs $k > $out/c5_k$k.json 2> $out/c5_k$k.err || exit 1
  done
  ;;
shares)  # the C5 node model at N = 2, 4, 8 with the default and neighbouring root shares
  for nk in ${NKS:-2:984 4:832 8:512 8:640}; do
    n=${nk%%:*}; k=${nk##*:}
    timeout -k 10 400 python bench.py --config C5 --no-cpu-baseline --no-decode --steps 200 --warmup 30 \
      --root-rehearsal $n --root-envs $k > $out/model_n${n}_k$k.json 2> $out/model_n${n}_k$k.err || exit 1
  done
  ;;
contract)  # the scoped obs contract: pool tests, zero-row tests, then the start-kit consumer's rate
  timeout -k 10 900 python -u -m pytest -x -v --timeout 170 --timeout-method thread \
    tests/test_gpu_obs_contract.py tests/test_gpu_zero_rows.py tests/test_gpu_vecenv.py \
    > $out/tests_contract.log 2>&1 || exit 1
  timeout -k 10 400 python bench.py --no-cpu-baseline --steps 100 --warmup 20 > $out/bench_default.json \
    2> $out/bench_default.err || exit 1
  ;;
longrun)  # the row state at full size over 300 ticks (tracked vs full write; sampled envs vs the oracle)
  timeout -k 10 400 python -u -m pytest -x -v --timeout 180 --timeout-method thread tests/test_gpu_longrun.py \
    > $out/tests_longrun.log 2>&1 || exit 1
  ;;
tile)  # dense Tile stores: long-horizon parity, then same-box A/B against the component skip + WRITE_SIZE
  export TMPDIR=/tmp
  timeout -k 10 400 python -u -m pytest -x -v --timeout 180 --timeout-method thread tests/test_gpu_longrun.py \
    tests/test_gpu_zero_rows.py > $out/tests_tile.log 2>&1 || exit 1
  timeout -k 10 600 bash tools/debug/ab_lib.sh "--steps 200 --warmup 30" base tileskip > $out/ab_tile.txt 2>&1 || exit 1
  for v in base tileskip; do
    L=nmmo_amd/lib/libnmmo_hip.so; [ $v = base ] || L=nmmo_amd/lib/libnmmo_hip_$v.so
    NMMO_LIB=$L NMMO_ALLOW_STALE=1 timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv \
      -d $out/pmc_tile_$v -o run -- python3 bench.py --steps 30 --warmup 5 --no-cpu-baseline --no-extras \
      > /dev/null 2>&1 || exit 1
    NMMO_LIB=$L NMMO_ALLOW_STALE=1 timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv \
      -d $out/kt_tile_$v -o run -- python3 bench.py --steps 30 --warmup 5 --no-cpu-baseline --no-extras \
      > $out/kt_tile_$v.json 2>/dev/null || exit 1
  done
  ;;
p2p)  # the native RCCL group (one GPU, self point-to-point) and the multi-rank gather tests
  timeout -k 10 300 python -u -m pytest -x -v -s --timeout 120 --timeout-method thread tests/test_gpu_p2p.py \
    tests/test_gpu_multirank.py > $out/tests_p2p.log 2>&1 || exit 1
  ;;
abc5)  # same-box A/B of library variants on the C5 line (N = 1, no model passes): VARIANTS="base name ..."
  timeout -k 10 200 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_wire.py \
    > $out/tests_abc5.log 2>&1 || exit 1
  timeout -k 10 900 bash tools/debug/ab_lib.sh "--config C5 --steps 300 --warmup 30 --no-decode --root-rehearsal 0" \
    ${VARIANTS:-base} > $out/ab_c5.txt 2>&1 || exit 1
  ;;
abc4)  # parity of the obs kernels, then same-box A/B on the C4 headline and C4-native: VARIANTS="base name ..."
  timeout -k 10 400 python -u -m pytest -x -q --timeout 170 --timeout-method thread tests/test_gpu_longrun.py \
    tests/test_gpu_zero_rows.py tests/test_gpu_native_obs.py tests/test_gpu_parity.py > $out/tests_abc4.log 2>&1 || exit 1
  timeout -k 10 600 bash tools/debug/ab_lib.sh "--steps 200 --warmup 30" ${VARIANTS:-base} > $out/ab_c4.txt 2>&1 || exit 1
  timeout -k 10 600 bash tools/debug/ab_lib.sh "--obs native --steps 200 --warmup 30" ${VARIANTS:-base} \
    > $out/ab_c4native.txt 2>&1 || exit 1
  ;;
*) echo "unknown step $1"; exit 2 ;;
esac
