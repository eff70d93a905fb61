# wire v3 + packed compaction: the obs / wire / storage / multirank / parity GPU tests, C5 and
# C4-native bench lines; then the tick library A/B
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out/v3 && set -o pipefail
timeout -k 10 600 python -u -m pytest -x -v --timeout 150 --timeout-method thread tests/test_gpu_wire.py \
  tests/test_gpu_native_obs.py tests/test_gpu_storage.py tests/test_gpu_multirank.py tests/test_gpu_parity.py \
  tests/test_gpu_observe.py > gpurun_out/v3/tests.log 2>&1 || exit 1
timeout -k 10 200 python bench.py --config C5 --steps 200 --warmup 30 --no-cpu-baseline > gpurun_out/v3/c5.json 2>gpurun_out/v3/c5.err || exit 1
timeout -k 10 200 python bench.py --config C4 --obs native --steps 200 --warmup 30 --no-cpu-baseline --no-extras > gpurun_out/v3/nat.json 2>gpurun_out/v3/nat.err || exit 1
bash tools/debug/ab_tick_lib.sh
