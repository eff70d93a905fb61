# obs kernels + tick: the obs/tick GPU tests, C4-native / C5 / C4 bench lines, kernel traces of
# C4-native and C5 (one bench batch), tick stamps C2 / C4
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out/obs && set -o pipefail
timeout -k 10 600 python -u -m pytest -x -v --timeout 150 --timeout-method thread tests/test_gpu_native_obs.py \
  tests/test_gpu_wire.py tests/test_gpu_storage.py tests/test_gpu_observe.py tests/test_gpu_wrapper.py \
  tests/test_gpu_fullsize.py tests/test_gpu_multirank.py tests/test_gpu_parity.py > gpurun_out/obs/tests.log 2>&1 || exit 1
timeout -k 10 200 python bench.py --config C4 --obs native --steps 200 --warmup 30 --no-cpu-baseline --no-extras > gpurun_out/obs/nat.json 2>gpurun_out/obs/nat.err || exit 1
timeout -k 10 200 python bench.py --config C5 --steps 200 --warmup 30 --no-cpu-baseline > gpurun_out/obs/c5.json 2>gpurun_out/obs/c5.err || exit 1
for cfg in nat c5; do
  if [ $cfg = nat ]; then A="--config C4 --obs native"; else A="--config C5 --no-decode"; fi
  timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/obs/kt_$cfg -o run -- python3 bench.py $A --batches 1 --steps 30 --warmup 5 --no-cpu-baseline --no-extras > gpurun_out/obs/kt_$cfg.log 2>&1 || exit 1
done
STAMPS_STAGGER=64 timeout -k 10 200 python tools/stamps.py C2 256 40 > gpurun_out/obs/stamps_C2.txt 2>&1 || exit 1
STAMPS_STAGGER=64 timeout -k 10 200 python tools/stamps.py C4 512 40 > gpurun_out/obs/stamps_C4.txt 2>&1 || exit 1
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/obs/default.json 2>gpurun_out/obs/default.err
