# native / wire obs kernels: the obs-related GPU tests, then C4-native and C5 bench lines
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out/obs && set -o pipefail
timeout -k 10 400 python -u -m pytest -x -v --timeout 150 --timeout-method thread tests/test_gpu_native_obs.py \
  tests/test_gpu_wire.py tests/test_gpu_storage.py tests/test_gpu_observe.py tests/test_gpu_wrapper.py \
  tests/test_gpu_fullsize.py tests/test_gpu_multirank.py > gpurun_out/obs/tests.log 2>&1 || exit 1
timeout -k 10 120 python bench.py --config C4 --obs native --steps 200 --warmup 30 --no-cpu-baseline --no-extras > gpurun_out/obs/nat.json 2>gpurun_out/obs/nat.err || exit 1
timeout -k 10 120 python bench.py --config C5 --steps 200 --warmup 30 --no-cpu-baseline > gpurun_out/obs/c5.json 2>gpurun_out/obs/c5.err
