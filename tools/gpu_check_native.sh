set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_native_obs.py tests/test_gpu_storage.py -x -v --timeout 120 --timeout-method thread > gpurun_out/gpu_tests_native.log 2>&1 && \
timeout -k 10 300 python bench.py --config C4 --obs native --steps 100 --warmup 20 --no-cpu-baseline > gpurun_out/bench_C4n.json 2> gpurun_out/bench_C4n.err
