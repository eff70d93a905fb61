set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 && \
timeout -k 10 300 python tools/bench_storage.py > gpurun_out/bench_storage.json 2> gpurun_out/bench_storage.err && \
timeout -k 10 300 python bench.py --config C4 --obs native --steps 100 --warmup 20 > gpurun_out/bench_C4n.json 2> gpurun_out/bench_C4n.err && \
timeout -k 10 300 python bench.py --config C5 --steps 50 --warmup 10 --no-cpu-baseline > gpurun_out/bench_C5.json 2> gpurun_out/bench_C5.err
