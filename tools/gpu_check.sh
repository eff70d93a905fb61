set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 && \
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 && \
timeout -k 10 300 python bench.py > gpurun_out/bench_default.json 2> gpurun_out/bench_default.err && \
timeout -k 10 300 python bench.py --config C3 --steps 200 --warmup 20 > gpurun_out/bench_C3.json 2> gpurun_out/bench_C3.err && \
timeout -k 10 300 python bench.py --config C4 --steps 100 --warmup 20 > gpurun_out/bench_C4.json 2> gpurun_out/bench_C4.err
