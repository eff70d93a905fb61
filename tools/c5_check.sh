# C5 path checks on the GPU box: wire / multirank / fault tests, then the default C5 bench line
mkdir -p gpurun_out/c5
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_wire.py tests/test_gpu_multirank.py tests/test_gpu_faults.py > gpurun_out/c5/tests.log 2>&1 && \
timeout -k 10 300 python bench.py --config C5 --no-cpu-baseline > gpurun_out/c5/bench.json 2> gpurun_out/c5/bench.err
