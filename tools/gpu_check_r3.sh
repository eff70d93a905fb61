# round 3 GPU checks. `bash tools/gpu_check_r3.sh tests`: the new wire / gather tests first, then
# the whole -m gpu suite and smoke(); `... bench`: C5 and the default bench line, tick stamps.
set -o pipefail
mkdir -p gpurun_out
if [ "$1" = "tests" ]; then
timeout -k 10 400 python -u -m pytest tests/test_gpu_wire.py tests/test_gpu_storage.py tests/test_gpu_multirank.py tests/test_gpu_vecenv.py -x -v --timeout 120 --timeout-method thread > gpurun_out/gpu_new.log 2>&1 && \
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 150 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 && \
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
else
timeout -k 10 300 python bench.py --config C5 --steps 300 --warmup 50 --no-cpu-baseline > gpurun_out/bench_c5.json 2> gpurun_out/bench_c5.err && \
timeout -k 10 400 python bench.py > gpurun_out/bench_default.json 2> gpurun_out/bench_default.err && \
STAMPS_STAGGER=64 timeout -k 10 200 python tools/stamps.py C4 512 40 > gpurun_out/stamps_C4.txt 2>&1 && \
STAMPS_STAGGER=64 timeout -k 10 200 python tools/stamps.py C2 256 40 > gpurun_out/stamps_C2.txt 2>&1
fi
