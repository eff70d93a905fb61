# round 4 GPU checks. `bash tools/gpu_check_r4.sh tests`: the new pool / fault / parity tests
# first, then the whole -m gpu suite and smoke(); `... bench`: the default bench line.
set -o pipefail
mkdir -p gpurun_out
if [ "$1" = "tests" ]; then
timeout -k 10 500 python -u -m pytest tests/test_gpu_vecenv.py tests/test_gpu_faults.py "tests/test_gpu_parity.py::test_can_see_tile_regrowth_parity_without_npc" tests/test_gpu_multirank.py -x -v --timeout 150 --timeout-method thread > gpurun_out/gpu_new.log 2>&1 && \
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 150 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 && \
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
else
timeout -k 10 400 python bench.py > gpurun_out/bench_default.json 2> gpurun_out/bench_default.err
fi
if [ "$1" = "stamps" ]; then
STAMPS_STAGGER=64 timeout -k 10 200 python tools/stamps.py C4 512 40 > gpurun_out/stamps_C4.txt 2>&1 && \
STAMPS_STAGGER=64 timeout -k 10 200 python tools/stamps.py C3 512 40 > gpurun_out/stamps_C3.txt 2>&1 && \
STAMPS_STAGGER=64 timeout -k 10 200 python tools/stamps.py C2 128 40 > gpurun_out/stamps_C2.txt 2>&1
fi
