# conditional barriers: parity / wrapper / observe tests, C2 / C3 / C4 stamps, C2 / C3 A/B vs the
# committed tick, then the remaining round-3 profiles (C5, C2, C3)
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out/r3 && set -o pipefail
timeout -k 10 600 python -u -m pytest -x -q --timeout 150 --timeout-method thread tests/test_gpu_parity.py \
  tests/test_gpu_wrapper.py tests/test_gpu_observe.py tests/test_gpu_fullsize.py > gpurun_out/r3/tests.log 2>&1 || exit 1
STAMPS_STAGGER=64 timeout -k 10 200 python tools/stamps.py C2 256 40 > gpurun_out/r3/stamps_C2.txt 2>&1 || exit 1
STAMPS_STAGGER=64 timeout -k 10 200 python tools/stamps.py C3 1024 40 > gpurun_out/r3/stamps_C3.txt 2>&1 || exit 1
STAMPS_STAGGER=64 timeout -k 10 200 python tools/stamps.py C4 512 40 > gpurun_out/r3/stamps_C4.txt 2>&1 || exit 1
bash tools/debug/ab_tick_lib.sh ab || exit 1
bash profiles/run_rocprof.sh r03 C5 C2 C3
