# tick change check: parity tests (rollouts, full size, item stress, wrapper), phase stamps for
# C2 / C3 / C4, then C2 / C3 / C4-native / C5 bench lines
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out/tq && set -o pipefail
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_parity.py \
  tests/test_gpu_fullsize.py tests/test_gpu_wrapper.py > gpurun_out/tq/tests.log 2>&1 || { echo TESTS FAILED; tail -30 gpurun_out/tq/tests.log; exit 1; }
tail -1 gpurun_out/tq/tests.log
STAMPS_STAGGER=64 timeout -k 10 150 python tools/stamps.py C4 512 40 > gpurun_out/tq/stamps_C4.txt 2>&1 || exit 1
STAMPS_STAGGER=64 timeout -k 10 150 python tools/stamps.py C3 1024 40 > gpurun_out/tq/stamps_C3.txt 2>&1 || exit 1
STAMPS_STAGGER=64 timeout -k 10 150 python tools/stamps.py C2 128 40 > gpurun_out/tq/stamps_C2.txt 2>&1 || exit 1
for c in "C2" "C3" "C4 --obs native" "C5"; do
  n=$(echo $c | tr -d ' -')
  timeout -k 10 150 python bench.py --config $c --no-cpu-baseline --no-extras > gpurun_out/tq/$n.json 2> gpurun_out/tq/$n.err || { echo BENCH $c failed; tail -3 gpurun_out/tq/$n.err; exit 1; }
done
echo OK
