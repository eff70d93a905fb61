# New wire obs kernel: wire tests + C5 bench; A/B of agents per native obs workgroup
# (NMMO_OBS_APB) with parity spot checks; C4 tick sub-stamps.
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out/apb && set -o pipefail
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_wire.py tests/test_gpu_storage.py tests/test_gpu_multirank.py > gpurun_out/apb/wire_tests.log 2>&1 || exit 1
timeout -k 10 120 python bench.py --config C5 --steps 200 --warmup 30 --no-cpu-baseline > gpurun_out/apb/c5_new.json 2>gpurun_out/apb/c5_new.err || exit 1
for apb in 32 64; do
  NMMO_OBS_APB=$apb timeout -k 10 200 python -u -m pytest -x -q --timeout 120 --timeout-method thread \
    tests/test_gpu_native_obs.py > gpurun_out/apb/par_$apb.log 2>&1 || exit 1
done
for apb in 16 32 64 16; do
  NMMO_OBS_APB=$apb timeout -k 10 120 python bench.py --config C4 --obs native --steps 200 --warmup 30 --no-cpu-baseline --no-extras > gpurun_out/apb/nat_$apb.json 2>/dev/null || exit 1
done
STAMPS_STAGGER=64 timeout -k 10 200 python tools/stamps.py C4 512 40 > gpurun_out/apb/stamps_C4b.txt 2>&1
