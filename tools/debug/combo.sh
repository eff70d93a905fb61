# native obs at 5 waves + single-atomic tick counters: tests + bench lines; tick A/B (C2 / C3)
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out/combo && set -o pipefail
timeout -k 10 400 python -u -m pytest -x -q --timeout 150 --timeout-method thread tests/test_gpu_native_obs.py \
  tests/test_gpu_wire.py tests/test_gpu_parity.py tests/test_gpu_observe.py > gpurun_out/combo/tests.log 2>&1 || exit 1
timeout -k 10 200 python bench.py --config C4 --obs native --steps 200 --warmup 30 --no-cpu-baseline --no-extras > gpurun_out/combo/nat.json 2>gpurun_out/combo/nat.err || exit 1
bash tools/debug/ab_tick_lib.sh ab
