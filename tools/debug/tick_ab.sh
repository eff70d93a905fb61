# Tick-kernel change check on one GPU: parity (rollouts + full-size grids), phase stamps for C2/C3
# (needs lib/libnmmo_hip_stamps.so built here first), then the C2 / C3 / C4-native bench lines.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py -m gpu -x -q \
  --timeout 200 --timeout-method thread > gpurun_out/par.log 2>&1 || exit 1
timeout -k 10 120 python tools/stamps.py C2 128 40 > gpurun_out/stamps_C2.txt 2>&1 || exit 1
timeout -k 10 120 python tools/stamps.py C3 512 40 > gpurun_out/stamps_C3.txt 2>&1 || exit 1
for c in C2 C3; do
  timeout -k 10 200 python bench.py --config $c --no-cpu-baseline --no-extras > gpurun_out/$c.json 2> gpurun_out/$c.err || exit 1
done
timeout -k 10 200 python bench.py --config C4 --obs native --no-cpu-baseline --no-extras > gpurun_out/C4n.json 2> gpurun_out/C4n.err || exit 1
