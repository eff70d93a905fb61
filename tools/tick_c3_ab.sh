# C3 tick occupancy variants: parity of one, then same-box C3 A/B and rocprofv3 solo of each
L=nmmo_amd/lib
NMMO_LIB=$L/libnmmo_hip_wpe6.so NMMO_ALLOW_STALE=1 timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_parity.py > gpurun_out/gpu_wpe6.log 2>&1 || exit 1
timeout -k 10 300 bash tools/ab_obs.sh C3 $L/libnmmo_hip.so,$L/libnmmo_hip_wpe6.so,$L/libnmmo_hip_wpe4.so > gpurun_out/ab_wpe_C3.txt 2>&1 || exit 1
export TMPDIR=/tmp
for v in libnmmo_hip libnmmo_hip_wpe6; do
  NMMO_LIB=$L/$v.so NMMO_ALLOW_STALE=1 timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_wpe/$v -o run -- python3 bench.py --config C3 --steps 100 --warmup 20 --no-cpu-baseline --no-extras > /dev/null 2>&1 || exit 1
done
