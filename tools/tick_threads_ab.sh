# tick workgroup size A/B: parity of the 512-thread variant, then C2 / C3 / C4 same box
L=nmmo_amd/lib
NMMO_LIB=$L/libnmmo_hip_t512.so NMMO_ALLOW_STALE=1 timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_fullsize.py > gpurun_out/gpu_t512.log 2>&1 || exit 1
for c in C2 C3 C4; do
  timeout -k 10 300 bash tools/ab_obs.sh $c $L/libnmmo_hip.so,$L/libnmmo_hip_t512.so > gpurun_out/ab_t512_$c.txt 2>&1 || exit 1
done
