# exp_at_level without a constant table: tick parity, then C3 / C4 same box against HEAD's library
L=nmmo_amd/lib
timeout -k 10 500 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_fullsize.py > gpurun_out/gpu_exp.log 2>&1 || exit 1
for c in C3 C4; do timeout -k 10 300 bash tools/ab_obs.sh $c $L/libnmmo_hip.so,$L/libnmmo_hip_head.so > gpurun_out/ab_exp_$c.txt 2>&1 || exit 1; done
