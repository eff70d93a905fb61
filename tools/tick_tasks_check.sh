# tick under task curricula: task + full parity with this tree, then head vs this tree (tools/debug/tick_tasks_ab.py)
L=nmmo_amd/lib
timeout -k 10 500 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_fullsize.py > gpurun_out/gpu_tasks.log 2>&1 || exit 1
for r in 1 2; do for lib in libnmmo_hip libnmmo_hip_head; do for c in cansee manual heldout; do
  NMMO_LIB=$L/$lib.so NMMO_ALLOW_STALE=1 timeout -k 10 120 python tools/debug/tick_tasks_ab.py $c 2>/dev/null | sed "s/^/$lib /" >> gpurun_out/tick_tasks.txt || exit 1
done; done; done
