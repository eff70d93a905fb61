# CanSeeTile rows per batch: 5 (this tree) vs 1 (variant) vs before the task changes, on the bench
# ticks (C2 / C3: TickGE) and under the curricula
L=nmmo_amd/lib
for c in C2 C3; do timeout -k 10 300 bash tools/ab_obs.sh $c $L/libnmmo_hip.so,$L/libnmmo_hip_see1.so,$L/libnmmo_hip_pre.so > gpurun_out/ab_see_$c.txt 2>&1 || exit 1; done
for r in 1 2; do for lib in libnmmo_hip libnmmo_hip_see1; do for c in cansee manual; do
  NMMO_LIB=$L/$lib.so NMMO_ALLOW_STALE=1 timeout -k 10 120 python tools/debug/tick_tasks_ab.py $c 2>/dev/null | sed "s/^/$lib /" >> gpurun_out/tick_see1.txt || exit 1
done; done; done
