# round 4 GPU checks. `bash tools/gpu_check_r4.sh tests`: the new tests first, then the whole
# -m gpu suite and smoke(); `... bench`: the default bench line; `... stamps`: tick phase stamps.
set -o pipefail
mkdir -p gpurun_out
if [ "$1" = "tests" ]; then
timeout -k 10 500 python -u -m pytest tests/test_gpu_wire.py tests/test_gpu_multirank.py tests/test_gpu_faults.py -x -v --timeout 150 --timeout-method thread > gpurun_out/gpu_new.log 2>&1 && \
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 150 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 && \
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
elif [ "$1" = "bench" ]; then
timeout -k 10 400 python bench.py > gpurun_out/bench_default.json 2> gpurun_out/bench_default.err
elif [ "$1" = "stamps" ]; then
STAMPS_STAGGER=64 timeout -k 10 200 python tools/stamps.py C4 512 40 > gpurun_out/stamps_C4.txt 2>&1 && \
STAMPS_STAGGER=64 timeout -k 10 200 python tools/stamps.py C3 512 40 > gpurun_out/stamps_C3.txt 2>&1 && \
STAMPS_STAGGER=64 timeout -k 10 200 python tools/stamps.py C2 128 40 > gpurun_out/stamps_C2.txt 2>&1
fi
if [ "$1" = "abnative" ]; then
L=nmmo_amd/lib
timeout -k 10 900 bash tools/ab_obs.sh C4 $L/libnmmo_hip.so,$L/libnmmo_hip_no8w32.so,$L/libnmmo_hip_no8w32x.so,$L/libnmmo_hip_no4w16x.so,$L/libnmmo_hip_no4w32.so --obs native > gpurun_out/ab_native.txt 2>&1
fi
if [ "$1" = "abflat" ]; then
L=nmmo_amd/lib
timeout -k 10 900 bash tools/ab_obs.sh C4 $L/libnmmo_hip.so,$L/libnmmo_hip_obsw4.so,$L/libnmmo_hip_obst16.so,$L/libnmmo_hip_obst16w4.so > gpurun_out/ab_flat.txt 2>&1
fi
if [ "$1" = "abwire" ]; then
L=nmmo_amd/lib
timeout -k 10 900 bash tools/ab_obs.sh C5 $L/libnmmo_hip.so,$L/libnmmo_hip_wo16w64.so,$L/libnmmo_hip_wo16w128.so,$L/libnmmo_hip_wonoloop.so --no-decode > gpurun_out/ab_wire.txt 2>&1
fi
if [ "$1" = "quick" ]; then
timeout -k 10 400 python -u -m pytest tests/test_gpu_wire.py tests/test_gpu_multirank.py tests/test_gpu_faults.py -x -v --timeout 150 --timeout-method thread > gpurun_out/gpu_new.log 2>&1 && \
timeout -k 10 300 python bench.py --config C5 > gpurun_out/bench_c5.json 2> gpurun_out/bench_c5.err && \
timeout -k 10 300 python bench.py > gpurun_out/bench_default.json 2> gpurun_out/bench_default.err && \
STAMPS_STAGGER=64 timeout -k 10 200 python tools/stamps.py C4 512 40 > gpurun_out/stamps_C4.txt 2>&1
fi
if [ "$1" = "abwe" ]; then
L=nmmo_amd/lib
timeout -k 10 900 bash tools/ab_obs.sh C5 $L/libnmmo_hip.so,$L/libnmmo_hip_wsplit.so,$L/libnmmo_hip_we8.so,$L/libnmmo_hip_we4.so --no-decode > gpurun_out/ab_we.txt 2>&1 && \
STAMPS_STAGGER=64 timeout -k 10 200 python tools/stamps.py C4 512 40 > gpurun_out/stamps_C4.txt 2>&1 && \
STAMPS_STAGGER=64 timeout -k 10 200 python tools/stamps.py C3 512 40 > gpurun_out/stamps_C3.txt 2>&1 && \
STAMPS_STAGGER=64 timeout -k 10 200 python tools/stamps.py C2 128 40 > gpurun_out/stamps_C2.txt 2>&1
fi
if [ "$1" = "abtick" ]; then
L=nmmo_amd/lib
timeout -k 10 600 bash tools/ab_obs.sh C4 $L/libnmmo_hip.so,$L/libnmmo_hip_tprev.so --obs native > gpurun_out/ab_tick.txt 2>&1 && \
STAMPS_STAGGER=64 timeout -k 10 200 python tools/stamps.py C4 512 40 > gpurun_out/stamps_C4.txt 2>&1 && \
NMMO_LIB=$L/libnmmo_hip_tprev_stamps.so NMMO_ALLOW_STALE=1 STAMPS_STAGGER=64 timeout -k 10 200 python tools/stamps.py C4 512 40 > gpurun_out/stamps_C4_prev.txt 2>&1 && \
STAMPS_STAGGER=64 timeout -k 10 200 python tools/stamps.py C4 512 40 > gpurun_out/stamps_C4_b.txt 2>&1 && \
timeout -k 10 300 python bench.py --config C5 --no-cpu-baseline > gpurun_out/bench_c5.json 2> gpurun_out/bench_c5.err
fi
if [ "$1" = "wire2" ]; then
L=nmmo_amd/lib
timeout -k 10 300 python -u -m pytest tests/test_gpu_wire.py tests/test_gpu_multirank.py -x -v --timeout 150 --timeout-method thread > gpurun_out/gpu_wire.log 2>&1 && \
timeout -k 10 900 bash tools/ab_obs.sh C5 $L/libnmmo_hip.so,$L/libnmmo_hip_wbase.so,$L/libnmmo_hip_wo16w4.so,$L/libnmmo_hip_wo64w8.so --no-decode > gpurun_out/ab_wire2.txt 2>&1
fi
if [ "$1" = "wire3" ]; then
L=nmmo_amd/lib
timeout -k 10 300 python -u -m pytest tests/test_gpu_wire.py -x -v --timeout 150 --timeout-method thread > gpurun_out/gpu_wire.log 2>&1 && \
timeout -k 10 900 bash tools/ab_obs.sh C5 $L/libnmmo_hip.so,$L/libnmmo_hip_wo8w2.so,$L/libnmmo_hip_wo16w8.so,$L/libnmmo_hip_wo32w4.so --no-decode > gpurun_out/ab_wire3.txt 2>&1 && \
bash profiles/run_rocprof.sh r04 C5 > gpurun_out/prof_c5.log 2>&1
fi
if [ "$1" = "cusplit" ]; then
B="python bench.py --steps 200 --warmup 30 --no-cpu-baseline --no-extras"
for a in "" "--no-graph" "--cu-split 16" "--cu-split 32" "--cu-split 64" "" "--cu-split 32"; do
  timeout -k 10 200 $B $a > gpurun_out/cs.json 2> gpurun_out/cs.err || { echo "FAIL $a"; tail -5 gpurun_out/cs.err; exit 1; }
  python -c "import json,sys; d=json.loads(open('gpurun_out/cs.json').read().strip().splitlines()[-1]); print(repr(sys.argv[1]), round(d['value']/1e6,2), d['ms_per_step'], d['kernel_ms'])" "$a"
done > gpurun_out/cusplit.txt 2>&1
fi
if [ "$1" = "wire4" ]; then
L=nmmo_amd/lib
timeout -k 10 300 python -u -m pytest tests/test_gpu_wire.py tests/test_gpu_multirank.py -x -v --timeout 150 --timeout-method thread > gpurun_out/gpu_wire.log 2>&1 && \
timeout -k 10 900 bash tools/ab_obs.sh C5 $L/libnmmo_hip.so,$L/libnmmo_hip_wbase.so --no-decode > gpurun_out/ab_wire4.txt 2>&1
fi
if [ "$1" = "tick" ]; then
L=nmmo_amd/lib
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py -x -v --timeout 200 --timeout-method thread > gpurun_out/gpu_tick.log 2>&1 && \
STAMPS_STAGGER=64 timeout -k 10 200 python tools/stamps.py C4 512 40 > gpurun_out/stamps_C4.txt 2>&1 && \
timeout -k 10 600 bash tools/ab_obs.sh C5 $L/libnmmo_hip.so,$L/libnmmo_hip_tbase.so --no-decode > gpurun_out/ab_tick.txt 2>&1 && \
timeout -k 10 600 bash tools/ab_obs.sh C3 $L/libnmmo_hip.so,$L/libnmmo_hip_tbase.so > gpurun_out/ab_tick_c3.txt 2>&1
fi
if [ "$1" = "ablnat" ]; then
L=nmmo_amd/lib
timeout -k 10 900 bash tools/ab_obs.sh C4 $L/libnmmo_hip.so,$L/libnmmo_hip_nnoloop.so,$L/libnmmo_hip_notile.so,$L/libnmmo_hip_nozero.so --obs native > gpurun_out/abl_nat.txt 2>&1
fi
