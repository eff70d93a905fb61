# round 5 GPU checks: `bash tools/gpu_check_r5.sh <mode>` on the GPU box (every step under its own
# time limit, chained with &&: the first failure ends the call).
set -o pipefail
mkdir -p gpurun_out
L=nmmo_amd/lib
PYT="python -u -m pytest -x -v --timeout 200 --timeout-method thread"
case "$1" in
contract)  # the pool's obs contract + incremental rows, then the full-write A/B (round-4 knobs vs Task registers)
  timeout -k 10 400 $PYT tests/test_gpu_obs_contract.py tests/test_gpu_zero_rows.py tests/test_gpu_vecenv.py \
    > gpurun_out/gpu_contract.log 2>&1 && \
  NMMO_OBS_REZERO=1 timeout -k 10 600 bash tools/ab_obs.sh C4 $L/libnmmo_hip.so,$L/libnmmo_hip_fullr4.so \
    > gpurun_out/ab_full.txt 2>&1
  ;;
tests)  # the whole -m gpu suite and smoke()
  timeout -k 10 900 $PYT tests -m gpu > gpurun_out/gpu_tests.log 2>&1 && \
  timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
  ;;
bench)  # the default bench line (N = 1)
  timeout -k 10 600 python bench.py > gpurun_out/bench_default.json 2> gpurun_out/bench_default.err
  ;;
flat)  # the flat-obs parity tests, then the C4 A/B (this tree vs the round-4 flat kernel)
  timeout -k 10 600 $PYT tests/test_gpu_parity.py tests/test_gpu_zero_rows.py tests/test_gpu_obs_contract.py \
    tests/test_gpu_wrapper.py tests/test_gpu_fullsize.py tests/test_gpu_native_obs.py tests/test_gpu_wire.py > gpurun_out/gpu_flat.log 2>&1 && \
  timeout -k 10 600 bash tools/ab_obs.sh C4 $L/libnmmo_hip.so,$L/libnmmo_hip_flatv1.so > gpurun_out/ab_flat.txt 2>&1 && \
  timeout -k 10 900 bash tools/ab_obs.sh C4 $L/libnmmo_hip.so,$L/libnmmo_hip_fa1.so,$L/libnmmo_hip_fa2.so,$L/libnmmo_hip_fa4.so,$L/libnmmo_hip_fa16.so,$L/libnmmo_hip_fa32.so > gpurun_out/abl_flat.txt 2>&1
  ;;
vmm)  # the standalone VMM reproducer (tools/vmm_repro.hip), four variants; rc 1 = wrong contents seen
  for v in "unmap=whole free=1" "unmap=chunk free=1" "unmap=chunk sync=1 free=1" "unmap=chunk free=0"; do
    timeout -k 10 120 tools/vmm_repro $v cycles=48 >> gpurun_out/vmm_repro.txt 2>&1; rc=$?
    [ $rc -le 1 ] || { echo "vmm_repro $v: rc $rc" >> gpurun_out/vmm_repro.txt; exit $rc; }
  done
  ;;
ab)  # same-box A/B of variant libraries: ab <config> <lib,lib,...> [bench args]
  CFG=$2; LIBS=$3; shift 3
  timeout -k 10 900 bash tools/ab_obs.sh $CFG $LIBS "$@" > gpurun_out/ab_$CFG.txt 2>&1
  ;;
*) echo "unknown mode $1"; exit 2 ;;
esac
