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
  for v in "unmap=whole free=1 tmp=1" "unmap=chunk free=1 attrs=1 tmp=1" "unmap=chunk free=0 attrs=1 tmp=1"; do
    timeout -k 10 120 tools/vmm_repro $v cycles=48 >> gpurun_out/vmm_repro.txt 2>&1; rc=$?
    [ $rc -le 1 ] || { echo "vmm_repro $v: rc $rc" >> gpurun_out/vmm_repro.txt; exit $rc; }
  done
  ;;
pmcflat)  # SQ counters of the flat obs kernel (C4, one 1,024-env batch), then the VMM reproducer and the default bench
  export TMPDIR=/tmp; mkdir -p gpurun_out/pmf
  B="python3 bench.py --config C4 --batches 1 --steps 12 --warmup 3 --no-cpu-baseline --no-extras"
  timeout -k 10 180 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS --output-format csv -d gpurun_out/pmf/p1 -o run -- $B > gpurun_out/pmf/p1.log 2>&1 && \
  timeout -k 10 180 rocprofv3 --pmc SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SMEM SQ_BUSY_CYCLES SQ_INSTS_BRANCH --output-format csv -d gpurun_out/pmf/p2 -o run -- $B > gpurun_out/pmf/p2.log 2>&1 && \
  timeout -k 10 180 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_MISC SQ_INST_LEVEL_LDS SQ_LDS_BANK_CONFLICT --output-format csv -d gpurun_out/pmf/p3 -o run -- $B > gpurun_out/pmf/p3.log 2>&1 && \
  timeout -k 10 180 rocprofv3 --pmc TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum --output-format csv -d gpurun_out/pmf/p4 -o run -- $B > gpurun_out/pmf/p4.log 2>&1 && \
  bash tools/gpu_check_r5.sh vmm && \
  timeout -k 10 600 python bench.py > gpurun_out/bench_default.json 2> gpurun_out/bench_default.err
  ;;
pmcflat2)  # the flat obs kernel's SQ counters only (passes 1-3)
  export TMPDIR=/tmp; mkdir -p gpurun_out/pmf
  B="python3 bench.py --config C4 --batches 1 --steps 12 --warmup 3 --no-cpu-baseline --no-extras"
  timeout -k 10 180 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS --output-format csv -d gpurun_out/pmf/p1 -o run -- $B > gpurun_out/pmf/p1.log 2>&1 && \
  timeout -k 10 180 rocprofv3 --pmc SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SMEM SQ_BUSY_CYCLES SQ_INSTS_BRANCH --output-format csv -d gpurun_out/pmf/p2 -o run -- $B > gpurun_out/pmf/p2.log 2>&1 && \
  timeout -k 10 180 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_MISC SQ_INST_LEVEL_LDS SQ_LDS_BANK_CONFLICT --output-format csv -d gpurun_out/pmf/p3 -o run -- $B > gpurun_out/pmf/p3.log 2>&1
  ;;
fost)  # per-section stamps of the flat obs kernel (the NMMO_FO_STAMPS variant)
  NMMO_LIB=nmmo_amd/lib/libnmmo_hip_fost.so NMMO_ALLOW_STALE=1 timeout -k 10 300 python tools/debug/fo_stamps.py > gpurun_out/fo_stamps.txt 2>&1
  ;;
fix1)  # flat obs fixes (Market loop vmcnt, wrapper scratch) vs HEAD, parity first; then the C5 kernel stats
  export TMPDIR=/tmp
  timeout -k 10 600 $PYT tests/test_gpu_parity.py tests/test_gpu_wrapper.py tests/test_gpu_native_obs.py tests/test_gpu_wire.py tests/test_gpu_zero_rows.py > gpurun_out/gpu_fix1.log 2>&1 && \
  timeout -k 10 600 bash tools/ab_obs.sh C4 $L/libnmmo_hip.so,$L/libnmmo_hip_head.so > gpurun_out/ab_fix1.txt 2>&1 && \
  timeout -k 10 600 bash tools/ab_obs.sh C4 $L/libnmmo_hip.so,$L/libnmmo_hip_head.so --wrapper neurips23_start_kit > gpurun_out/ab_fix1_wrap.txt 2>&1 && \
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_c5 -o run -- python3 bench.py --config C5 --steps 60 --warmup 10 --no-cpu-baseline > gpurun_out/prof_c5.json 2> gpurun_out/prof_c5.err
  ;;
c5)  # devmem (kept ranges), wire + multirank tests (batched check), then C5 at N = 1 (root_loaded pass)
  timeout -k 10 600 $PYT tests/test_gpu_devmem.py tests/test_gpu_wire.py tests/test_gpu_multirank.py tests/test_gpu_storage.py > gpurun_out/gpu_c5.log 2>&1 && \
  NMMO_DEVMEM_FREE_VA=1 timeout -k 10 200 python tools/debug/dbg_vmm.py > gpurun_out/dbg_vmm.txt 2>&1 && \
  timeout -k 10 300 python bench.py --config C5 --no-cpu-baseline > gpurun_out/bench_c5.json 2> gpurun_out/bench_c5.err
  ;;
tick1)  # tick parity with compile-time S/P, then same-box C2 / C3 / C4 against HEAD's library
  timeout -k 10 600 $PYT tests/test_gpu_parity.py tests/test_gpu_fullsize.py > gpurun_out/gpu_tick1.log 2>&1 && \
  timeout -k 10 300 bash tools/ab_obs.sh C2 $L/libnmmo_hip.so,$L/libnmmo_hip_head.so > gpurun_out/ab_tick_c2.txt 2>&1 && \
  timeout -k 10 300 bash tools/ab_obs.sh C3 $L/libnmmo_hip.so,$L/libnmmo_hip_head.so > gpurun_out/ab_tick_c3.txt 2>&1 && \
  timeout -k 10 300 bash tools/ab_obs.sh C4 $L/libnmmo_hip.so,$L/libnmmo_hip_head.so > gpurun_out/ab_tick_c4.txt 2>&1
  ;;
ext)  # flat rows' extended state (tracked chunks, inventory, Tile position): parity, then C4 / start-kit A/B vs HEAD
  timeout -k 10 600 $PYT tests/test_gpu_parity.py tests/test_gpu_zero_rows.py tests/test_gpu_obs_contract.py tests/test_gpu_wrapper.py \
    tests/test_gpu_fullsize.py tests/test_gpu_vecenv.py > gpurun_out/gpu_ext.log 2>&1 && \
  timeout -k 10 600 bash tools/ab_obs.sh C4 $L/libnmmo_hip.so,$L/libnmmo_hip_head.so > gpurun_out/ab_ext.txt 2>&1 && \
  timeout -k 10 600 bash tools/ab_obs.sh C4 $L/libnmmo_hip.so,$L/libnmmo_hip_head.so --wrapper neurips23_start_kit > gpurun_out/ab_ext_wrap.txt 2>&1
  ;;
prof)  # round-5 rocprofv3 summaries, then env batches per GPU (2 vs 4) on C4
  timeout -k 10 1000 bash profiles/run_rocprof.sh r05 C4 C4-native C4-rezero C5 C2 C3 > gpurun_out/prof_r05.log 2>&1 && \
  for b in 2 4 2 4; do timeout -k 10 120 python bench.py --batches $b --steps 200 --warmup 30 --no-cpu-baseline --no-extras > gpurun_out/bat_$b.json 2>/dev/null && \
    python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], round(d['value']/1e6,2), d['ms_per_step'], d['kernel_ms'])" gpurun_out/bat_$b.json $b >> gpurun_out/batches.txt || exit 1; done
  ;;
ab)  # same-box A/B of variant libraries: ab <config> <lib,lib,...> [bench args]
  CFG=$2; LIBS=$3; shift 3
  timeout -k 10 900 bash tools/ab_obs.sh $CFG $LIBS "$@" > gpurun_out/ab_$CFG.txt 2>&1
  ;;
*) echo "unknown mode $1"; exit 2 ;;
esac
