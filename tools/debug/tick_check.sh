# tick changes: parity tests, C4 sub-stamps, C4 / C4-native bench lines, then SQ counters of the
# native obs kernel (one bench batch), one --pmc pass each
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out/tk && set -o pipefail
timeout -k 10 500 python -u -m pytest -x -v --timeout 150 --timeout-method thread tests/test_gpu_parity.py \
  tests/test_gpu_fullsize.py tests/test_gpu_wrapper.py > gpurun_out/tk/tests.log 2>&1 || exit 1
STAMPS_STAGGER=64 timeout -k 10 200 python tools/stamps.py C4 512 40 > gpurun_out/tk/stamps_C4.txt 2>&1 || exit 1
timeout -k 10 120 python bench.py --config C4 --obs native --steps 200 --warmup 30 --no-cpu-baseline --no-extras > gpurun_out/tk/nat.json 2>/dev/null || exit 1
B="python3 bench.py --config C4 --obs native --batches 1 --steps 30 --warmup 5 --no-cpu-baseline --no-extras"
timeout -k 10 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS --output-format csv -d gpurun_out/tk/p1 -o run -- $B > /dev/null 2>&1 && \
timeout -k 10 120 rocprofv3 --pmc SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SMEM SQ_BUSY_CYCLES SQ_INSTS_BRANCH --output-format csv -d gpurun_out/tk/p2 -o run -- $B > /dev/null 2>&1 && \
timeout -k 10 120 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_MISC SQ_INST_LEVEL_LDS SQ_LDS_BANK_CONFLICT --output-format csv -d gpurun_out/tk/p3 -o run -- $B > /dev/null 2>&1 && \
timeout -k 10 120 rocprofv3 --pmc TA_BUSY_avr TA_FLAT_WRITE_WAVEFRONTS_sum TCP_TCC_WRITE_REQ_sum TCP_PENDING_STALL_CYCLES_sum --output-format csv -d gpurun_out/tk/p4 -o run -- $B > /dev/null 2>&1
timeout -k 10 120 python bench.py --config C4 --steps 200 --warmup 30 --no-cpu-baseline --no-extras > gpurun_out/tk/c4.json 2>/dev/null
