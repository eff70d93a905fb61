# SQ counters of the flat obs kernel (C4, one 1,024-env batch), one --pmc pass per counter set
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out/pmf && set -o pipefail
timeout -k 10 200 python -c "import torch; torch.cuda.init()" || exit 1
B="python3 bench.py --config C4 --batches 1 --steps 12 --warmup 3 --no-cpu-baseline --no-extras"
timeout -k 10 180 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS --output-format csv -d gpurun_out/pmf/p1 -o run -- $B > gpurun_out/pmf/p1.log 2>&1 || exit 1
timeout -k 10 180 rocprofv3 --pmc SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SMEM SQ_BUSY_CYCLES SQ_INSTS_BRANCH --output-format csv -d gpurun_out/pmf/p2 -o run -- $B > gpurun_out/pmf/p2.log 2>&1 || exit 1
timeout -k 10 180 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_MISC SQ_INST_LEVEL_LDS SQ_LDS_BANK_CONFLICT --output-format csv -d gpurun_out/pmf/p3 -o run -- $B > gpurun_out/pmf/p3.log 2>&1 || exit 1
