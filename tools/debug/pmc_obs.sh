# SQ counters of the native obs kernel (C4 --obs native) and the wire obs kernel (C5), one bench
# batch each, one --pmc pass per counter set
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out/pmo && set -o pipefail
timeout -k 10 200 python -c "import torch; torch.cuda.init()" || exit 1
for cfg in nat c5; do
  if [ $cfg = nat ]; then A="--config C4 --obs native"; else A="--config C5 --no-decode"; fi
  B="python3 bench.py $A --batches 1 --steps 30 --warmup 5 --no-cpu-baseline --no-extras"
  timeout -k 10 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS --output-format csv -d gpurun_out/pmo/$cfg/p1 -o run -- $B > gpurun_out/pmo/$cfg.p1.log 2>&1 || exit 1
  timeout -k 10 120 rocprofv3 --pmc SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SMEM SQ_BUSY_CYCLES SQ_INSTS_BRANCH --output-format csv -d gpurun_out/pmo/$cfg/p2 -o run -- $B > gpurun_out/pmo/$cfg.p2.log 2>&1 || exit 1
  timeout -k 10 120 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_MISC SQ_INST_LEVEL_LDS SQ_LDS_BANK_CONFLICT --output-format csv -d gpurun_out/pmo/$cfg/p3 -o run -- $B > gpurun_out/pmo/$cfg.p3.log 2>&1 || exit 1
  timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/pmo/$cfg/kt -o run -- $B > gpurun_out/pmo/$cfg.kt.log 2>&1 || exit 1
done
