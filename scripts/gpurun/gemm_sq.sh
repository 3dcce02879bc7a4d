#!/bin/bash
# SQ counter passes (one rocprofv3 run each) over scripts/prof_gemm_sq.py
# usage: bash scripts/gpurun/gemm_sq.sh <tag>
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/gemm_sq_$1 || exit 1
P1="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE"
P2="SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_MFMA SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_SALU"
P3="SQ_INST_LEVEL_VMEM SQ_INSTS_VMEM SQ_ACTIVE_INST_VMEM SQ_LDS_DATA_FIFO_FULL SQ_VMEM_TA_ADDR_FIFO_FULL SQ_VMEM_TA_CMD_FIFO_FULL SQ_ACTIVE_INST_SCA SQ_INSTS_SMEM"
i=0
for P in "$P1" "$P2" "$P3"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $P --kernel-trace --output-format csv -d gpurun_out/gemm_sq_$1/p$i -o run -- python3 scripts/prof_gemm_sq.py > gpurun_out/gemm_sq_$1/p$i.log 2>&1 || { echo "pass $i failed"; exit 1; }
  echo "pass $i ok"
done
python3 scripts/sq_summary.py gpurun_out/gemm_sq_$1 gemm_f32x6 > gpurun_out/gemm_sq_$1/summary.txt
find gpurun_out/gemm_sq_$1 -name "*_kernel_trace.csv" -delete
