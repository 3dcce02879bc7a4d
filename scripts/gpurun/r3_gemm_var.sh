#!/bin/bash
# rmbx_linear_f32x6 variants (RMBX_GEMM_VAR) on the ACT shapes
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
for v in ${GEMM_VARS:-0 1 2 4 8 16 0}; do
  echo "== RMBX_GEMM_VAR=$v" >> gpurun_out/gemm_var.log
  RMBX_GEMM_VAR=$v timeout -k 10 200 python3 -u scripts/prof_gemm.py >> gpurun_out/gemm_var.log 2>&1 || exit 1
done
