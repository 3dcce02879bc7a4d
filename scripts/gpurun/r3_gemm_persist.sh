#!/bin/bash
# rmbx_linear_f32x6: default (16) vs persistent blocks (80) vs persistent + next-tile A prefetch (208)
# on the ACT transformer shapes (time + error vs f64 per variant)
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
for v in 16 80 208 16; do
  echo "== RMBX_GEMM_VAR=$v" >> gpurun_out/r3_gemm_persist.log
  RMBX_GEMM_VAR=$v timeout -k 10 200 python3 -u scripts/prof_gemm.py >> gpurun_out/r3_gemm_persist.log 2>&1 || exit 1
done
