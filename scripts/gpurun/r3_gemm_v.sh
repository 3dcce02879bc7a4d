#!/bin/bash
# round 3: rmbx_linear_f32x6 schedule variants (RMBX_GEMM_VARIANT) + correctness
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gemm_gpu.py > gpurun_out/gemm_tests.log 2>&1 && \
for v in ${VARIANTS:-1}; do
  echo "== variant $v" >> gpurun_out/prof_gemm_v.log
  RMBX_GEMM_VARIANT=$v timeout -k 10 200 python3 -u scripts/prof_gemm.py >> gpurun_out/prof_gemm_v.log 2>&1 || exit 1
done
