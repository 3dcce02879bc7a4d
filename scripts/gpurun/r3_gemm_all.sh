#!/bin/bash
# rmbx_linear_f32x6: tests, per-shape timing, SQ counter passes (tag $1)
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gemm_gpu.py > gpurun_out/gemm_tests.log 2>&1 && \
timeout -k 10 200 python3 -u scripts/prof_gemm.py > gpurun_out/prof_gemm_$1.log 2>&1 && \
bash scripts/gpurun/gemm_sq.sh $1
