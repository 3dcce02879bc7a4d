#!/bin/bash
# Winograd pre-split: tests, then the bench A/B
set -o pipefail
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_presplit_gpu.py \
  tests/test_wino_x6_gpu.py tests/test_gemm_gpu.py tests/test_act_full_gpu.py tests/test_act_batch_gpu.py > gpurun_out/r5_s_tests.log 2>&1; rc=$?
grep -E "FAIL|Error|assert|passed|failed" gpurun_out/r5_s_tests.log | tail -20
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u scripts/prof_wino_presplit.py 2>&1 | grep -v amdgpu.ids
bash scripts/gpurun/r5_n.sh
