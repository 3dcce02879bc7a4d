#!/bin/bash
# persistent pre-split form: equality tests, then timing; then the bench A/B
set -o pipefail
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu tests/test_presplit_gpu.py \
  > gpurun_out/r5_o_tests.log 2>&1; rc=$?
grep -E "FAIL|Error|assert|passed|failed" gpurun_out/r5_o_tests.log | tail -20
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u scripts/prof_gemm_presplit.py > gpurun_out/r5_o_prof.log 2>&1 || { echo "prof rc=$?"; tail -20 gpurun_out/r5_o_prof.log; exit 1; }
grep -v amdgpu.ids gpurun_out/r5_o_prof.log | head -4
bash scripts/gpurun/r5_n.sh
