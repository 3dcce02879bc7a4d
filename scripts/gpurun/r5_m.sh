#!/bin/bash
# pre-split A GEMM: tests, then timing
set -o pipefail
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_presplit_gpu.py \
  tests/test_act_full_gpu.py tests/test_act_batch_gpu.py > gpurun_out/r5_m_tests.log 2>&1; rc=$?
grep -E "PASS|FAIL|Error|assert|passed|failed" gpurun_out/r5_m_tests.log | tail -30
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u scripts/prof_gemm_presplit.py > gpurun_out/r5_m_prof.log 2>&1 || { echo "prof rc=$?"; tail -20 gpurun_out/r5_m_prof.log; exit 1; }
grep -v amdgpu.ids gpurun_out/r5_m_prof.log
