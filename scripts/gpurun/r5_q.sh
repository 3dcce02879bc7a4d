#!/bin/bash
# FFN chain in the pre-split form: tests, ACT parity, image tests, then the bench A/B
set -o pipefail
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_presplit_gpu.py \
  tests/test_act_full_gpu.py tests/test_act_batch_gpu.py tests/test_image_gpu.py > gpurun_out/r5_q_tests.log 2>&1; rc=$?
grep -E "FAIL|Error|assert|passed|failed" gpurun_out/r5_q_tests.log | tail -20
[ $rc -ne 0 ] && exit $rc
bash scripts/gpurun/r5_n.sh
