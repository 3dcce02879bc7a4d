#!/bin/bash
# round 3, first GPU call: DataKey routing + composed Pick workloads (configs 4/5), then the conv1d capture diagnostic
set -o pipefail
export MIOPEN_DEBUG_CONV_DIRECT_NAIVE_CONV_FWD=0
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -v --timeout 400 --timeout-method thread -m gpu \
  tests/test_motion_routing.py tests/test_pick_workloads_gpu.py > gpurun_out/r3_t1_tests.log 2>&1
rc=$?
echo "tests rc=$rc"
[ $rc -ne 0 ] && exit $rc
MIOPEN_ENABLE_LOGGING=1 timeout -k 10 240 python -u scripts/diag_conv1d_capture.py 1024 > gpurun_out/r3_conv1d_capture.log 2>&1
echo "diag rc=$?"
