#!/bin/bash
# round 3: Winograd F(4x4, 3x3) correctness (both schedules), then per-layer timing vs F(2x2)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_winograd_gpu.py -k winograd4 > gpurun_out/r3_wino4_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; [ $rc -ne 0 ] && exit $rc
RMBX_WINO4_SPLIT=1 timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_winograd_gpu.py -k winograd4 > gpurun_out/r3_wino4s_tests.log 2>&1
rc=$?; echo "tests split rc=$rc"; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u scripts/prof_winograd4.py 1024 --dbg > gpurun_out/r3_wino4_prof.log 2>&1
echo "prof rc=$?"
