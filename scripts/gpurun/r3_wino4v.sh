#!/bin/bash
# round 3: Winograd F(4x4) schedule variants: correctness of each, then per-layer timing
# usage: bash scripts/gpurun/r3_wino4v.sh <tag> <vars comma-separated>
set -o pipefail
mkdir -p gpurun_out
for v in ${2//,/ }; do
  export RMBX_WINO4_VAR=$v
  timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_winograd_gpu.py -k winograd4 > gpurun_out/r3_wino4v_$1_tests_$v.log 2>&1
  rc=$?; echo "tests var $v rc=$rc"; [ $rc -ne 0 ] && exit $rc
done
unset RMBX_WINO4_VAR
timeout -k 10 300 python -u scripts/prof_winograd4.py 1024 --vars $2 > gpurun_out/r3_wino4v_$1_prof.log 2>&1
rc=$?; echo "prof rc=$rc"; cat gpurun_out/r3_wino4v_$1_prof.log; exit $rc
