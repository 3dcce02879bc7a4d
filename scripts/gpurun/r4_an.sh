#!/bin/bash
# round 4 (not run: no box was free before the round ended): Hessian entries with a multiply-shift e / NVP (variant at-274e944) -- engine parity tests
# on that library, then physics time vs the default library (alternating, one process each)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
RMBX_LIB_VARIANT=at-274e944 timeout -k 10 600 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu tests/test_engine_gpu.py tests/test_insert_gpu.py tests/test_pick_gpu.py tests/test_bad_state_gpu.py > gpurun_out/r4_an_engine_tests.log 2>&1 || exit 1
for v in at-274e944 "" at-274e944 ""; do
  echo "== variant $v" >> gpurun_out/r4_an_solver_ab.log
  RMBX_LIB_VARIANT=$v timeout -k 10 200 python3 -u scripts/prof_physics.py 1024 >> gpurun_out/r4_an_solver_ab.log 2>&1 || exit 1
done
