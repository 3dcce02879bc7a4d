#!/bin/bash
# round 4 box 3: the three-wave solver (RMBX_SOLVER_THREADS=192) -- engine parity tests with it, then
# the physics env-step time per variant (alternating, one process each) at 1024 Cable envs and
# 2048 Pick envs
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
RMBX_SOLVER_THREADS=192 timeout -k 10 600 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_engine_gpu.py tests/test_insert_gpu.py tests/test_pick_gpu.py tests/test_bad_state_gpu.py > gpurun_out/r4_solver192_tests.log 2>&1 || exit 1
for v in 256 192 256 192; do
  echo "== RMBX_SOLVER_THREADS=$v" >> gpurun_out/r4_solver_threads.log
  RMBX_SOLVER_THREADS=$v timeout -k 10 200 python3 -u scripts/prof_physics.py 1024 >> gpurun_out/r4_solver_threads.log 2>&1 || exit 1
done
for v in 256 192; do
  echo "== pick 2048 RMBX_SOLVER_THREADS=$v" >> gpurun_out/r4_solver_threads.log
  RMBX_SOLVER_THREADS=$v timeout -k 10 200 python3 -u scripts/prof_physics.py 2048 --env pick >> gpurun_out/r4_solver_threads.log 2>&1 || exit 1
done
