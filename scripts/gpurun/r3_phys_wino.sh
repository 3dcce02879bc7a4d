#!/bin/bash
# round 3: physics after the MuJoCo-exact divergence reset (engine + oracle), then the F(4x4) schedules
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_bad_state_gpu.py tests/test_engine_gpu.py tests/test_known_answers.py > gpurun_out/r3_phys_tests.log 2>&1
rc=$?; echo "phys tests rc=$rc"; [ $rc -ne 0 ] && exit $rc
bash scripts/gpurun/r3_wino4.sh
timeout -k 10 300 python -u scripts/prof_physics.py 256 --env pick > gpurun_out/r3_phys_pick_256.log 2>&1
echo "pick prof 256 rc=$?"
timeout -k 10 300 python -u scripts/prof_physics.py 1024 > gpurun_out/r3_phys_cable_1024.log 2>&1
echo "cable prof 1024 rc=$?"
