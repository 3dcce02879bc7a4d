#!/bin/bash
# round 3: two-level broadphase: engine vs oracle on every scene, then Pick / Cable physics profiles
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_pick_gpu.py tests/test_engine_gpu.py tests/test_bad_state_gpu.py tests/test_known_answers.py tests/test_insert_gpu.py > gpurun_out/r3_bp2_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u scripts/prof_physics.py 256 --env pick > gpurun_out/r3_phys_pick_256_bp2.log 2>&1
echo "pick prof rc=$?"
timeout -k 10 300 python -u scripts/prof_physics.py 2048 --env pick > gpurun_out/r3_phys_pick_2048_bp2.log 2>&1
echo "pick prof 2048 rc=$?"
timeout -k 10 300 python -u scripts/prof_physics.py 1024 > gpurun_out/r3_phys_cable_1024_bp2.log 2>&1
echo "cable prof rc=$?"
RMBX_WINO_TILE=f4 timeout -k 10 400 python bench.py --no_cpu_baseline > gpurun_out/r3_bench_f4b.json.log 2> gpurun_out/r3_bench_f4b.err
echo "bench f4 rc=$?"
