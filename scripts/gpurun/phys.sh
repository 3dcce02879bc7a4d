cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out &&
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_engine_gpu.py tests/test_insert_gpu.py tests/test_door_gpu.py > gpurun_out/phys_tests.log 2>&1 &&
timeout -k 10 120 python scripts/prof_physics.py 1024 > gpurun_out/phys_prof.log 2>&1
