# physics tests + stage profile at 64 / 1024 envs.  usage: bash scripts/gpurun/phys2.sh <tag>
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out &&
timeout -k 10 600 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_engine_gpu.py tests/test_known_answers.py tests/test_bad_state_gpu.py tests/test_insert_gpu.py tests/test_door_gpu.py tests/test_cabinet_gpu.py tests/test_toolbox_gpu.py tests/test_pick_gpu.py tests/test_ring.py > gpurun_out/phys_tests_$1.log 2>&1 &&
for n in 64 1024; do timeout -k 10 120 python scripts/prof_physics.py $n > gpurun_out/phys_prof_$1_$n.log 2>&1 || exit $?; done
