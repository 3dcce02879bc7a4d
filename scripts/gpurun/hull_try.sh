cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out &&
timeout -k 10 600 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_engine_gpu.py tests/test_bad_state_gpu.py tests/test_glue_gpu.py tests/test_rollout_gpu.py tests/test_product_schedule.py > gpurun_out/hull_tests.log 2>&1 &&
timeout -k 10 120 python scripts/prof_physics.py 1024 > gpurun_out/hull_prof_1024.log 2>&1 &&
timeout -k 10 420 python bench.py --no_cpu_baseline --steps 20 --warmup 4 > gpurun_out/hull_bench.json.log 2> gpurun_out/hull_bench.err
