# Winograd trunk in the product path: trunk/ACT parity tests, then a short bench line (no CPU leg)
# usage: bash scripts/gpurun/wino_bench.sh <tag>
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out &&
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_nn_gpu.py -k "trunk or f32" tests/test_act_full_gpu.py tests/test_winograd_gpu.py > gpurun_out/wino_bench_tests_$1.log 2>&1 &&
timeout -k 10 600 python bench.py --steps 12 --warmup 3 --no_cpu_baseline > gpurun_out/wino_bench_$1.json 2> gpurun_out/wino_bench_$1.err
