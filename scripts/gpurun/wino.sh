# Winograd f32 conv: parity tests, per-shape profile, trunk + production-size ACT fp32 tests
# usage: bash scripts/gpurun/wino.sh <tag>
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out &&
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu tests/test_winograd_gpu.py > gpurun_out/wino_tests_$1.log 2>&1 &&
timeout -k 10 300 python -u scripts/prof_winograd.py 1024 > gpurun_out/wino_prof_$1.log 2>&1 &&
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu tests/test_nn_gpu.py -k "trunk" > gpurun_out/wino_trunk_$1.log 2>&1 &&
timeout -k 10 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_act_full_gpu.py > gpurun_out/wino_act_full_$1.log 2>&1
