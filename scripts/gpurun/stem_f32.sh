# f32 stem: parity tests, the production-size ACT fp32 test, and the stem profile
# usage: bash scripts/gpurun/stem_f32.sh <tag>
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out &&
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu tests/test_nn_gpu.py -k "stem" > gpurun_out/stem_tests_$1.log 2>&1 &&
timeout -k 10 120 python scripts/prof_stem.py 1024 > gpurun_out/stem_prof_$1.log 2>&1 &&
timeout -k 10 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_act_full_gpu.py > gpurun_out/act_full_$1.log 2>&1
