# Winograd f32 conv per-shape profile with phase skips
# usage: bash scripts/gpurun/wino_prof.sh <tag>
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out &&
timeout -k 10 200 python -u -m pytest -x -q --timeout 100 --timeout-method thread -m gpu tests/test_winograd_gpu.py > gpurun_out/wino_tests_$1.log 2>&1 &&
timeout -k 10 400 python -u scripts/prof_winograd.py 1024 > gpurun_out/wino_prof_$1.log 2>&1
