cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out &&
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_nn_gpu.py -k act > gpurun_out/act_tests.log 2>&1 &&
timeout -k 10 300 python scripts/prof_act_cross.py > gpurun_out/act_cross.log 2>&1
