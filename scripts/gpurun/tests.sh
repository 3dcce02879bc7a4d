# usage: bash scripts/gpurun/tests.sh <pytest args...>   (GPU tests into gpurun_out/tests.log)
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out &&
timeout -k 10 600 python -u -m pytest -x -v --timeout 200 --timeout-method thread "$@" > gpurun_out/tests.log 2>&1
