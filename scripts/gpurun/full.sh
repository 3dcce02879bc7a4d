cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out &&
timeout -k 10 900 python -u -m pytest -v --timeout 300 --timeout-method thread -m gpu tests > gpurun_out/full_tests.log 2>&1 &&
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
