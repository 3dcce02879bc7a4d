#!/bin/bash
# round 3 close: u8 stem with DPP pooling as the default -- stem + renderer tests, ACT production
# parity, smoke, the default bench
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -v --timeout 250 --timeout-method thread tests/test_nn_gpu.py -k "stem or render_s2d" tests/test_multicam_gpu.py > gpurun_out/r3_dpp_tests.log 2>&1 || exit 1
timeout -k 10 400 python -u -m pytest -x -v -s --timeout 380 --timeout-method thread tests/test_act_full_gpu.py > gpurun_out/r3_dpp_act_full.log 2>&1 || exit 1
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r3_dpp_smoke.log 2>&1 || exit 1
timeout -k 10 600 python -u bench.py > gpurun_out/r3_bench_dpp.json.log 2> gpurun_out/r3_bench_dpp.err
