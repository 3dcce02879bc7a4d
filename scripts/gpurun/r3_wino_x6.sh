#!/bin/bash
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
export MIOPEN_DEBUG_CONV_DIRECT_NAIVE_CONV_FWD=0
timeout -k 10 300 python3 -u -m pytest -x -q -s --timeout 200 --timeout-method thread tests/test_wino_x6_gpu.py tests/test_gemm_gpu.py > gpurun_out/wino_x6_tests.log 2>&1 && \
timeout -k 10 400 python3 -u scripts/prof_wino_x6.py > gpurun_out/prof_wino_x6.log 2>&1 && \
timeout -k 10 500 python3 -u -m pytest -x -v -s --timeout 480 --timeout-method thread tests/test_act_full_gpu.py > gpurun_out/act_full_winox6.log 2>&1 && \
timeout -k 10 500 python3 -u bench.py --no_cpu_baseline > gpurun_out/bench_winox6.json.log 2> gpurun_out/bench_winox6.err
