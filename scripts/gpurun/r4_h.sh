#!/bin/bash
# round 4 box h: f16x3 GEMM phase skips; GEMM + conv + ACT tests with the stride-1 128-channel convs
# on the implicit GEMM (new default); the default bench
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 300 python -u scripts/prof_gemm_h3_phases.py > gpurun_out/r4_h_gemm_phases.log 2>&1 || exit 1
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gemm_gpu.py tests/test_nn_gpu.py > gpurun_out/r4_h_gemm_nn_tests.log 2>&1 || exit 1
timeout -k 10 600 python -u -m pytest -x -v -s --timeout 380 --timeout-method thread tests/test_act_batch_gpu.py tests/test_act_full_gpu.py > gpurun_out/r4_h_act_tests.log 2>&1 || exit 1
timeout -k 10 600 python -u bench.py > gpurun_out/r4_h_bench.json.log 2> gpurun_out/r4_h_bench.err
