#!/bin/bash
# round 3: rmbx_linear_f32x6 tests, per-shape timing, ACT parity with the x6 GEMMs, bench
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 300 python3 -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gemm_gpu.py > gpurun_out/gemm_tests.log 2>&1 && \
timeout -k 10 200 python3 -u scripts/prof_gemm.py > gpurun_out/prof_gemm.log 2>&1 && \
timeout -k 10 400 python3 -u -m pytest -x -v -s --timeout 380 --timeout-method thread tests/test_act_full_gpu.py > gpurun_out/act_full_x6.log 2>&1 && \
timeout -k 10 400 python3 -u bench.py --no_cpu_baseline > gpurun_out/bench_x6.json.log 2> gpurun_out/bench_x6.err
