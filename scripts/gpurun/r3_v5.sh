#!/bin/bash
# v5 GEMM epilogue default: GEMM / conv / Winograd tests, ACT parity, DP tests (determinism), bench
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 600 python3 -u -m pytest -x -v -s --timeout 300 --timeout-method thread tests/test_gemm_gpu.py tests/test_wino_x6_gpu.py tests/test_act_full_gpu.py tests/test_diffusion_policy_gpu.py tests/test_multicam_gpu.py > gpurun_out/v5_tests.log 2>&1 || exit 1
timeout -k 10 200 python3 -u scripts/prof_gemm.py > gpurun_out/prof_gemm_v5.log 2>&1 || exit 1
timeout -k 10 500 python3 -u bench.py --no_cpu_baseline > gpurun_out/bench_v5.json.log 2> gpurun_out/bench_v5.err
