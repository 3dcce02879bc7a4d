#!/bin/bash
# round 4 box n: f16x3 GEMM back on two LDS stages, rmbx_gemm.hip built without SLP packing --
# tests, A/B against the SLP build (same box, separate processes), producer / consumer form, bench
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gemm_gpu.py > gpurun_out/r4_n_gemm_tests.log 2>&1 || exit 1
timeout -k 10 300 python -u scripts/prof_gemm_pc.py > gpurun_out/r4_n_gemm_pc_noslp.log 2>&1 || exit 1
RMBX_LIB_VARIANT=slp timeout -k 10 300 python -u scripts/prof_gemm_pc.py > gpurun_out/r4_n_gemm_pc_slp.log 2>&1 || exit 1
timeout -k 10 300 python -u scripts/prof_gemm_h3.py > gpurun_out/r4_n_gemm_h3_ab.log 2>&1 || exit 1
timeout -k 10 600 python -u -m pytest -x -v -s --timeout 380 --timeout-method thread tests/test_act_batch_gpu.py tests/test_act_full_gpu.py > gpurun_out/r4_n_act_tests.log 2>&1 || exit 1
timeout -k 10 400 python -u bench.py --no_cpu_baseline --no_bf16_secondary > gpurun_out/r4_n_bench.json.log 2> gpurun_out/r4_n_bench.err || exit 1
RMBX_GEMM_PC=1 timeout -k 10 400 python -u bench.py --no_cpu_baseline --no_bf16_secondary > gpurun_out/r4_n_bench_pc.json.log 2> gpurun_out/r4_n_bench_pc.err
