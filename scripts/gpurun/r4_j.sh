#!/bin/bash
# round 4 box j: the f16x3 GEMM's 64-column tile -- tests, layer-1 conv A/B vs the fused Winograd,
# bench A/B of the stride-1 64-channel convs on the GEMM
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gemm_gpu.py > gpurun_out/r4_j_gemm_tests.log 2>&1 || exit 1
timeout -k 10 300 python -u scripts/prof_conv64_gemm.py > gpurun_out/r4_j_conv64_ab.log 2>&1 || exit 1
timeout -k 10 400 python -u bench.py --no_cpu_baseline --no_bf16_secondary > gpurun_out/r4_j_bench_default.json.log 2> gpurun_out/r4_j_bench_default.err || exit 1
RMBX_S1_GEMM=64,128 timeout -k 10 400 python -u bench.py --no_cpu_baseline --no_bf16_secondary > gpurun_out/r4_j_bench_s1gemm64.json.log 2> gpurun_out/r4_j_bench_s1gemm64.err
