#!/bin/bash
# round 4 box o: the f16x3 GEMM's 256-wide tile -- tests (bitwise vs the default tile), A/B, bench A/B
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gemm_gpu.py > gpurun_out/r4_o_gemm_tests.log 2>&1 || exit 1
timeout -k 10 300 python -u scripts/prof_gemm_wide.py > gpurun_out/r4_o_gemm_wide_ab.log 2>&1 || exit 1
timeout -k 10 400 python -u bench.py --no_cpu_baseline --no_bf16_secondary > gpurun_out/r4_o_bench.json.log 2> gpurun_out/r4_o_bench.err || exit 1
RMBX_GEMM_WIDE=1 timeout -k 10 400 python -u bench.py --no_cpu_baseline --no_bf16_secondary > gpurun_out/r4_o_bench_wide.json.log 2> gpurun_out/r4_o_bench_wide.err
