#!/bin/bash
# round 4 box m: f16x3 GEMM schedules -- phase skips (waits fixed) with the two-stage variant, the
# producer / consumer form, ACT parity, benches default vs producer / consumer
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gemm_gpu.py > gpurun_out/r4_m_gemm_tests.log 2>&1 || exit 1
timeout -k 10 300 python -u scripts/prof_gemm_h3_phases.py > gpurun_out/r4_m_gemm_phases.log 2>&1 || exit 1
timeout -k 10 600 python -u -m pytest -x -v -s --timeout 380 --timeout-method thread tests/test_act_batch_gpu.py tests/test_act_full_gpu.py > gpurun_out/r4_m_act_tests.log 2>&1 || exit 1
timeout -k 10 400 python -u bench.py --no_cpu_baseline --no_bf16_secondary > gpurun_out/r4_m_bench.json.log 2> gpurun_out/r4_m_bench.err || exit 1
RMBX_GEMM_PC=1 timeout -k 10 400 python -u bench.py --no_cpu_baseline --no_bf16_secondary > gpurun_out/r4_m_bench_pc.json.log 2> gpurun_out/r4_m_bench_pc.err
