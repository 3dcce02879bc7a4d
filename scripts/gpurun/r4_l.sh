#!/bin/bash
# round 4 box l: f16x3 GEMM with three LDS stages + the producer / consumer form -- tests, A/Bs,
# phase skips, ACT parity, the default bench
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gemm_gpu.py > gpurun_out/r4_l_gemm_tests.log 2>&1 || exit 1
timeout -k 10 300 python -u scripts/prof_gemm_pc.py > gpurun_out/r4_l_gemm_pc_ab.log 2>&1 || exit 1
timeout -k 10 300 python -u scripts/prof_gemm_h3_phases.py > gpurun_out/r4_l_gemm_phases.log 2>&1 || exit 1
timeout -k 10 600 python -u -m pytest -x -v -s --timeout 380 --timeout-method thread tests/test_act_batch_gpu.py tests/test_act_full_gpu.py > gpurun_out/r4_l_act_tests.log 2>&1 || exit 1
timeout -k 10 400 python -u bench.py --no_cpu_baseline --no_bf16_secondary > gpurun_out/r4_l_bench.json.log 2> gpurun_out/r4_l_bench.err || exit 1
RMBX_GEMM_PC=1 timeout -k 10 400 python -u bench.py --no_cpu_baseline --no_bf16_secondary > gpurun_out/r4_l_bench_pc.json.log 2> gpurun_out/r4_l_bench_pc.err
