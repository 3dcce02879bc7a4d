#!/bin/bash
# round 4 box i: GEMM with the A loads and W DMA hand-counted (single-accumulator f16x3); u8 stem
# f16 form -- tests, A/Bs, phase skips, ACT parity, the default bench
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gemm_gpu.py > gpurun_out/r4_i_gemm_tests.log 2>&1 || exit 1
timeout -k 10 300 python -u scripts/prof_gemm_h3.py > gpurun_out/r4_i_gemm_h3_ab.log 2>&1 || exit 1
timeout -k 10 300 python -u scripts/prof_gemm_h3_phases.py > gpurun_out/r4_i_gemm_phases.log 2>&1 || exit 1
timeout -k 10 300 python -u scripts/prof_stem_u8_forms.py > gpurun_out/r4_i_stem_forms.log 2>&1 || exit 1
timeout -k 10 600 python -u -m pytest -x -v -s --timeout 380 --timeout-method thread tests/test_nn_gpu.py tests/test_act_batch_gpu.py tests/test_act_full_gpu.py > gpurun_out/r4_i_act_tests.log 2>&1 || exit 1
timeout -k 10 600 python -u bench.py --no_cpu_baseline > gpurun_out/r4_i_bench.json.log 2> gpurun_out/r4_i_bench.err
