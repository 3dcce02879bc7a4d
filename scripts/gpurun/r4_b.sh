#!/bin/bash
# round 4 box 2: batch-invariant ACT + info tests, GEMM stagger A/B, full GPU suite, smoke, bench
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v -s --timeout 300 --timeout-method thread tests/test_act_batch_gpu.py tests/test_env_info_gpu.py > gpurun_out/r4_new_tests_b.log 2>&1 || exit 1
timeout -k 10 300 python -u scripts/prof_gemm_persist.py > gpurun_out/r4_gemm_stagger_ab.log 2>&1 || exit 1
timeout -k 10 900 python -u -m pytest -v --timeout 300 --timeout-method thread -m gpu tests/ > gpurun_out/r4_full_gpu_tests_b.log 2>&1
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r4_smoke_b.log 2>&1 || exit 1
timeout -k 10 600 python -u bench.py > gpurun_out/r4_bench_b.json.log 2> gpurun_out/r4_bench_b.err
