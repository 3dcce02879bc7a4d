#!/bin/bash
# round 4 box f: the f16x3 GEMM form -- GEMM tests (both forms), f16x3 vs bf16x6 A/B, ACT parity and
# batch invariance with f16x3 as the default, smoke, the default bench
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gemm_gpu.py > gpurun_out/r4_f_gemm_tests.log 2>&1 || exit 1
timeout -k 10 300 python -u scripts/prof_gemm_h3.py > gpurun_out/r4_f_gemm_h3_ab.log 2>&1 || exit 1
timeout -k 10 600 python -u -m pytest -x -v -s --timeout 380 --timeout-method thread tests/test_act_batch_gpu.py tests/test_act_full_gpu.py tests/test_rollout_gpu.py > gpurun_out/r4_f_act_tests.log 2>&1 || exit 1
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r4_f_smoke.log 2>&1 || exit 1
timeout -k 10 600 python -u bench.py > gpurun_out/r4_f_bench.json.log 2> gpurun_out/r4_f_bench.err
