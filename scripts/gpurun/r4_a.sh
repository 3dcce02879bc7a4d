#!/bin/bash
# round 4 first box: the new production-batch / info-contract / GEMM tests, the persistent-GEMM A/B,
# the padded Winograd F(4x4) LDS images, then the full GPU suite and smoke
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -v -s --timeout 200 --timeout-method thread tests/test_gemm_gpu.py > gpurun_out/r4_gemm_tests.log 2>&1 || exit 1
timeout -k 10 200 python -u scripts/prof_gemm_persist.py > gpurun_out/r4_gemm_persist_ab.log 2>&1 || exit 1
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_winograd_gpu.py tests/test_wino_x6_gpu.py > gpurun_out/r4_wino_tests.log 2>&1 || exit 1
timeout -k 10 300 python -u scripts/prof_winograd4.py 1024 --vars 6,16 > gpurun_out/r4_wino4_padded.log 2>&1 || exit 1
timeout -k 10 600 python -u -m pytest -x -v -s --timeout 300 --timeout-method thread tests/test_act_batch_gpu.py tests/test_env_info_gpu.py > gpurun_out/r4_new_tests.log 2>&1 || exit 1
timeout -k 10 900 python -u -m pytest -v --timeout 300 --timeout-method thread -m gpu tests/ > gpurun_out/r4_full_gpu_tests_a.log 2>&1 || exit 1
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r4_smoke_a.log 2>&1
