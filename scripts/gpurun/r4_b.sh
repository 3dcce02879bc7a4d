#!/bin/bash
# round 4 box 2: batch-invariant ACT + info tests, GEMM stagger A/B, the three-wave solver
# (RMBX_SOLVER_THREADS=192: engine parity tests with it, physics time per variant), smoke, bench
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v -s --timeout 300 --timeout-method thread tests/test_act_batch_gpu.py tests/test_env_info_gpu.py > gpurun_out/r4_new_tests_b.log 2>&1 || exit 1
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gemm_gpu.py > gpurun_out/r4_gemm_tests_b.log 2>&1 || exit 1
timeout -k 10 400 python -u scripts/prof_gemm_persist.py > gpurun_out/r4_gemm_stagger_ab.log 2>&1 || exit 1
RMBX_SOLVER_THREADS=192 timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_engine_gpu.py tests/test_insert_gpu.py tests/test_pick_gpu.py tests/test_bad_state_gpu.py > gpurun_out/r4_solver192_tests.log 2>&1 || exit 1
for v in 256 192 256 192; do
  echo "== RMBX_SOLVER_THREADS=$v" >> gpurun_out/r4_solver_threads.log
  RMBX_SOLVER_THREADS=$v timeout -k 10 200 python3 -u scripts/prof_physics.py 1024 >> gpurun_out/r4_solver_threads.log 2>&1 || exit 1
done
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r4_smoke_b.log 2>&1 || exit 1
timeout -k 10 600 python -u bench.py > gpurun_out/r4_bench_b.json.log 2> gpurun_out/r4_bench_b.err
