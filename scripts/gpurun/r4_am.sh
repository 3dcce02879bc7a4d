#!/bin/bash
# round 4: Hessian entries with a multiply-shift e / NVP -- engine parity tests, physics time vs
# at-1877bac (alternating, one process each), PMC traffic
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu tests/test_engine_gpu.py tests/test_insert_gpu.py tests/test_pick_gpu.py tests/test_bad_state_gpu.py > gpurun_out/r4_am_engine_tests.log 2>&1 || exit 1
for v in "" at-1877bac "" at-1877bac; do
  echo "== variant $v" >> gpurun_out/r4_am_solver_ab.log
  RMBX_LIB_VARIANT=$v timeout -k 10 200 python3 -u scripts/prof_physics.py 1024 >> gpurun_out/r4_am_solver_ab.log 2>&1 || exit 1
done
mkdir -p gpurun_out/r4_am_pmc &&
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d gpurun_out/r4_am_pmc/pmc_fetch -o run -- python3 scripts/prof_physics.py --calib > gpurun_out/r4_am_pmc/fetch.log 2>&1 &&
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d gpurun_out/r4_am_pmc/pmc_write -o run -- python3 scripts/prof_physics.py --calib > gpurun_out/r4_am_pmc/write.log 2>&1 || exit 1
