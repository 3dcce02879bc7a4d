#!/bin/bash
# round 4: the Hessian as the full build +/- the net row change (one hsave write per solve), one code path
# after the gradient (no spills) -- engine parity tests, physics time vs at-94484c1, PMC traffic
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu tests/test_engine_gpu.py tests/test_insert_gpu.py tests/test_pick_gpu.py tests/test_bad_state_gpu.py > gpurun_out/r4_al_engine_tests.log 2>&1 || exit 1
for v in "" at-94484c1 "" at-94484c1; do
  echo "== variant $v" >> gpurun_out/r4_al_solver_ab.log
  RMBX_LIB_VARIANT=$v timeout -k 10 200 python3 -u scripts/prof_physics.py 1024 >> gpurun_out/r4_al_solver_ab.log 2>&1 || exit 1
done
mkdir -p gpurun_out/r4_al_pmc &&
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d gpurun_out/r4_al_pmc/pmc_fetch -o run -- python3 scripts/prof_physics.py --calib > gpurun_out/r4_al_pmc/fetch.log 2>&1 &&
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d gpurun_out/r4_al_pmc/pmc_write -o run -- python3 scripts/prof_physics.py --calib > gpurun_out/r4_al_pmc/write.log 2>&1 || exit 1
