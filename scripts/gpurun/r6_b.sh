#!/bin/bash
# full GPU suite, then the physics A/B at 512 envs (solver 2 blocks per CU vs 4) and 1024
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest -v -s --timeout 300 --timeout-method thread -m gpu tests/ > gpurun_out/r6b_gpu_tests.log 2>&1
rc=$?
grep -E "passed|failed" gpurun_out/r6b_gpu_tests.log | tail -2
grep -E "^FAILED|^ERROR" gpurun_out/r6b_gpu_tests.log | head -20
[ $rc -le 1 ] || exit $rc
for cfg in "512 auto" "512 4" "1024 auto"; do
  set -- $cfg
  if [ "$2" = auto ]; then unset RMBX_SOLVER_MINB; else export RMBX_SOLVER_MINB=$2; fi
  echo "== n=$1 minb=$2" >> gpurun_out/r6b_solver_ab.log
  timeout -k 10 120 python -u scripts/prof_physics.py $1 >> gpurun_out/r6b_solver_ab.log 2>&1 || exit 1
done
unset RMBX_SOLVER_MINB
cat gpurun_out/r6b_solver_ab.log | grep -v "^$" | tail -40
exit $rc
