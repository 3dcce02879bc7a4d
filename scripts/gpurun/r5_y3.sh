#!/bin/bash
# front-kernel launch LDS padded to spread the envs evenly over CUs and rounds (RMBX_FRONT_BALANCE,
# default 1) vs the plain need (0): cable 1024 / 2048, Pick 1024, one process per setting, twice;
# engine tests
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
L=gpurun_out/r5_y3_front_balance_ab.log
for r in 1 2; do
  for b in 0 1; do
    echo "== balance $b cable 1024" >> $L
    RMBX_FRONT_BALANCE=$b timeout -k 10 200 python -u scripts/prof_physics.py >> $L 2>&1 || exit 1
    echo "== balance $b pick 1024" >> $L
    RMBX_FRONT_BALANCE=$b timeout -k 10 200 python -u scripts/prof_physics.py 1024 --env pick >> $L 2>&1 || exit 1
    echo "== balance $b cable 2048" >> $L
    RMBX_FRONT_BALANCE=$b timeout -k 10 200 python -u scripts/prof_physics.py 2048 >> $L 2>&1 || exit 1
  done
done
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_engine_gpu.py tests/test_insert_gpu.py > gpurun_out/r5_y3_tests.log 2>&1 || { tail -30 gpurun_out/r5_y3_tests.log; exit 1; }
tail -2 gpurun_out/r5_y3_tests.log
