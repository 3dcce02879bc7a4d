#!/bin/bash
# physics env-step time per solver occupancy variant (RMBX_SOLVER_MINB), 1024 Cable envs
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
for v in 4 3 2 4; do
  echo "== RMBX_SOLVER_MINB=$v" >> gpurun_out/solver_minb.log
  RMBX_SOLVER_MINB=$v timeout -k 10 200 python3 -u scripts/prof_physics.py 1024 >> gpurun_out/solver_minb.log 2>&1 || exit 1
done
