#!/bin/bash
# round-6: renderer phase skips on the rollout's front-camera call
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/r6s
O=gpurun_out/r6s
timeout -k 10 300 python -u scripts/prof_render_phases.py > $O/phases.log 2>&1 || { tail -20 $O/phases.log; exit 1; }
cat $O/phases.log
