#!/bin/bash
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 300 python -u scripts/prof_render_cams.py > gpurun_out/r6ag_render_cams.log 2>&1 || { tail -20 gpurun_out/r6ag_render_cams.log; exit 1; }
grep -v amdgpu.ids gpurun_out/r6ag_render_cams.log
