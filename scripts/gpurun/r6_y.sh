#!/bin/bash
# round-6: FFN pair back to back vs row chunks on two streams
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/r6y
timeout -k 10 300 python -u scripts/prof_ffn_overlap.py > gpurun_out/r6y/ab.log 2>&1 || { tail -20 gpurun_out/r6y/ab.log; exit 1; }
cat gpurun_out/r6y/ab.log
