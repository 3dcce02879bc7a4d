#!/bin/bash
# round-6: phase skips of the pipelined DMA attention
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/r6o
O=gpurun_out/r6o
timeout -k 10 200 python -u scripts/prof_attn_phases.py > $O/phases.log 2>&1 || { tail -20 $O/phases.log; exit 1; }
cat $O/phases.log
