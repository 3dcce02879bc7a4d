#!/bin/bash
# round 3 (u8 stem tree): stem timing of both layouts, the end-of-round measurement (full GPU
# suite, smoke, default bench, bench under rocprofv3)
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 120 python -u scripts/prof_stem_u8.py > gpurun_out/r3_u8_stem_prof.log 2>&1 || exit 1
RMBX_STEM_U8_LAYOUT=10 timeout -k 10 120 python -u scripts/prof_stem_u8.py >> gpurun_out/r3_u8_stem_prof.log 2>&1 || exit 1
bash scripts/gpurun/r3_final.sh $1 || exit $?
