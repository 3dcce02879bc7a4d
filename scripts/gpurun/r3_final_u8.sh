#!/bin/bash
# round 3 (u8 stem tree): stem timing of both layouts, the end-of-round measurement (full GPU
# suite, smoke, default bench, bench under rocprofv3), then -- if time is left -- the GEMM
# persistent-block A/B
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 120 python -u scripts/prof_stem_u8.py > gpurun_out/r3_u8_stem_prof.log 2>&1 || exit 1
RMBX_STEM_U8_LAYOUT=10 timeout -k 10 120 python -u scripts/prof_stem_u8.py >> gpurun_out/r3_u8_stem_prof.log 2>&1 || exit 1
bash scripts/gpurun/r3_final.sh $1 || exit $?
if [ $SECONDS -lt 880 ]; then
  for v in 16 80 208; do
    echo "== RMBX_GEMM_VAR=$v" >> gpurun_out/r3_gemm_persist.log
    RMBX_GEMM_VAR=$v timeout -k 10 90 python3 -u scripts/prof_gemm.py >> gpurun_out/r3_gemm_persist.log 2>&1 || exit 1
  done
fi
