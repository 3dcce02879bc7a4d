#!/bin/bash
# renderer register cap A/B (default vs 5 waves per SIMD), one process per library, one box
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
for v in "" render5 "" render5; do
  RMBX_LIB_VARIANT=$v timeout -k 10 200 python -u scripts/prof_render_u8.py >> gpurun_out/r4_ae_render_ab.log 2>&1 || exit 1
done
