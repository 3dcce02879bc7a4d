#!/bin/bash
# round 4: f16x3 attention with its staging offsets recomputed per tile (174 registers, was 215)
# -- attention tests, then the ACT attention shapes per library (default / attn3 = 3 waves per
# SIMD / at-c196881 = the commit before), alternating, one process each
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu tests/test_attention_gpu.py > gpurun_out/r4_aj_attn_tests.log 2>&1 || exit 1
RMBX_LIB_VARIANT=attn3 timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu tests/test_attention_gpu.py > gpurun_out/r4_aj_attn3_tests.log 2>&1 || exit 1
for v in "" attn3 at-c196881 "" attn3 at-c196881; do
  echo "== variant $v" >> gpurun_out/r4_aj_attn_ab.log
  RMBX_LIB_VARIANT=$v timeout -k 10 200 python -u scripts/prof_attn_forms.py >> gpurun_out/r4_aj_attn_ab.log 2>&1 || exit 1
done
