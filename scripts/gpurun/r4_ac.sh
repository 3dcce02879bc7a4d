#!/bin/bash
# f16x3 attention: 4-wave blocks (two per CU) vs 5-wave blocks; tests with both
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
RMBX_ATTN_WAVES=4 timeout -k 10 300 python -u -m pytest -v --timeout 120 --timeout-method thread -m gpu tests/test_attention_gpu.py > gpurun_out/r4_ac_attn_tests_w4.log 2>&1 || exit 1
timeout -k 10 200 python -u scripts/prof_attn_forms.py > gpurun_out/r4_ac_attn_forms.log 2>&1 || exit 1
