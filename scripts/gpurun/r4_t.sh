#!/bin/bash
# f16x3 attention with the query parts of a head paired on one XCD: tests + in-process A/B
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -v --timeout 120 --timeout-method thread -m gpu tests/test_attention_gpu.py > gpurun_out/r4_t_attn_tests.log 2>&1 || exit 1
timeout -k 10 200 python -u scripts/prof_attn_forms.py > gpurun_out/r4_t_attn_forms.log 2>&1 || exit 1
