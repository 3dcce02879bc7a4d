#!/bin/bash
# patch conv: the two-blocks-per-CU configuration (RMBX_CONVP_CFG=1) -- tests for both, A/B
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -v --timeout 120 --timeout-method thread -m gpu tests/test_convp_gpu.py > gpurun_out/r4_x_convp_tests.log 2>&1 || exit 1
RMBX_CONVP_CFG=1 timeout -k 10 300 python -u -m pytest -v --timeout 120 --timeout-method thread -m gpu tests/test_convp_gpu.py > gpurun_out/r4_x_convp_tests_cfg1.log 2>&1 || exit 1
timeout -k 10 300 python -u scripts/prof_convp.py > gpurun_out/r4_x_convp_ab.log 2>&1 || exit 1
