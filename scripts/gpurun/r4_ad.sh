#!/bin/bash
# u8 -> f16 ring refill by byte permutes: stem tests, ACT u8 test, phase skips
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -v --timeout 120 --timeout-method thread -m gpu tests/test_nn_gpu.py -k stem > gpurun_out/r4_ad_stem_tests.log 2>&1 || exit 1
timeout -k 10 400 python -u -m pytest -v --timeout 300 --timeout-method thread -m gpu tests/test_act_batch_gpu.py tests/test_act_full_gpu.py > gpurun_out/r4_ad_act_tests.log 2>&1 || exit 1
timeout -k 10 200 python -u scripts/prof_stem_phases.py > gpurun_out/r4_ad_stem_phases.log 2>&1 || exit 1
