#!/bin/bash
# round 4 box: producer/consumer Winograd F(4x4) -- equality tests, per-layer A/B -- then the full
# GPU suite
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_winograd_gpu.py > gpurun_out/r4_wino_spec_tests.log 2>&1 || exit 1
timeout -k 10 300 python -u scripts/prof_wino4_spec.py 1024 > gpurun_out/r4_wino4_spec_ab.log 2>&1 || exit 1
timeout -k 10 900 python -u -m pytest -v --timeout 300 --timeout-method thread -m gpu tests/ > gpurun_out/r4_full_gpu_tests_d.log 2>&1
