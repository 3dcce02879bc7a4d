#!/bin/bash
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_groupnorm_gpu.py tests/test_policy_parity_gpu.py > gpurun_out/r5_y7_tests.log 2>&1 || { tail -30 gpurun_out/r5_y7_tests.log; exit 1; }
tail -2 gpurun_out/r5_y7_tests.log
for r in 1 2; do
  timeout -k 10 400 python scripts/bench_policy.py DiffusionPolicy --num_envs 2048 --precision fp32 2>&1 | tail -1 >> gpurun_out/r5_y7_bp.log || exit 1
  timeout -k 10 300 python scripts/bench_policy.py DiffusionPolicy3d --num_envs 1024 --precision fp32 --tactile 2>&1 | tail -1 >> gpurun_out/r5_y7_bp.log || exit 1
done
