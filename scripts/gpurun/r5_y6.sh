#!/bin/bash
# fused GroupNorm + Mish in the DP / DP3 UNet (RMBX_UNET_FUSED_GN=1, default) vs torch's ops (0):
# GPU tests, then C4 and C5 A/B, one process per setting
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_groupnorm_gpu.py tests/test_policy_parity_gpu.py tests/test_pick_workloads_gpu.py > gpurun_out/r5_y6_tests.log 2>&1 || { tail -30 gpurun_out/r5_y6_tests.log; exit 1; }
tail -2 gpurun_out/r5_y6_tests.log
L=gpurun_out/r5_y6_unet_gn_ab.log
for r in 1 2; do
  for f in 0 1; do
    echo "== fused_gn $f C4" >> $L
    RMBX_UNET_FUSED_GN=$f timeout -k 10 400 python scripts/bench_policy.py DiffusionPolicy --num_envs 2048 --precision fp32 2>&1 | tail -1 >> $L || exit 1
    echo "== fused_gn $f C5" >> $L
    RMBX_UNET_FUSED_GN=$f timeout -k 10 300 python scripts/bench_policy.py DiffusionPolicy3d --num_envs 1024 --precision fp32 --tactile 2>&1 | tail -1 >> $L || exit 1
  done
done
