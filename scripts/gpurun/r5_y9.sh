#!/bin/bash
# GroupNorm + Mish reading the conv GEMM [B, T, C] rows (RMBX_UNET_GN_ROWS=1, default: no transpose copy)
# vs after the transpose copy (0): tests, then C4 / C5 A/B on one box
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_groupnorm_gpu.py tests/test_policy_parity_gpu.py tests/test_pick_workloads_gpu.py > gpurun_out/r5_y9_tests.log 2>&1 || { tail -30 gpurun_out/r5_y9_tests.log; exit 1; }
tail -2 gpurun_out/r5_y9_tests.log
L=gpurun_out/r5_y9_gn_rows_ab.log
for r in 1 2; do
  for v in 0 1; do
    echo "== gn_rows '$v'" >> $L
    RMBX_UNET_GN_ROWS=$v timeout -k 10 400 python scripts/bench_policy.py DiffusionPolicy --num_envs 2048 --precision fp32 2>&1 | tail -1 >> $L || exit 1
    RMBX_UNET_GN_ROWS=$v timeout -k 10 300 python scripts/bench_policy.py DiffusionPolicy3d --num_envs 1024 --precision fp32 --tactile 2>&1 | tail -1 >> $L || exit 1
  done
done
