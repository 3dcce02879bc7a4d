#!/bin/bash
# configs 4 / 5 (BASELINE.json) on the round-5 tree: DiffusionPolicy x2048 and DP3 x1024 + tactile,
# MujocoUR5ePick, fp32 (the reference's precision)
set -o pipefail
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out
timeout -k 10 500 python -u scripts/bench_policy.py DiffusionPolicy --num_envs 2048 --steps 24 --warmup 8 --precision fp32 \
  > gpurun_out/r5_bp_dp_2048_fp32.log 2>&1 || { echo "dp rc=$?"; tail -5 gpurun_out/r5_bp_dp_2048_fp32.log; exit 1; }
tail -2 gpurun_out/r5_bp_dp_2048_fp32.log
timeout -k 10 400 python -u scripts/bench_policy.py DiffusionPolicy3d --num_envs 1024 --tactile --precision fp32 \
  > gpurun_out/r5_bp_dp3_1024_fp32.log 2>&1 || { echo "dp3 rc=$?"; tail -5 gpurun_out/r5_bp_dp3_1024_fp32.log; exit 1; }
tail -2 gpurun_out/r5_bp_dp3_1024_fp32.log
