#!/bin/bash
# the diffusion UNet's fp32 GEMMs on rmbx_linear_f32x6: DP / DP3 tests, then C4 / C5 fp32 lines
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 600 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_diffusion_policy_gpu.py tests/test_policy_parity_gpu.py tests/test_pick_workloads_gpu.py > gpurun_out/dp_x6_tests.log 2>&1 || exit 1
for cfg in "DiffusionPolicy3d --num_envs 1024 --tactile --precision fp32" "DiffusionPolicy --num_envs 2048 --precision fp32"; do
  tag=$(echo $cfg | tr ' ' '_' | tr -d '-')
  timeout -k 10 420 python3 -u scripts/bench_policy.py $cfg --steps 48 --warmup 24 > gpurun_out/r3x6_bp_$tag.log 2>&1 || exit 1
done
