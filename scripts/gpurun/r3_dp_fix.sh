#!/bin/bash
# DP encoder on rmbx kernels (direct stem, x6 convs / keypoint conv), the two-camera ACT test, GEMM variants, C4 fp32 line
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 600 python3 -u -m pytest -x -v -s --timeout 300 --timeout-method thread tests/test_gemm_gpu.py tests/test_multicam_gpu.py tests/test_diffusion_policy_gpu.py tests/test_policy_parity_gpu.py tests/test_pick_workloads_gpu.py > gpurun_out/dp_fix_tests.log 2>&1 || exit 1
bash scripts/gpurun/r3_gemm_var.sh || exit 1
timeout -k 10 420 python3 -u scripts/bench_policy.py DiffusionPolicy --num_envs 2048 --precision fp32 --steps 48 --warmup 24 > gpurun_out/r3x6_bp_DiffusionPolicy_num_envs_2048_precision_fp32.log 2>&1
