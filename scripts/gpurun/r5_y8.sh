#!/bin/bash
# GroupNorm + Mish: register-resident spans (default build) vs the three-pass kernel (at-HEAD), C4 / C5
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
L=gpurun_out/r5_y8_gn_reg_ab.log
for r in 1 2; do
  for v in at-HEAD ""; do
    echo "== variant '$v'" >> $L
    RMBX_LIB_VARIANT=$v timeout -k 10 400 python scripts/bench_policy.py DiffusionPolicy --num_envs 2048 --precision fp32 2>&1 | tail -1 >> $L || exit 1
    RMBX_LIB_VARIANT=$v timeout -k 10 300 python scripts/bench_policy.py DiffusionPolicy3d --num_envs 1024 --precision fp32 --tactile 2>&1 | tail -1 >> $L || exit 1
  done
done
