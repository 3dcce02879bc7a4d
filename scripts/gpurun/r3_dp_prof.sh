#!/bin/bash
# the fp32 DP x2048 line after the encoder fix, deterministic on / off
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 400 python3 -u scripts/bench_policy.py DiffusionPolicy --num_envs 2048 --precision fp32 --steps 24 --warmup 24 > gpurun_out/dp_det.log 2>&1 || exit 1
RMBX_DP_DETERMINISTIC=0 timeout -k 10 400 python3 -u scripts/bench_policy.py DiffusionPolicy --num_envs 2048 --precision fp32 --steps 24 --warmup 24 > gpurun_out/dp_nondet.log 2>&1
