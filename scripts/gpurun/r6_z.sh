#!/bin/bash
# round-6: configs 4 / 5 with the render cache off / on (one box)
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
L=gpurun_out/r6z_c45_render_cache_ab.log
: > $L
for v in 0 1; do
  echo "== RMBX_RENDER_CACHE=$v" >> $L
  RMBX_RENDER_CACHE=$v timeout -k 10 400 python scripts/bench_policy.py DiffusionPolicy --num_envs 2048 --precision fp32 2>&1 | tail -1 >> $L || exit 1
  RMBX_RENDER_CACHE=$v timeout -k 10 300 python scripts/bench_policy.py DiffusionPolicy3d --num_envs 1024 --precision fp32 --tactile 2>&1 | tail -1 >> $L || exit 1
done
cat $L
