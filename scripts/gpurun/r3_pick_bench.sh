#!/bin/bash
# round 3: the UNet capture diagnostic, then configs 4 / 5 as bench_policy lines (bf16 and fp32)
set -o pipefail
mkdir -p gpurun_out
MIOPEN_ENABLE_LOGGING=1 timeout -k 10 240 python -u scripts/diag_conv1d_capture.py 1024 --unet > gpurun_out/r3_unet_capture.log 2>&1
echo "unet diag rc=$?"
for cfg in "DiffusionPolicy --num_envs 2048 --precision bf16" "DiffusionPolicy3d --num_envs 1024 --tactile --precision bf16" \
           "DiffusionPolicy3d --num_envs 1024 --tactile --precision fp32" "DiffusionPolicy --num_envs 2048 --precision fp32"; do
  tag=$(echo $cfg | tr ' ' '_' | tr -d '-')
  timeout -k 10 420 python -u scripts/bench_policy.py $cfg --steps 48 --warmup 24 > gpurun_out/r3_bp_$tag.log 2>&1
  rc=$?
  echo "$cfg rc=$rc"
  [ $rc -ne 0 ] && exit $rc
done
exit 0
