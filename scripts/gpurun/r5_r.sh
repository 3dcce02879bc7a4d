#!/bin/bash
# A/B: the 256 / 512-channel stride-1 convs on the patch-staged f16x3 conv instead of the explicit
# Winograd F(4x4) (RMBX_S1_PATCH), same box, driver-shaped bench
set -o pipefail
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out
for v in "64,128" "64,128,256" "64,128,256,512"; do
  RMBX_S1_PATCH=$v timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no_bf16_secondary --no_cpu_baseline \
    > gpurun_out/r5_r_bench_$v.json.log 2> gpurun_out/r5_r_bench.err || { echo "bench rc=$?"; tail -20 gpurun_out/r5_r_bench.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/r5_r_bench_$v.json.log'));print('$v',d['value'],d['ms_per_step'],d['policy_inference_us_per_call'],d['roofline']['frac'],d['roofline_conv3x3']['frac'])"
done
RMBX_S1_PATCH=64,128,256,512 timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_act_full_gpu.py tests/test_act_batch_gpu.py > gpurun_out/r5_r_tests.log 2>&1; tail -2 gpurun_out/r5_r_tests.log
