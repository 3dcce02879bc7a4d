#!/bin/bash
# Newton-path diagnostic, then the rest of r5_a (attention / info / shard tests, bench with phases)
set -o pipefail
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out
timeout -k 10 300 python -u scripts/diag_newton.py > gpurun_out/r5_b_newton.log 2>&1 || { echo "diag rc=$?"; tail -20 gpurun_out/r5_b_newton.log; exit 1; }
timeout -k 10 600 python -u -m pytest -v --timeout 300 --timeout-method thread -m gpu \
  tests/test_attention_gpu.py tests/test_env_info_gpu.py tests/test_shard_gpu.py tests/test_native_abi.py \
  > gpurun_out/r5_b_tests.log 2>&1 || { echo "tests rc=$?"; tail -30 gpurun_out/r5_b_tests.log; }
tail -3 gpurun_out/r5_b_tests.log
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no_bf16_secondary --no_cpu_baseline \
  > gpurun_out/r5_b_bench.json.log 2> gpurun_out/r5_b_bench.err || { echo "bench rc=$?"; tail -20 gpurun_out/r5_b_bench.err; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/r5_b_bench.json.log'));print(d['value'],d['ms_per_step'],d['policy_inference_us_per_call'],d['physics_kernel_ms']);print(json.dumps(d.get('phases')))"
