#!/bin/bash
# renderer vs oracle test, then the driver's bench command (per-phase split) with meshes rendered
set -o pipefail
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out
timeout -k 10 300 python -u scripts/prof_render_mesh.py > gpurun_out/r5_f_render.log 2>&1 && cat gpurun_out/r5_f_render.log
timeout -k 10 600 python -u -m pytest -v --timeout 500 --timeout-method thread -m gpu -s \
  tests/test_render_gpu.py > gpurun_out/r5_f_tests.log 2>&1 || { echo "tests rc=$?"; }
grep -E "PASS|FAIL|mesh pixels|passed|failed|Error" gpurun_out/r5_f_tests.log | tail -30
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no_bf16_secondary --no_cpu_baseline \
  > gpurun_out/r5_f_bench.json.log 2> gpurun_out/r5_f_bench.err || { echo "bench rc=$?"; tail -20 gpurun_out/r5_f_bench.err; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/r5_f_bench.json.log'));print(d['value'],d['ms_per_step'],d['policy_inference_us_per_call'],d['physics_kernel_ms']);print(json.dumps(d.get('phases')))"
