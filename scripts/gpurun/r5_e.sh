#!/bin/bash
# render timing (mesh visibility pass), renderer vs oracle test
set -o pipefail
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out
timeout -k 10 300 python -u scripts/prof_render_mesh.py > gpurun_out/r5_e_render.log 2>&1 || { echo "render rc=$?"; tail -20 gpurun_out/r5_e_render.log; exit 1; }
cat gpurun_out/r5_e_render.log
timeout -k 10 600 python -u -m pytest -v --timeout 500 --timeout-method thread -m gpu -s \
  tests/test_render_gpu.py tests/test_env_info_gpu.py tests/test_image_gpu.py > gpurun_out/r5_e_tests.log 2>&1 || { echo "tests rc=$?"; }
grep -E "PASS|FAIL|mesh pixels|passed|failed|Error" gpurun_out/r5_e_tests.log | tail -30
