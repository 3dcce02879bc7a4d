#!/bin/bash
# render timing (projected-box culling, prefetching traversal; occupancy variants), renderer vs
# oracle test, engine tests (box-box edge support fix, Newton path)
set -o pipefail
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out
timeout -k 10 300 python -u scripts/prof_render_mesh.py > gpurun_out/r5_d_render.log 2>&1 || { echo "render rc=$?"; tail -20 gpurun_out/r5_d_render.log; exit 1; }
for v in rmeshw5 rmeshw6; do
  RENDER_ONLY_ASSET=1 RMBX_LIB_VARIANT=$v timeout -k 10 300 python -u scripts/prof_render_mesh.py 2>&1 | grep "asset" | sed "s/^/$v /" >> gpurun_out/r5_d_render.log || exit 1
done
cat gpurun_out/r5_d_render.log
timeout -k 10 900 python -u -m pytest -v --timeout 600 --timeout-method thread -m gpu -s \
  tests/test_render_gpu.py tests/test_engine_gpu.py > gpurun_out/r5_d_tests.log 2>&1 || { echo "tests rc=$?"; }
grep -E "PASS|FAIL|mesh pixels|Newton|passed|failed" gpurun_out/r5_d_tests.log | tail -30
