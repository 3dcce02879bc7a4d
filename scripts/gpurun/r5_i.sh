#!/bin/bash
# render: determinism, oracle parity, per-camera time + kernel split
set -o pipefail
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u scripts/diag_render_batch.py > gpurun_out/r5_i_batch.log 2>&1 || { echo "diag rc=$?"; tail -20 gpurun_out/r5_i_batch.log; exit 1; }
cat gpurun_out/r5_i_batch.log | grep -v amdgpu.ids
timeout -k 10 400 python -u -m pytest -v -s --timeout 300 --timeout-method thread -m gpu tests/test_render_gpu.py tests/test_shard_gpu.py \
  > gpurun_out/r5_i_tests.log 2>&1 || { echo "tests rc=$?"; grep -E "PASS|FAIL|Error|assert" gpurun_out/r5_i_tests.log | tail -20; exit 1; }
grep -E "PASS|FAIL|mesh pixels|passed|failed" gpurun_out/r5_i_tests.log | tail -14
RENDER_ONLY_ASSET=1 RENDER_ALL_CAMS=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r5_i_prof -o r5i --output-format csv -- \
  python3 -u scripts/prof_render_mesh.py > gpurun_out/r5_i_render.log 2>&1 || { echo "prof rc=$?"; tail -20 gpurun_out/r5_i_render.log; exit 1; }
grep "ms per" gpurun_out/r5_i_render.log
grep -i "raster\|render_kernel" gpurun_out/r5_i_prof/r5i_kernel_stats.csv | cut -d, -f1-7
