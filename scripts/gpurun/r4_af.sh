#!/bin/bash
# renderer register targets: 4 / 5 (default) / 6 waves per SIMD, one process per library, one box;
# then the render tests on the default
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
for v in render4 "" render6 render4 "" render6; do
  RMBX_LIB_VARIANT=$v timeout -k 10 200 python -u scripts/prof_render_u8.py >> gpurun_out/r4_af_render_ab.log 2>&1 || exit 1
done
timeout -k 10 400 python -u -m pytest -v --timeout 200 --timeout-method thread -m gpu tests/test_render_gpu.py tests/test_multicam_gpu.py > gpurun_out/r4_af_render_tests.log 2>&1 || exit 1
