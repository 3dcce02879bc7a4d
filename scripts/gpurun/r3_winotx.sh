#!/bin/bash
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_wino_x6_gpu.py > gpurun_out/winotx_tests.log 2>&1 || exit 1
for v in 0 1; do
  echo "== RMBX_WINOTX_VEC=$v" >> gpurun_out/prof_winotx.log
  RMBX_WINOTX_VEC=$v timeout -k 10 300 python3 -u scripts/prof_wino_x6.py >> gpurun_out/prof_winotx.log 2>&1 || exit 1
done
