#!/bin/bash
# u8 stem: horizontal-pool neighbours by DPP wave shifts vs LDS permutes -- tests with DPP on, timing A/B
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
RMBX_STEM_U8_DPP=1 timeout -k 10 300 python -u -m pytest -x -v --timeout 250 --timeout-method thread tests/test_nn_gpu.py -k "stem_conv_maxpool_u8" > gpurun_out/r3_stem_dpp_tests.log 2>&1 || exit 1
for d in 0 1 0 1; do
  RMBX_STEM_U8_DPP=$d timeout -k 10 120 python -u scripts/prof_stem_u8.py >> gpurun_out/r3_stem_dpp_prof.log 2>&1 || exit 1
done
