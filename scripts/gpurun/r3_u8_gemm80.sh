#!/bin/bash
# u8 stem: tests, timing of both layouts; GEMM persistent variant A/B; ACT production parity; bench
set -o pipefail
true
timeout -k 10 120 python -u scripts/prof_stem_u8.py > gpurun_out/r3_u8_stem_prof.log 2>&1 || exit 1
RMBX_STEM_U8_LAYOUT=10 timeout -k 10 120 python -u scripts/prof_stem_u8.py >> gpurun_out/r3_u8_stem_prof.log 2>&1 || exit 1
for v in 16 80; do
  echo "== RMBX_GEMM_VAR=$v" >> gpurun_out/r3_gemm_persist.log
  RMBX_GEMM_VAR=$v timeout -k 10 200 python3 -u scripts/prof_gemm.py >> gpurun_out/r3_gemm_persist.log 2>&1 || exit 1
done
timeout -k 10 400 python -u -m pytest -x -v -s --timeout 380 --timeout-method thread tests/test_act_full_gpu.py > gpurun_out/r3_u8_act_full.log 2>&1 || exit 1
timeout -k 10 300 python -u bench.py > gpurun_out/r3_bench_u8.json.log 2>&1 || exit 1
