#!/bin/bash
# round 4 box g: f16x3 GEMM SQ counters; stride-1 128-channel convs on the f16x3 implicit GEMM vs
# the fused Winograd (bench A/B); the default bench under rocprofv3 (timed window); f16x3 GEMM
# HBM-traffic PMC passes
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
RMBX_SQ_FORM=f16x3 bash scripts/gpurun/gemm_sq.sh r4g_h3 || exit 1
timeout -k 10 400 python -u bench.py --no_cpu_baseline --no_bf16_secondary > gpurun_out/r4_g_bench_default.json.log 2> gpurun_out/r4_g_bench_default.err || exit 1
RMBX_S1_GEMM=128 timeout -k 10 400 python -u bench.py --no_cpu_baseline --no_bf16_secondary > gpurun_out/r4_g_bench_s1gemm128.json.log 2> gpurun_out/r4_g_bench_s1gemm128.err || exit 1
bash scripts/gpurun/r3_benchprof.sh r4g || exit 1
bash scripts/gpurun/gemm_pmc.sh r4g_h3 || exit 1
